#!/bin/bash
# MFMA utilisation of the roofline kernels: one rocprofv3 --pmc pass (kernel trace
# only) over tools/roofline_driver.py with SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES
# and GRBM_GUI_ACTIVE, then tools/pmc_mfma_parse.py -> gpurun_out/pmc_mfma.json
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/MFMA -o run -- python3 $R/tools/roofline_driver.py > $OUT/MFMA.log 2>&1 || { echo "pmc mfma failed"; exit 1; }
python3 $R/tools/pmc_mfma_parse.py $OUT/MFMA $R/gpurun_out/pmc_mfma.json
