#!/bin/bash
# PMC passes over the training step + in-step probes (tools/roofline_driver.py):
# FETCH_SIZE and WRITE_SIZE in separate passes (gfx950 slot limits), then the MFMA
# busy cycles; kernel traces of the same driver for the duration agreement.
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 $R/tools/roofline_driver.py > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/MFMA -o run -- python3 $R/tools/roofline_driver.py > $OUT/MFMA.log 2>&1 || { echo "pmc mfma failed"; exit 2; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/TRACE -o run -- python3 $R/tools/roofline_driver.py > $OUT/TRACE.log 2>&1 || { echo "trace failed"; exit 3; }
python3 $R/tools/pmc_parse.py $OUT $R/gpurun_out/pmc_traffic.json > /dev/null
python3 $R/tools/pmc_mfma_parse.py $OUT/MFMA $R/gpurun_out/pmc_mfma.json > /dev/null
echo pmc done
