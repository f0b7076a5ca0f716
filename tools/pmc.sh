#!/bin/bash
# PMC passes over tools/kbench.py (one rocprofv3 --pmc pass per counter group; kernel-trace only).
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $line --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/kbench.py --iters 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU
FETCH_SIZE
WRITE_SIZE
LIST
echo pmc done
