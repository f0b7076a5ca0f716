#!/bin/bash
# LDS bank conflicts / LDS issue stalls / MFMA busy of the 64-channel conv kernels (one --pmc pass each)
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_lds; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/conv_only.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-28:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
