#!/bin/bash
# Fabric traffic per launch of the C5 inference kernels (one --pmc pass per counter)
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_inf; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 $R/bench.py --no-train --no-edsr --infer-iters 1 "$@" > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail $OUT/$c.log; exit 1; }
done
python3 $R/tools/pmc_parse.py $OUT $R/gpurun_out/pmc_infer.json
python3 -c "
import json; d=json.load(open('$R/gpurun_out/pmc_infer.json'))
for k,v in d.items():
  if isinstance(v,dict) and 'hbm_bytes_per_launch' in v: print(round(v['hbm_bytes_per_launch']/1e6,2),'MB', round(v['fetch_bytes']/1e6,2), round(v['write_bytes']/1e6,2), k[:60])"
