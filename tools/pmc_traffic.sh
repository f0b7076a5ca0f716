#!/bin/bash
# HBM traffic per launch of the roofline kernels: one rocprofv3 --pmc pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel
# trace only, then tools/pmc_parse.py -> gpurun_out/pmc_traffic.json
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 $R/tools/roofline_driver.py > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 $R/tools/pmc_parse.py $OUT $R/gpurun_out/pmc_traffic.json
