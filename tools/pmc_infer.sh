#!/bin/bash
# Fabric traffic per launch of the C5 inference kernels (one --pmc pass per counter),
# then the MFMA busy cycles of the same run; the summary records its configuration
# (region side, engine flags) so that bench.py quotes it only for the same one.
#   bash tools/pmc_infer.sh [--infer-region S] [--no-rcab-infer]
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_inf; mkdir -p $OUT
SIDE=4096; FLAGS=0
args=("$@"); for ((i=0; i<${#args[@]}; i++)); do
  [ "${args[i]}" = "--infer-region" ] && SIDE=${args[i+1]}
  [ "${args[i]}" = "--no-rcab-infer" ] && FLAGS=2
done
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 $R/bench.py --no-train --no-edsr --infer-iters 1 "$@" > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail $OUT/$c.log; exit 1; }
done
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d $OUT/MFMA -o run -- python3 $R/bench.py --no-train --no-edsr --infer-iters 1 "$@" > $OUT/MFMA.log 2>&1 || { echo "pmc mfma failed"; exit 2; }
python3 $R/tools/pmc_parse.py $OUT $R/gpurun_out/pmc_infer.json > /dev/null
python3 $R/tools/pmc_mfma_parse.py $OUT/MFMA $R/gpurun_out/pmc_infer_mfma.json > /dev/null
python3 -c "
import json
for p in ('$R/gpurun_out/pmc_infer_mfma.json', '$R/gpurun_out/pmc_infer.json'):
  d=json.load(open(p))
  d['config'] = {'infer_region': $SIDE, 'flags': $FLAGS, 'command': 'bench.py --no-train --no-edsr --infer-iters 1 $*'}
  json.dump(d, open(p, 'w'), indent=1)
for k,v in d.items():
  if isinstance(v,dict) and 'hbm_bytes_per_launch' in v: print(round(v['hbm_bytes_per_launch']/1e6,2),'MB', round(v['fetch_bytes']/1e6,2), round(v['write_bytes']/1e6,2), k[:60])"
echo pmc_infer done
