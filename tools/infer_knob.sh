#!/bin/bash
# C5 inference line under environment knob settings: bash tools/infer_knob.sh "ENV1" "ENV2" ... ("-" = none)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=""
  env $cfg timeout -k 10 300 python -c "
import sys, torch; sys.path[:0] = ['super-resolution-climate_amd', '.']
import bench
d = torch.device('cuda', 0); torch.cuda.set_device(d)
r = bench.inference_bench(d, 4096, 5)
print('[$cfg]', r['value'], r['ms_per_region'])
" 2>&1 | grep "^\[" || exit 1
done
