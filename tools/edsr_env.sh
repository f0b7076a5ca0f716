#!/bin/bash
# C4 EDSR line under environment knob settings ("-" = none)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
cat > /tmp/edsr_only.py <<'PY'
import sys, torch
sys.path[:0] = [sys.argv[1] + '/super-resolution-climate_amd', sys.argv[1]]
import bench
d = torch.device('cuda', 0); torch.cuda.set_device(d)
print(bench.edsr_bench(d, 64, 10, 3)['value'])
PY
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=""
  echo "[$cfg] $(env $cfg timeout -k 10 200 python /tmp/edsr_only.py $R 2>/dev/null | tail -1)"
done
