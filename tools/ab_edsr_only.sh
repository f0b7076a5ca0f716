#!/bin/bash
# C4 EDSR x8 fp32 line only (bench.edsr_bench): in-tree library vs alternative builds, interleaved
#   bash tools/ab_edsr_only.sh alt/libA.so alt/libB.so
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
cat > /tmp/edsr_only.py <<'PY'
import sys, torch
sys.path[:0] = [sys.argv[1] + '/super-resolution-climate_amd', sys.argv[1]]
import bench
d = torch.device('cuda', 0); torch.cuda.set_device(d)
r = bench.edsr_bench(d, 64, 6, 2)
print(r['value'], r['ms_per_step'])
PY
for rep in 1 2; do
  for lib in "" "$@"; do
    v=$(SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python /tmp/edsr_only.py $R 2>>gpurun_out/ab_edsr.err | tail -1) || exit 1
    echo "${lib:-main}: edsr $v" | tee -a gpurun_out/ab_edsr.log
  done
done
