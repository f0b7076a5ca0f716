#!/bin/bash
# C4 EDSR x8 fp32 line (bench.edsr_bench) and the C2 training line: in-tree library vs ALT, interleaved
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
ALT=${1:-$R/alt/libsrmi_prev.so}
cat > /tmp/edsr_only.py <<'PY'
import sys, torch
sys.path[:0] = [sys.argv[1] + '/super-resolution-climate_amd', sys.argv[1]]
import bench
d = torch.device('cuda', 0); torch.cuda.set_device(d)
r = bench.edsr_bench(d, 64, 6, 2)
print(r['value'], r['ms_per_step'])
PY
for rep in 1 2; do
  for lib in "" "$ALT"; do
    v=$(SRMI_LIB=$lib timeout -k 10 200 python /tmp/edsr_only.py $R 2>>gpurun_out/ab_edsr.err | tail -1) || exit 1
    t=$(SRMI_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 2>>gpurun_out/ab_edsr.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'])") || exit 2
    echo "${lib:-main}: edsr $v  c2 $t" | tee -a gpurun_out/ab_edsr.log
  done
done
