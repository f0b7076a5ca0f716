#!/bin/bash
# A/B of fused-backward CU splits: bench.py training leg per variant library and micro setting
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
for lib in alt/libsrmi_fuse_*.so; do
  for m in 1 2; do
    v=$(SRMI_LIB=$R/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 4 --micro $m 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$lib micro=$m $v" >> gpurun_out/ab_fuse.log
  done
done
done
