#!/bin/bash
# One B=32 engine alone (half the C2 batch) on a 128-CU budget / the whole chip, vs the C2 step
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for args in "--batch 32 --micro 1 --cu-budget 128" "--batch 32 --micro 1 --cu-budget 0" "--batch 64 --micro 2" "--batch 64 --micro 1"; do
  v=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 $args 2>>gpurun_out/half.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$args: $v" | tee -a gpurun_out/half_engine.log
done
