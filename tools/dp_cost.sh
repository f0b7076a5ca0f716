#!/bin/bash
# DP machinery cost at one rank (bench --force-dp: RCCL group, reducer, bucketed all-reduce) vs the N=1 path
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
for args in "--micro 2" "--micro 2 --force-dp" "--micro 1" "--micro 1 --force-dp"; do
  v=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 4 $args 2>>gpurun_out/dp_cost.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['host_enqueue_idle_ms_per_step'])") || exit 1
  echo "$args: $v" | tee -a gpurun_out/dp_cost.log
done
done
