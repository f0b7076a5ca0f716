#!/bin/bash
# DP machinery cost at one rank (bench --force-dp: RCCL group + bucketed all-reduce)
# against the N=1 path: the staged schedule (default: the all-reduce enqueued on the
# last engine's stream between backward stages) and --dp-reducer-stream (a reducer
# stream waiting on the engines' residual-group events).  Interleaved, one box.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out; O=gpurun_out/dp_cost.log; rm -f $O
for rep in 1 2; do
for args in "" "--force-dp" "--force-dp --dp-reducer-stream"; do
  v=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --no-dp-probe --steps 20 --warmup 4 $args 2>>gpurun_out/dp_cost.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['host_enqueue_idle_ms_per_step'])") || exit 1
  echo "micro 2 ${args:-plain}: tiles/s ms/step host_enqueue host_enqueue_idle = $v" | tee -a $O
done
done
