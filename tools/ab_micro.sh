#!/bin/bash
# bench.py training leg at several micro-batch counts (interleaved repetitions)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
for m in "$@"; do
  v=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 4 --micro $m 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])") || exit 1
  echo "micro=$m $v" | tee -a gpurun_out/ab_micro.log
done
done
