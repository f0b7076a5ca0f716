#!/bin/bash
# bench.py training leg: micro-batch count x per-engine CU budget, interleaved repetitions
#   bash tools/ab_budget.sh "2:128" "2:192" "2:256" "1:0"
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
for mb in "$@"; do
  m=${mb%:*}; b=${mb#*:}
  v=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 4 --micro $m --cu-budget $b 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['host_enqueue_idle_ms_per_step'])") || exit 1
  echo "micro=$m budget=$b $v" | tee -a gpurun_out/ab_budget.log
done
done
