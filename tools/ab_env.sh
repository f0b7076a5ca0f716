#!/bin/bash
# A/B of engine environment knobs on the training bench (no CPU baseline, no inference).
#   bash tools/ab_env.sh "ARGS" "ENV1" "ENV2" ...     (ENV = space-separated K=V, or "-" for none)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
ARGS=$1; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  [ "$cfg" = "-" ] && cfg=""
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 10 --warmup 3 $ARGS > gpurun_out/ab_$i.log 2>&1 || { echo "run $i ($cfg) failed"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  v=$(grep -o '"value": [0-9.]*' gpurun_out/ab_$i.log | head -1)
  l=$(grep -o '"loss": [0-9.]*' gpurun_out/ab_$i.log | head -1)
  l="$l $(grep -o '"host_enqueue_ms_per_step": [0-9.]*' gpurun_out/ab_$i.log | head -1)"
  echo "$i [$cfg] $v $l" | tee -a gpurun_out/ab_summary.txt
done
