#!/bin/bash
# Power / clock while the training bench runs (read-only amd-smi queries).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
O=gpurun_out/power.txt
: > $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-edsr --no-dp-probe --steps 600 --warmup 3 > gpurun_out/power_bench.json 2> gpurun_out/power_bench.err &
BP=$!
for i in $(seq 120); do grep -q "warm-up done" gpurun_out/power_bench.err 2>/dev/null && break; sleep 1; done
sleep 2
for i in 1 2 3 4 5; do
  echo "== sample $i $(date +%s.%N)" >> $O
  timeout -k 5 20 amd-smi metric --power --clock >> $O 2>&1
  sleep 1
done
wait $BP
echo power done
