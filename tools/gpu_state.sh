#!/bin/bash
# GPU check of the current tree: all -m gpu tests, bench with 1 and 2 micro-batches,
# then a kernel trace of a short training-only bench for the per-step timeline.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
for m in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --steps 10 --warmup 3 --micro $m > gpurun_out/bench_m$m.log 2>&1 || { echo "bench m$m failed"; exit 2; }
done
cd /tmp && export TMPDIR=/tmp
for m in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_m$m -o tr -- python3 $R/bench.py --no-cpu-baseline --no-inference --steps 3 --warmup 1 --micro $m > $R/gpurun_out/trace_m$m.log 2>&1 || { echo "trace m$m failed"; exit 3; }
  python3 $R/tools/step_timeline.py $(find $R/gpurun_out/trace_m$m -name '*kernel_trace.csv' | head -1) 2 > $R/gpurun_out/timeline_m$m.txt
done
echo state done
