#!/bin/bash
# GPU iteration: the -m gpu suite, then bench.py (training only) with the in-tree
# library vs ALT (default build/alt/libsrmi_prev.so), interleaved, at micro 1 and 2.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
ALT=${1:-$R/alt/libsrmi_prev.so}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
val() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" "$1"; }
for i in 1 2; do
  for m in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 --micro $m > gpurun_out/abn_$m.log 2>gpurun_out/ab.err || exit 2
    SRMI_LIB=$ALT timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 --micro $m > gpurun_out/abo_$m.log 2>>gpurun_out/ab.err || exit 3
    echo "rep $i micro $m new $(val gpurun_out/abn_$m.log) old $(val gpurun_out/abo_$m.log)" | tee -a gpurun_out/ab_micro12.log
  done
done
