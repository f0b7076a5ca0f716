#!/bin/bash
# A/B: bench.py (training only) with the in-tree library and an alternative build (SRMI_LIB), interleaved.
#   bash tools/ab_bench.sh [ALT_LIB] [extra bench args]
R=${GRAFT_REPO_ROOT:-/root/repo}
ALT=${1:-$R/build/alt/libsrmi_prev.so}
shift
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/ab_new_*.log gpurun_out/ab_old_*.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 "$@" > gpurun_out/ab_new_$i.log 2>&1 || exit 1
  SRMI_LIB=$ALT timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 "$@" > gpurun_out/ab_old_$i.log 2>&1 || exit 2
done
grep -o '"value": [0-9.]*' gpurun_out/ab_*.log
