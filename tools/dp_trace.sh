#!/bin/bash
# Kernel trace of the one-rank DP step (bench --force-dp, staged schedule) and its per-step timeline
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dp -o t -- python3 $R/bench.py --force-dp "$@" --steps 6 --warmup 2 --no-cpu-baseline --no-inference --no-edsr --no-dp-probe > $O/prof_dp.log 2>&1 || { echo "dp trace failed"; exit 1; }
python3 $R/tools/step_timeline.py $O/prof_dp/t_kernel_trace.csv 2 > $O/dp_timeline.txt 2>&1 || true
echo dp trace done
