#!/bin/bash
# rocprofv3 kernel-trace stats of the C5 inference leg (bench.py --no-train)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_infer -o t -- \
  python3 $R/bench.py --no-train --no-edsr --infer-iters 3 "$@" > $O/prof_infer.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_infer.log; exit 1; }
head -30 $O/prof_infer/t_kernel_stats.csv
gzip -f $O/prof_infer/t_kernel_trace.csv; rm -f $O/prof_infer/t_agent_info.csv
