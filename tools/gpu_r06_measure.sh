#!/bin/bash
# round 6 measurement pass on the in-tree library: the default bench line, a kernel
# trace of a short bench (in-step averages + per-step timeline), and the whole-step
# PMC traffic (tools/pmc_step_total.sh).  Each GPU step under its own time limit.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
tail -1 $O/bench.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o t -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-edsr --no-dp-probe > $O/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
python3 $R/tools/prof_summary.py $O/prof_bench/t_kernel_trace.csv $O/prof_bench.log $O/prof_summary.json > /dev/null || true
python3 $R/tools/step_timeline.py $O/prof_bench/t_kernel_trace.csv 2 > $O/step_timeline.txt 2>&1 || true
head -14 $O/step_timeline.txt
[ -n "${NOPMC:-}" ] && exit 0
bash $R/tools/pmc_step_total.sh || exit 5
