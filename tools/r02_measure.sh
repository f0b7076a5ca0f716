#!/bin/bash
# Round-2 measurement: the default bench line, a kernel trace of a short bench run
# (training + in-step rooflines), then the PMC passes (tools/pmc_step.sh).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o t -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-edsr > $O/prof_bench.log 2>&1 || { echo "prof failed"; exit 2; }
python3 $R/tools/prof_summary.py $O/prof_bench/t_kernel_trace.csv $O/prof_bench.log $O/prof_summary.json || true
[ "${1:-}" = "nopmc" ] && exit 0
bash $R/tools/pmc_step.sh
