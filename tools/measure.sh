#!/bin/bash
# Measurement of the in-tree library: every -m gpu test, smoke(), the default
# bench line, a kernel trace of a short bench (stats + per-step timeline + roofline
# agreement), then the PMC passes (tools/pmc_step.sh).  Each GPU step has its own limit.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
tail -1 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o t -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-edsr --no-dp-probe > $O/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
python3 $R/tools/prof_summary.py $O/prof_bench/t_kernel_trace.csv $O/prof_bench.log $O/prof_summary.json > /dev/null || true
python3 $R/tools/step_timeline.py $O/prof_bench/t_kernel_trace.csv 2 > $O/step_timeline.txt 2>&1 || true
[ "${1:-}" = "nopmc" ] && { echo measure done; exit 0; }
bash $R/tools/pmc_step.sh || exit 5
echo measure done
