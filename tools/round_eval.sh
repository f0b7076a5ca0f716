#!/bin/bash
# Full GPU evaluation: all -m gpu tests, smoke(), then the default bench command under
# rocprofv3 kernel-trace/stats (the summary that backs bench.py's roofline numbers).
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench -- python3 $R/bench.py > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; exit 3; }
python3 $R/tools/prof_summary.py $R/gpurun_out/prof_$TAG/bench_kernel_trace.csv $R/gpurun_out/bench_$TAG.log $R/gpurun_out/roofline_agreement_$TAG.json > /dev/null || exit 4
echo eval done
