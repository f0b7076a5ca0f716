#!/bin/bash
# rocprofv3 kernel traces of the training step with and without the data-parallel
# machinery at one rank (--force-dp: live RCCL communicator, reducer, collectives).
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_nodp -o t -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-inference --no-edsr > $R/gpurun_out/prof_nodp.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_dp -o t -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-inference --no-edsr --force-dp > $R/gpurun_out/prof_dp.log 2>&1 || exit 2
echo prof done
