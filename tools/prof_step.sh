#!/bin/bash
# rocprofv3 kernel trace of the training step (bench.py, training only) for the given bench args.
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-step}; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o t -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-inference --no-edsr "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 1
echo prof $TAG done
