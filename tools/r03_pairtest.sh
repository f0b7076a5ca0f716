#!/bin/bash
# kernel tests (in-tree) + model / full-size tests against an alternative library ($1),
# then the interleaved A/B of the remaining args (tools/r03_ab.sh)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
ALT=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_kern.log 2>&1 || { tail -30 gpurun_out/t_kern.log; exit 1; }
tail -1 gpurun_out/t_kern.log
SRMI_LIB=$R/$ALT timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_alt.log 2>&1 || { tail -30 gpurun_out/t_alt.log; exit 2; }
tail -1 gpurun_out/t_alt.log
bash tools/r03_ab.sh "$@" || exit 5
