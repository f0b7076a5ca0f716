#!/bin/bash
# GPU iteration: full GPU test suite, then kbench + interleaved bench A/B against build/alt/libsrmi_prev.so.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab_kb.sh
