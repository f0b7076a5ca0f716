#!/bin/bash
# Round 5: the in-group gradient stream as the pair -- every -m gpu test, then C2 A/B
# against the fp32 gradient stream (alt/libsrmi_base.so = the previous library)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
rm -f $O/ab_var.log
REPS=3 bash tools/ab_var.sh "gpair::" "base:alt/libsrmi_base.so:" || exit 3
