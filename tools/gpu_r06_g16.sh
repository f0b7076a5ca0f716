#!/bin/bash
# round 6: the bf16 in-group gradient stream -- the GPU tests that cover the backward,
# then an interleaved C2 A/B against the previous library (alt/libsrmi_base.so)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
SRMI_PARITY_REPORT=$O/c2_parity_g16.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06_g16_tests.log 2>&1 || { tail -40 $O/r06_g16_tests.log; exit 1; }
tail -2 $O/r06_g16_tests.log
REPS=3 bash tools/ab_var.sh "g16::" "base:alt/libsrmi_base.so:" || exit 2
