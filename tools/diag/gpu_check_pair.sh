#!/bin/bash
# Round 5: the byte-permute pair codec -- every -m gpu test, then C5 / C2 A/Bs against the
# previous (ldexp) codec (alt/libsrmi_base.so) and the integer-lo8 variant (alt/libsrmi_pint.so)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
rm -f $O/ab_infer_var.log $O/ab_var.log
REPS=2 bash tools/ab_infer_var.sh "perm::" "base:alt/libsrmi_base.so:" "pint:alt/libsrmi_pint.so:" || exit 3
REPS=2 bash tools/ab_var.sh "perm::" "base:alt/libsrmi_base.so:" "pint:alt/libsrmi_pint.so:" || exit 4
