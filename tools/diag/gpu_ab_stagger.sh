#!/bin/bash
# Round 5: the staggered deferred epilogue -- model / inference tests, then the C5 and
# C2 interleaved A/Bs against the HEAD library (alt/libsrmi_base.so)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_inference.py > $O/t_stag.log 2>&1 || { tail -30 $O/t_stag.log; exit 1; }
tail -1 $O/t_stag.log
rm -f $O/ab_infer_var.log $O/ab_var.log
REPS=2 bash tools/ab_infer_var.sh "stag::" "base:alt/libsrmi_base.so:" "stag48:alt/libsrmi_stag48.so:" "nostag:alt/libsrmi_nostag.so:" || exit 2
REPS=2 bash tools/ab_var.sh "stag::" "base:alt/libsrmi_base.so:" "nostag:alt/libsrmi_nostag.so:" || exit 3
