#!/bin/bash
# Round 5: the CA scale from conv1's border records -- stamps, model / inference / full-size
# tests, then C2 and C5 A/Bs against HEAD (alt/libsrmi_base.so)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_inference.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py > $O/t_scale.log 2>&1 || { tail -30 $O/t_scale.log; exit 2; }
tail -1 $O/t_scale.log
timeout -k 10 200 python -u tools/infer_stamps.py 221 > $O/infer_stamps.log 2>&1 || { tail $O/infer_stamps.log; exit 1; }
timeout -k 10 300 python -u tools/train_stamps.py > $O/train_stamps.log 2>&1 || { tail $O/train_stamps.log; exit 1; }
grep -E "ca_scale|scale|launch span|conv2 body|prologue|strip 0|span" $O/infer_stamps.log $O/train_stamps.log
rm -f $O/ab_infer_var.log $O/ab_var.log
REPS=2 bash tools/ab_var.sh "rec::" "base:alt/libsrmi_base.so:" || exit 3
REPS=2 bash tools/ab_infer_var.sh "rec::" "base:alt/libsrmi_base.so:" || exit 4
