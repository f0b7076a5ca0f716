#!/bin/bash
# Round 5: the training CA forward inside conv2 -- its GPU tests, then the interleaved
# C2 A/B of the three forms (scale in conv2's prologue, scale launch, CA pass).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O; rm -f $O/ab_var.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_model.py \
  tests/test_gpu_inference.py tests/test_gpu_fullsize.py > $O/t2.log 2>&1
rc=$?; tail -40 $O/t2.log; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-2} bash tools/ab_var.sh "default::" "fullco::--wgrad-full-co" "launch::--ca-scale-launch" "pass::--ca-pass" "fold::--ca-fold" "halfnb2:alt/libsrmi_halfnb2.so:"
