#!/bin/bash
# Round 5: interleaved C2 A/B of the training-step variants (CA forward in conv2's
# prologue / its own scale launch / the CA pass; co-halves vs whole-co filter gradients;
# the CA fold; a double-buffered co-halves build), then the model / inference /
# full-size GPU tests (all reported, not stopping at the first failure).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O; rm -f $O/ab_var.log
REPS=${REPS:-2} bash tools/ab_var.sh "default::" "fullco::--wgrad-full-co" "launch::--ca-scale-launch" \
  "pass::--ca-pass" "fold::--ca-fold" "halfnb2:alt/libsrmi_halfnb2.so:" || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_model.py \
  tests/test_gpu_inference.py tests/test_gpu_fullsize.py > $O/t2.log 2>&1
grep -E "PASSED|FAILED|ERROR" $O/t2.log | sed 's/ *\[ *[0-9]*%\]//' | tail -60
