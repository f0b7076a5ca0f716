#!/bin/bash
# Round 4: inference RCAB v2 builds -- parity (inference tests, C5 full region) per build, then C5 A/B
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
for v in v2 v2d v2dd; do
  SRMI_LIB=$R/alt/libsrmi_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_inference.py \
    tests/test_gpu_fullsize.py::test_c5_full_region_vs_fp32_oracle -x -q -m gpu --timeout 300 --timeout-method thread \
    > $O/infer_$v.log 2>&1 || { echo "$v tests failed"; tail -30 $O/infer_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/infer_$v.log)"
done
bash tools/ab_infer_var.sh "v1::" "v2:alt/libsrmi_v2.so:" "v2d:alt/libsrmi_v2d.so:" "v2dd:alt/libsrmi_v2dd.so:"
