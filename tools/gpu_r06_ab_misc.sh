rm -f gpurun_out/ab_var.log gpurun_out/ab_infer_var.log
SRMI_LIB=$GRAFT_REPO_ROOT/alt/libsrmi_split.so timeout -k 10 400 python -u -m pytest tests/test_gpu_inference.py tests/test_gpu_fullsize.py -k "c5 or infer or region" -x -q --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1; echo "split tests rc=$?"; tail -2 gpurun_out/split_tests.log
REPS=2 bash tools/ab_infer_var.sh "one::" "split:alt/libsrmi_split.so:" || exit 3
REPS=3 bash tools/ab_var.sh "main::" "wt0:alt/libsrmi_wt0.so:" "tf0:alt/libsrmi_tf0.so:"
