#!/bin/bash
# tests (TESTS) -> A/B variants (args) -> stamps (STAMPS=1)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_kernels.py tests/test_gpu_model.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/iter_tests.log 2>&1; rc=$?
  echo "tests rc=$rc" >> gpurun_out/iter_tests.log; tail -3 gpurun_out/iter_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
bash tools/r03_ab.sh "$@" || exit 5
if [ "${STAMPS:-1}" = "1" ]; then
  EPIS=${EPIS:-0,1,4,7} RS=0 bash tools/stamps_run.sh || exit 6
fi
echo go done
