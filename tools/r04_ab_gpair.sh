#!/bin/bash
# Round 4: GPU parity of the pair gradient stream (model + kernel tests), then an
# interleaved bench A/B (pair vs --fp32-gstream, and the engine stagger).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 200 \
  --timeout-method thread > $O/gpair_tests.log 2>&1 || { tail -40 $O/gpair_tests.log; exit 1; }
tail -2 $O/gpair_tests.log
bash tools/r04_stagger.sh "$@"
