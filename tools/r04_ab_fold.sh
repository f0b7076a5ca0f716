#!/bin/bash
# Round 4: the CA-backward fold.  GPU parity of the fold first (kernel + model + full-size
# + DP tests), then an interleaved bench A/B on this box: --ca-fold vs the default (materialised du).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -x -q -m gpu \
  --timeout 400 --timeout-method thread > $O/fold_tests.log 2>&1 || { tail -40 $O/fold_tests.log; exit 1; }
tail -2 $O/fold_tests.log
for rep in 1 2; do
  for flag in "--ca-fold" ""; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --no-dp-probe --steps 20 --warmup 3 $flag \
      > $O/abf.json 2>> $O/abf.err || exit 2
    python -c "
import json; d=json.loads(open('$O/abf.json').read().strip().splitlines()[-1])
print('fold' if d['ca_fold'] else 'nofold', d['value'], d['ms_per_step'], d['step_times']['median_ms'], 'F1', d['roofline']['per_stream_ms'], 'F2', d['roofline_f2']['per_stream_ms'])" | tee -a $O/ab_fold.log
  done
done
echo done
