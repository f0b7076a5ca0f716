#!/bin/bash
# Round 4: the one-launch inference RCAB.  Inference parity tests, then an interleaved
# C5 A/B on this box: one launch per RCAB (default) vs three (--no-rcab-infer).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_inference.py -x -q -m gpu --timeout 200 --timeout-method thread \
  > $O/infer_tests.log 2>&1 || { tail -40 $O/infer_tests.log; exit 1; }
tail -1 $O/infer_tests.log
for rep in 1 2; do
  for flag in "" "--no-rcab-infer"; do
    timeout -k 10 200 python bench.py --no-train --no-edsr --infer-iters 10 $flag > $O/abi.json 2>> $O/abi.err || exit 2
    python -c "
import json; d=json.loads(open('$O/abi.json').read().strip().splitlines()[-1])['inference']
print('one-launch' if d['rcab_one_launch'] else 'three', d['value'], d['ms_per_region'])" | tee -a $O/ab_infer.log
  done
done
echo done
