#!/bin/bash
# Interleaved bench A/B of variants "LIB|ARGS" (LIB empty = in-tree library), REPS rounds.
#   bash tools/r03_ab.sh "|" "alt/libsrmi_prev.so|" "|--stagger-us 12"
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
REPS=${REPS:-2}
STEPS=${STEPS:-20}
for rep in $(seq $REPS); do
  for v in "$@"; do
    lib=${v%%|*}; args=${v#*|}
    SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --no-dp-probe --steps $STEPS --warmup 3 $args > gpurun_out/ab.json 2>>gpurun_out/ab.err || exit 5
    python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print('[${lib:-new}|${args}]', d['value'], d['ms_per_step'], 'loss', repr(d['loss']), 'F1', d['roofline']['per_stream_ms'], 'F2', d['roofline_f2']['per_stream_ms'], 'conv', d['roofline_conv_fwd']['avg_launch_ms'])" | tee -a gpurun_out/ab.log
  done
done
echo ab done
