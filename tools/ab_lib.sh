#!/bin/bash
# bench.py training leg, in-tree library vs alternative builds (SRMI_LIB), interleaved; F1/F2 probe times
#   bash tools/ab_lib.sh "1 2" alt/libA.so alt/libB.so
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
MICROS=$1; shift
for rep in 1 2; do
for m in $MICROS; do
  for lib in "" "$@"; do
    SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 3 --micro $m > gpurun_out/abl.log 2>>gpurun_out/abl.err || exit 2
    python -c "
import json; d=json.loads(open('gpurun_out/abl.log').read().strip().splitlines()[-1])
print('micro $m ${lib:-main}', d['value'], d['ms_per_step'], 'F1', d['roofline']['avg_launch_ms'], d['roofline']['concurrent']['per_stream_ms'], 'F2', d['roofline_f2']['avg_launch_ms'], d['roofline_f2']['concurrent']['per_stream_ms'])" | tee -a gpurun_out/ab_lib.log
  done
done
done
