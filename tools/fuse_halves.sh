#!/bin/bash
# In-step durations of the two fused RCAB-backward launches (bench.py's probe) with the
# product library and the diagnostic builds that drop one half (alt/libsrmi_diag1.so:
# no filter gradient, alt/libsrmi_diag2.so: no dgrad conv), at micro 1 and 2.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for m in 1 2; do
  for lib in "" alt/libsrmi_diag1.so alt/libsrmi_diag2.so; do
    SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --steps 5 --warmup 2 --micro $m > gpurun_out/fh.log 2>>gpurun_out/fh.err || exit 2
    python -c "
import json,sys; d=json.loads(open('gpurun_out/fh.log').read().strip().splitlines()[-1])
print('micro $m lib ${lib:-main}', d['value'], 'F1', d['roofline']['per_stream_ms'], 'F2', d['roofline_f2']['per_stream_ms'])" | tee -a gpurun_out/fuse_halves.log
  done
done
