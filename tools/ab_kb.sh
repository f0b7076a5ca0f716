#!/bin/bash
# kbench (isolated kernels) + bench (training, inference) for the in-tree library and
# alternative builds (SRMI_LIB), interleaved:  bash tools/ab_kb.sh alt/libX.so ...
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for lib in "" "$@"; do
  echo "== kbench ${lib:-main}" >> gpurun_out/ab_kb.log
  SRMI_LIB=${lib:+$R/$lib} timeout -k 10 120 python tools/kbench.py --iters 50 > gpurun_out/kb.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/kb.json')); print(' '.join(f'{k}={v[\"us\"]}' for k,v in d.items()))" >> gpurun_out/ab_kb.log
done
for rep in 1 2; do
  for lib in "" "$@"; do
    SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python bench.py --no-cpu-baseline --no-edsr --steps 20 --warmup 3 > gpurun_out/abk.log 2>>gpurun_out/abk.err || exit 2
    python -c "
import json; d=json.loads(open('gpurun_out/abk.log').read().strip().splitlines()[-1])
print('${lib:-main}', d['value'], d['ms_per_step'], 'F1', d['roofline']['avg_launch_ms'], d['roofline']['concurrent']['per_stream_ms'], 'F2', d['roofline_f2']['avg_launch_ms'], d['roofline_f2']['concurrent']['per_stream_ms'], 'inf', d['inference']['value'])" >> gpurun_out/ab_kb.log
  done
done
cat gpurun_out/ab_kb.log
