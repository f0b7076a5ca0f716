#!/bin/bash
# Interleaved bench A/B of library builds and engine flags on ONE box (training leg only):
#   bash tools/ab_var.sh "main::" "redl:alt/libsrmi_redl.so:" "pass::--ca-pass"
# each variant = name:library (empty = in-tree):extra bench flags[:VAR=x,VAR2=y env]
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
REPS=${REPS:-2}
for rep in $(seq $REPS); do
  for v in "$@"; do
    IFS=: read -r name lib flags envs <<< "$v"
    env ${envs//,/ } SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python bench.py --no-cpu-baseline --no-inference --no-edsr --no-dp-probe \
      --steps 20 --warmup 3 $flags > $O/abv.json 2>> $O/abv.err || { echo "variant $name failed"; exit 2; }
    python -c "
import json; d=json.loads(open('$O/abv.json').read().strip().splitlines()[-1])
print('$name', d['value'], d['ms_per_step'], d['step_times']['median_ms'], 'F1', d['roofline']['avg_launch_ms'], d['roofline']['concurrent']['per_stream_ms'], 'F2', d['roofline_f2']['avg_launch_ms'], d['roofline_f2']['concurrent']['per_stream_ms'])" | tee -a $O/ab_var.log
  done
done
echo done
