#!/bin/bash
# Interleaved C5 inference A/B of library builds / flags on ONE box:
#   bash tools/ab_infer_var.sh "main::" "old:alt/libsrmi_old.so:" "m1:::SRMI_INFER_MICRO=1"
# each variant = name:library (empty = in-tree):extra bench flags[:VAR=x,VAR2=y env]
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
REPS=${REPS:-2}
for rep in $(seq $REPS); do
  for v in "$@"; do
    IFS=: read -r name lib flags envs <<< "$v"
    env ${envs//,/ } SRMI_LIB=${lib:+$R/$lib} timeout -k 10 200 python bench.py --no-train --no-edsr --infer-iters 10 $flags \
      > $O/abiv.json 2>> $O/abiv.err || { echo "variant $name failed"; exit 2; }
    python -c "
import json; d=json.loads(open('$O/abiv.json').read().strip().splitlines()[-1])['inference']
print('$name', d['value'], d['ms_per_region'], (d.get('roofline') or {}).get('frac'))" | tee -a $O/ab_infer_var.log
  done
done
echo done
