#!/bin/bash
# Interleaved inference (C5) + EDSR (C4) A/B over libraries (in-tree = "-").
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset SRMI_LIB; else export SRMI_LIB=$R/$lib; fi
    timeout -k 10 200 python bench.py --no-train ${INFARGS} > gpurun_out/inf.json 2>>gpurun_out/inf.err || exit 5
    python -c "
import json; d=json.loads(open('gpurun_out/inf.json').read().strip().splitlines()[-1])
i=d['inference']; e=d['edsr_x8']
print('[$lib]', 'C5', i and (i['value'], i['ms_per_region'], i['mfma_frac']), 'C4', e and (e['value'], e['ms_per_step']))" | tee -a gpurun_out/inf.log
  done
done
unset SRMI_LIB
echo inf done
