#!/bin/bash
# Round 4: calibrate torch.cuda._sleep, then A/B the engine stagger (engine 1 starts its
# forward / backward a fixed delay after engine 0).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 120 python -c "
import torch
torch.cuda.init(); s=torch.cuda.current_stream()
for c in (10000, 100000, 1000000):
    a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(c); a.record(); torch.cuda._sleep(c); b.record(); torch.cuda.synchronize()
    print('sleep', c, 'cycles', round(a.elapsed_time(b)*1000,2), 'us')
" | tee $O/stagger_cal.log || exit 1
REPS=${REPS:-2} bash tools/ab_var.sh "$@"
