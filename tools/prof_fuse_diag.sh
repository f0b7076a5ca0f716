#!/bin/bash
# kernel traces of the training step with the fused backward's conv part or wgrad part
# skipped (diagnostic builds alt/libsrmi_diag{1,2}.so): the duration of each part alone
R=${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
for d in 1 2; do
  SRMI_LIB=$R/alt/libsrmi_diag$d.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_diag$d -o t -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-inference --no-edsr --micro 1 > $R/gpurun_out/prof_diag$d.log 2>&1 || exit $d
done
echo done
