#!/bin/bash
# Round 5: the byte-permute pair codec in training -- conv2 stamps (new vs previous codec), C2 A/B REPS=3
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O; rm -f $O/pair2.log
for v in perm base; do
  lib=$R/super-resolution-climate_amd/srmi/libsrmi_stamps.so; [ $v != perm ] && lib=$R/alt/libsrmi_stamps_$v.so
  echo "== $v" >> $O/pair2.log
  SRMI_LIB=$lib timeout -k 10 200 python -u tools/train_stamps.py > $O/ts.log 2>&1 || { tail $O/ts.log; exit 2; }
  grep -v "scale:\|body start\|amdgpu" $O/ts.log >> $O/pair2.log
done
cat $O/pair2.log
rm -f $O/ab_var.log
REPS=3 bash tools/ab_var.sh "perm::" "base:alt/libsrmi_base.so:" || exit 4
