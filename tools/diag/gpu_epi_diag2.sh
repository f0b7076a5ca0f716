#!/bin/bash
# TEMPORARY (round 5): the integer lo8 pair codec -- stamps, then C5 / C2 A/B against HEAD
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O; rm -f $O/epi_diag2.log
for v in base pint px; do
  lib=$R/super-resolution-climate_amd/srmi/libsrmi_stamps.so; [ $v != base ] && lib=$R/alt/libsrmi_stamps_$v.so
  echo "== $v" >> $O/epi_diag2.log
  SRMI_LIB=$lib timeout -k 10 120 python -u tools/infer_stamps.py 221 > $O/is.log 2>&1 || { tail $O/is.log; exit 1; }
  grep -E "launch span|conv2 body|conv2 strip" $O/is.log >> $O/epi_diag2.log
  SRMI_LIB=$lib timeout -k 10 200 python -u tools/train_stamps.py > $O/ts.log 2>&1 || { tail $O/ts.log; exit 2; }
  grep -A5 "conv2 CA_RESID_U" $O/ts.log | grep -E "CA_RESID_U|prologue|strip" >> $O/epi_diag2.log
done
cat $O/epi_diag2.log
rm -f $O/ab_infer_var.log $O/ab_var.log
REPS=2 bash tools/ab_infer_var.sh "pint:alt/libsrmi_pint.so:" "base:alt/libsrmi_base.so:" "px:alt/libsrmi_px.so:" || exit 3
REPS=2 bash tools/ab_var.sh "pint:alt/libsrmi_pint.so:" "base:alt/libsrmi_base.so:" "px:alt/libsrmi_px.so:" || exit 4
