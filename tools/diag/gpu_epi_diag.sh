#!/bin/bash
# TEMPORARY (round 5): where the CA residual epilogue's time goes -- phase stamps of the
# inference RCAB and the training convs with parts of the epilogue compiled out (wrong results)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O; rm -f $O/epi_diag.log
for v in 0 1 2 4 7; do
  lib=$R/super-resolution-climate_amd/srmi/libsrmi_stamps.so; [ $v != 0 ] && lib=$R/alt/libsrmi_stamps_ed$v.so
  echo "== SRMI_EPI_DIAG=$v" >> $O/epi_diag.log
  SRMI_LIB=$lib timeout -k 10 120 python -u tools/infer_stamps.py 221 > $O/is.log 2>&1 || { tail $O/is.log; exit 1; }
  grep -E "conv2 body|conv2 strip" $O/is.log >> $O/epi_diag.log
  SRMI_LIB=$lib timeout -k 10 200 python -u tools/train_stamps.py > $O/ts.log 2>&1 || { tail $O/ts.log; exit 2; }
  grep -A5 "conv2 CA_RESID_U" $O/ts.log | grep -E "CA_RESID_U|prologue|strip" >> $O/epi_diag.log
done
cat $O/epi_diag.log
