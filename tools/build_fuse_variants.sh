#!/bin/bash
# Diagnostic builds of the fused-backward CU split (SRMI_FUSE_WG2 / SRMI_FUSE_WG1 %) -> alt/libsrmi_fuse_A_B.so
R=${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p $R/alt
for v in "$@"; do
  a=${v%,*}; b=${v#*,}
  make -C "$R" -j8 OBJDIR=build/fuse_${a}_${b} OUT=alt/libsrmi_fuse_${a}_${b}.so EXTRA="-DSRMI_FUSE_WG2=$a -DSRMI_FUSE_WG1=$b" > /dev/null || exit 1
done
