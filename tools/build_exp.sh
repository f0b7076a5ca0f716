#!/bin/bash
# Diagnostic wgrad48 builds (-DSRMI_WGRAD_EXP=N, see wgrad3x3.hip) -> build/alt/libsrmi_eN.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for n in "$@"; do
  make -C "$R" -j8 OBJDIR=build/exp_$n OUT=build/alt/libsrmi_e$n.so EXTRA="-DSRMI_WGRAD_EXP=$n" > /dev/null
done
ls -la "$R"/build/alt/
