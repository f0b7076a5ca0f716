#!/bin/bash
# Build the working tree's libsrmi.so with extra compile-time switches into
# alt/libsrmi_<name>.so (for the interleaved A/Bs of tools/ab_lib.sh / ab_kb.sh):
#   bash tools/build_variant.sh nowt "-DSRMI_TRAIN_WT=0"   (switches: csrc/tuning.hpp)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$R/alt"
make -C "$R" -j8 OBJDIR="build/obj_$NAME" OUT="$R/alt/libsrmi_$NAME.so" EXTRA="$*" > /dev/null
ls -la "$R/alt/libsrmi_$NAME.so"
