#!/bin/bash
# Build libsrmi.so from git revision $1 (default HEAD) into build/alt/libsrmi_prev.so (for tools/ab_bench.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
T=$(mktemp -d)
git -C "$R" archive "$REV" Makefile include super-resolution-climate_amd/csrc | tar -x -C "$T"
mkdir -p "$R/build/alt"
make -C "$T" -j8 OUT="$R/build/alt/libsrmi_prev.so" > /dev/null
rm -rf "$T"
ls -la "$R/build/alt/libsrmi_prev.so"
