#!/bin/bash
# register / spill / LDS figures of every kernel of one HIP source (device code only):
#   bash tools/kstats.sh super-resolution-climate_amd/csrc/wgrad3x3.hip [EXTRA flags]
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; shift
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include "$@" --offload-device-only --no-gpu-bundle-output -c $SRC -o $T/k.co || exit 1
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | awk '/\.name:/{n=$2} /\.vgpr_count:/{v=$2} /\.vgpr_spill_count:/{vs=$2} /\.sgpr_spill_count:/{ss=$2} /\.group_segment_fixed_size:/{l=$2} /\.agpr_count:/{if(n!="") {} } /\.wavefront_size:/{print n, "vgpr", v, "vspill", vs, "sspill", ss}' | c++filt | sed 's/(srmi::[^)]*)//'
rm -rf $T
