#!/bin/bash
# kbench of the in-tree library and every alt/libsrmi_*.so variant
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/kbench.py > gpurun_out/kbv_intree.log 2>&1 || exit 5
for f in alt/libsrmi_*.so; do
  b=$(basename $f .so)
  SRMI_LIB=$R/$f timeout -k 10 120 python tools/kbench.py > gpurun_out/kbv_$b.log 2>&1 || exit 6
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/kbv_*.log")):
    s = open(f).read(); d = json.loads(s[s.find("{"):])
    print(f, {k: v.get("us") for k, v in d.items()})
PY
