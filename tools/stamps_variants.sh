#!/bin/bash
# conv1 / conv2 phase stamps (tools/train_stamps.py) of several diagnostic builds in one
# call, each under its own limit:  bash tools/stamps_variants.sh name1 name2 ...
# (alt/libsrmi_<name>.so, built with make stamps STAMPOUT=...)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
for v in "$@"; do
  SRMI_LIB=$R/alt/libsrmi_$v.so timeout -k 10 200 python3 -u tools/train_stamps.py > $O/ts_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "== $v"; sed -n 2,6p $O/ts_$v.log
done
