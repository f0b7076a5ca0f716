#!/bin/bash
# Phase stamps (s_memtime) of the Cin=64 conv kernel per epilogue and of wgrad48,
# from the diagnostic build (make stamps -> libsrmi_stamps.so, built on the CPU side).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
KBENCH_STAMPS=1 KBENCH_EPI=${EPIS:-0,1,4,5} KBENCH_RS=${RS:-0,2} timeout -k 10 240 python3 -u tools/kbench.py > gpurun_out/stamps.log 2>&1 || exit 1
echo stamps done
