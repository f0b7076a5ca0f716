R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_new.log 2>&1 || exit 5
SRMI_LIB=$R/build/alt/libsrmi_prev.so timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_old.log 2>&1 || exit 6
bash tools/ab_bench.sh
