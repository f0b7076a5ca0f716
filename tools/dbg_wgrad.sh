mkdir -p gpurun_out
for d in 0 1 2 4 5; do
  echo "=== dbg $d" >> gpurun_out/dbg.log
  SRMI_WGRAD_DBG=$d KBENCH_STAMPS=1 KBENCH_RS=3 timeout -k 10 120 python tools/kbench.py >> gpurun_out/dbg.log 2>&1 || exit 1
done
