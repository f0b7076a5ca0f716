cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for i in 1 2; do
 for m in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-inference --steps 10 --warmup 3 --micro $m > gpurun_out/abm_${m}_$i.log 2>&1 || exit 1
 done
done
