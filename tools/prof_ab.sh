#!/bin/bash
# rocprofv3 kernel stats of a short training bench: in-tree library vs build/alt/libsrmi_prev.so
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab_new -o b -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-inference --no-edsr > $R/gpurun_out/pab_new.log 2>&1 || exit 1
SRMI_LIB=$R/build/alt/libsrmi_prev.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab_old -o b -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-inference --no-edsr > $R/gpurun_out/pab_old.log 2>&1 || exit 2
for v in new old; do echo "== $v"; python3 - $R/gpurun_out/pab_$v/b_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("tail_", "head_", "slab_reduce")):
        print(f'{float(r["AverageNs"])/1000:9.2f} us  x{r["Calls"]:>5}  {n[:70]}')
PY
done
