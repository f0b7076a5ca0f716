#!/bin/bash
# rocprofv3 kernel stats of the C4 EDSR line: in-tree library vs build/alt/libsrmi_prev.so
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
cat > /tmp/edsr_only.py <<'PY'
import sys, torch
sys.path[:0] = [sys.argv[1] + '/super-resolution-climate_amd', sys.argv[1]]
import bench
d = torch.device('cuda', 0); torch.cuda.set_device(d)
print(bench.edsr_bench(d, 64, 5, 2)['value'])
PY
for v in new old; do
  if [ $v = old ]; then [ -f "$R/alt/libsrmi_prev.so" ] || continue; export SRMI_LIB=$R/alt/libsrmi_prev.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pe_$v -o e -- python3 /tmp/edsr_only.py $R > $R/gpurun_out/pe_$v.log 2>&1 || exit 1
  echo "== $v $(grep -v Warn $R/gpurun_out/pe_$v.log | tail -1)"
  python3 - $R/gpurun_out/pe_$v/e_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms {float(r["AverageNs"])/1000:9.2f} us x{r["Calls"]:>5} {r["Name"][:60]}')
PY
done
