#!/bin/bash
# rocprofv3 kernel trace of the C5 inference line (bench.inference_bench)
R=${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
cat > /tmp/infer_only.py <<'PY'
import sys, torch
sys.path[:0] = [sys.argv[1] + '/super-resolution-climate_amd', sys.argv[1]]
import bench
d = torch.device('cuda', 0); torch.cuda.set_device(d)
r = bench.inference_bench(d, 4096, 5)
print(r['value'], r['ms_per_region'])
PY
timeout -k 10 300 python3 /tmp/infer_only.py $R > $R/gpurun_out/infer_plain.log 2>&1 || exit 1
tail -1 $R/gpurun_out/infer_plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pinf -o i -- python3 /tmp/infer_only.py $R > $R/gpurun_out/pinf.log 2>&1 || exit 2
python3 - $R/gpurun_out/pinf/i_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms {float(r["AverageNs"])/1000:9.2f} us x{r["Calls"]:>5} {r["Name"][:60]}')
PY
