#!/bin/bash
# rocprofv3 kernel trace of the bench training leg for several variants (name:lib:flags),
# one per-step kernel table each (tools/step_timeline.py) -> gpurun_out/tl_<name>.txt
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  IFS=: read -r name lib flags <<< "$v"
  SRMI_LIB=${lib:+$R/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$name -o t -- \
    python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-inference --no-edsr --no-dp-probe $flags \
    > $O/prof_$name.log 2>&1 || { echo "prof $name failed"; exit 1; }
  python3 $R/tools/step_timeline.py $O/prof_$name/t_kernel_trace.csv 1 > $O/tl_$name.txt 2>&1 || true
  head -20 $O/tl_$name.txt
  gzip -f $O/prof_$name/t_kernel_trace.csv; rm -f $O/prof_$name/t_agent_info.csv
done
echo done
