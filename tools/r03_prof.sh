#!/bin/bash
# rocprofv3 kernel traces of a short training bench for each library given (in-tree = "-"),
# then the per-step timeline of each.
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset SRMI_LIB; else export SRMI_LIB=$R/$lib; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$i -o t -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-inference --no-edsr --no-dp-probe > $R/gpurun_out/prof_$i.log 2>&1) || exit 1
  python3 $R/tools/step_timeline.py $R/gpurun_out/prof_$i/t_kernel_trace.csv 1 > $R/gpurun_out/timeline_$i.txt 2>&1
  echo "== $lib" >> $R/gpurun_out/timelines.txt; cat $R/gpurun_out/timeline_$i.txt >> $R/gpurun_out/timelines.txt
done
unset SRMI_LIB
echo prof done
