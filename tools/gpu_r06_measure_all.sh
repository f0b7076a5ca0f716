#!/bin/bash
# The round's measurement set on the in-tree library (each GPU step under its own limit):
#   part 1: smoke, the default bench line, a kernel trace of a short bench (in-step
#           averages, per-step timeline), the whole-step PMC traffic
#   part 2: the per-kernel PMC passes over tools/roofline_driver.py (FETCH_SIZE,
#           WRITE_SIZE, MFMA busy) and the C5 inference leg's PMC passes + kernel stats
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
PART=${1:-1}
if [ "$PART" = 1 ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
  tail -2 $O/smoke.log
  NOPMC= bash tools/gpu_r06_measure.sh || exit 3
  exit 0
fi
bash tools/pmc_step.sh || exit 5
bash tools/pmc_infer.sh || exit 6
bash tools/prof_infer.sh > /dev/null || exit 7
echo part2 done
