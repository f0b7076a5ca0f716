#!/bin/bash
# HBM bytes of a whole C2 training step: FETCH_SIZE and WRITE_SIZE passes (separate
# runs) over tools/roofline_driver.py --reps 0 (the bench's FusedTrainer, STEPS steps,
# no probes), every dispatch of the run summed, / STEPS -> gpurun_out/pmc_step.json
# (tools/pmc_step_parse.py; gfx950 corrections as tools/pmc_parse.py).
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_steptot
STEPS=${STEPS:-4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 $R/tools/roofline_driver.py --steps $STEPS --reps 0 > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 $R/tools/pmc_step_parse.py $OUT $STEPS $R/gpurun_out/pmc_step.json
