#!/bin/bash
# round 6: -m gpu tests on the in-tree library, then an interleaved C2 A/B of the in-tree
# build against the variants named in $AB (tools/ab_var.sh syntax), REPS rounds
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=$R/gpurun_out; mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  SRMI_PARITY_REPORT=$O/c2_parity_ab.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06_ab_tests.log 2>&1 || { tail -40 $O/r06_ab_tests.log; exit 1; }
  tail -2 $O/r06_ab_tests.log
fi
rm -f $O/ab_var.log
REPS=${REPS:-3} bash tools/ab_var.sh "new::" $AB || exit 2
