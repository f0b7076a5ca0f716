"""Whole-step HBM traffic from the two rocprofv3 --pmc passes of tools/pmc_step_total.sh:
every dispatch of the run (STEPS training steps + the trainer's one initial filter
pack) summed per counter, FETCH_SIZE x2 (gfx950: a 16 B/lane read counts half its
bytes, MI355X_MICROARCH.md HBM section), WRITE_SIZE as is, both KiB -> bytes, / STEPS.

    python tools/pmc_step_parse.py <pmc dir> <steps> <out.json>
"""
import json
import sys
from collections import defaultdict

from pmc_parse import per_kernel  # noqa: E402  (tools/ on sys.path when run as a script)


def main(root, steps, out):
    fetch, nf = per_kernel(root, "FETCH_SIZE")
    write, nw = per_kernel(root, "WRITE_SIZE")
    per = defaultdict(dict)
    tot_f = tot_w = 0.0
    for k in set(fetch) | set(write):
        fb = fetch.get(k, 0.0) * nf.get(k, 0) * 1024.0 * 2.0 / steps
        wb = write.get(k, 0.0) * nw.get(k, 0) * 1024.0 / steps
        tot_f += fb
        tot_w += wb
        per[k] = {"bytes_per_step": fb + wb, "dispatches_per_step": nf.get(k, 0) / steps}
    top = dict(sorted(per.items(), key=lambda kv: -kv[1]["bytes_per_step"])[:12])
    res = {"steps": steps, "fetch_bytes_per_step": tot_f, "write_bytes_per_step": tot_w,
           "bytes_per_step": tot_f + tot_w, "config": "C2: rcan-10-20-64, 2-var, B=64, micro=2 (bench.py default)",
           "note": "all dispatches of the run / steps (includes the trainer's initial filter pack, <0.2 %)",
           "top_kernels": top}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "top_kernels"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
