"""Per-step GPU timeline of a training bench from a rocprofv3 kernel trace.

Steps are delimited by the Adam kernel (one launch per step).  For each of the
last steps it reports the wall time (first downsample of the step to the end of
its last kernel), the GPU-busy time (union of kernel intervals), idle gaps, and
the per-kernel total / count inside the step (summed durations: kernels on two
streams overlap, so the sum can exceed the wall).

    python tools/step_timeline.py <kernel_trace.csv> [n_steps=2]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("srmi::", "")


def main(path, nsteps=2):
    rows = list(csv.DictReader(open(path)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    adam = [i for i, e in enumerate(ev) if "adam_kernel" in e[2]]
    if len(adam) < 2:
        print("fewer than 2 adam launches")
        return
    # training steps of the headline RCAN config only: other phases of a bench
    # trace (roofline leg, tiled inference, the EDSR line) end in an Adam too
    def is_train(seg):
        names = [e[2] for e in seg]
        return (sum("rcab_bwd_kernel" in n for n in names) >= 100 and not any("region_to_tiles" in n for n in names)
                and not any("<32," in n for n in names))
    ks = [k for k in range(1, len(adam)) if is_train(ev[adam[k - 1] + 1:adam[k] + 1])]
    for k in ks[-nsteps:]:
        seg = ev[adam[k - 1] + 1:adam[k] + 1]
        ds = [i for i, e in enumerate(seg) if "downsample_kernel" in e[2]]
        if ds:
            seg = seg[ds[0]:]
        t0, t1 = seg[0][0], max(e[1] for e in seg)
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        for s, e, _ in seg:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        tot = defaultdict(lambda: [0, 0])
        for s, e, n in seg:
            tot[short(n)][0] += e - s
            tot[short(n)][1] += 1
        wall = t1 - t0
        print(f"step {k}: wall {wall / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(wall - busy) / 1e6:.3f} ms "
              f"in {len(gaps)} gaps (max {max(gaps, default=0) / 1e3:.1f} us)  launches {len(seg)}")
        for n, (d, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:25]:
            print(f"   {d / 1e6:8.3f} ms  {c:5d} x {d / c / 1e3:8.2f} us  {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
