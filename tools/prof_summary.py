"""Summarise a rocprofv3 kernel trace of `bench.py` for profiles/.

The bench's roofline kernels are timed in isolation right after the timed step
loop (5 warm-up + 50 timed launches each); inside the training step the filter-
gradient kernels run on a side stream concurrently with the dgrad chain, so
their in-step durations are stretched by sharing the GPU.  This reports both,
per kernel: the isolated roofline-phase average (what bench.py's `roofline`
uses) and the in-step average/total.

    python tools/prof_summary.py <kernel_trace.csv> <bench_log_with_json_line> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def main(trace, bench_log, out):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    line = None
    for ln in open(bench_log):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    res = {"bench": {k: line[k] for k in ("value", "unit", "ms_per_step")} if line else None, "kernels": {}}
    names = {"wgrad": "wgrad48_kernel", "conv_fwd": "conv64_kernel<48, 0, 2>"}
    for key, pat in names.items():
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if pat in r["Kernel_Name"]]
        if not d:
            continue
        # the roofline phase is the last 55 launches of the kernel before the inference section:
        # find the 55-launch run of isolated dispatches (no other srmi kernel in between)
        idx = [i for i, r in enumerate(rows) if pat in r["Kernel_Name"]]
        iso = []
        for j in range(len(idx) - 1, -1, -1):
            i = idx[j]
            prev_ok = j > 0 and idx[j - 1] == i - 1
            if prev_ok or (iso and idx[j + 1] == i + 1):
                iso.append(i)
                if len(iso) == 55:
                    break
            elif iso:
                iso = []
        iso_d = [int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"]) for i in sorted(iso)[5:]]
        res["kernels"][key] = {
            "name_contains": pat, "dispatches": len(d), "avg_us_all": round(sum(d) / len(d) / 1e3, 3),
            "roofline_phase_avg_us": round(sum(iso_d) / len(iso_d) / 1e3, 3) if iso_d else None,
            "roofline_phase_dispatches": len(iso_d),
        }
        if line:
            rk = "roofline" if key == "wgrad" else "roofline_conv_fwd"
            res["kernels"][key]["bench_event_avg_us"] = round(line[rk]["avg_launch_ms"] * 1e3, 3)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
