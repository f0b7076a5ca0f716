"""Summarise a rocprofv3 kernel trace of `bench.py` for profiles/.

Reports the kernel table of the run (dispatches, average and total duration per
kernel), and for the two fused RCAB-backward kernels the average duration of the
roofline-phase dispatches (bench.py fused_rooflines, after the timed steps: engine 0
alone, 3 warm-up + 20 timed launches, then every engine at once) next to the bench's
HIP-event per-launch average, plus the average over the in-step dispatches.

    python tools/prof_summary.py <kernel_trace.csv> <bench_log_with_json_line> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict

REPS, WARM = 20, 3


def main(trace, bench_log, out):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    line = None
    for ln in open(bench_log):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    res = {"bench": {k: line[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup")} if line else None,
           "fused": {}, "kernels": {}}
    dur = defaultdict(list)
    for r in rows:
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in dur.values())
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        res["kernels"][k[:120]] = {"dispatches": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 3),
                                   "total_ms": round(sum(v) / 1e6, 3), "share": round(sum(v) / tot, 4)}
    n_eng = 1
    if line and line.get("roofline"):
        n_eng = line["roofline"].get("concurrent", {}).get("launches_per_slot", 1)
    for key, pat, rk in (("F1", "rcab_bwd_kernel<11", "roofline"), ("F2", "rcab_bwd_kernel<4", "roofline_f2")):
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if pat in r["Kernel_Name"]]
        if not d:
            continue
        # bench.fused_rooflines after the timed steps: engine 0 alone (WARM + REPS launches),
        # then every engine at once (WARM + REPS each)
        tail = d[-(REPS + WARM) * (1 + n_eng):]
        alone = tail[WARM:WARM + REPS]
        instep = d[:-(REPS + WARM) * (1 + n_eng)]
        rec = {"name_contains": pat, "dispatches": len(d),
               "roofline_phase_avg_us": round(sum(alone) / len(alone) / 1e3, 3),
               "in_step_avg_us": round(sum(instep) / len(instep) / 1e3, 3) if instep else None}
        if line and line.get(rk):
            rec["bench_event_avg_us"] = round(line[rk]["avg_launch_ms"] * 1e3, 3)
        res["fused"][key] = rec
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["fused"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
