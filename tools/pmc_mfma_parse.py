"""Per-dispatch MFMA busy cycles of the roofline kernels from a rocprofv3 --pmc csv.

Reports, per kernel, the average SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES and
GRBM_GUI_ACTIVE per dispatch, the kernel-trace duration, and
  mfma_frac_at_max_clock = SQ_VALU_MFMA_BUSY_CYCLES / (median duration * 2.4 GHz * 1024 SIMDs)
a LOWER bound on the MFMA utilisation (the chip runs at or below 2.4 GHz).  The
GRBM_GUI_ACTIVE-based clock (GRBM / 8 / duration) is reported only for dispatches of
0.3 ms or more: it reads high on shorter ones (MI355X_MICROARCH.md "DVFS give-back";
round 1 printed 2850-3006 MHz from 20 us dispatches).
next to the algorithmic MFMA cycles the kernel needs (FLOP / 1024 FLOP per SIMD-cycle
for bf16 16x16x32 / 32x32x16), so the counter's unit can be checked against a known
instruction count.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

FLOP = {}  # kernel-name prefix -> algorithmic FLOP per dispatch (optional check of the counter's unit)


def main(root, out):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
        for k, cs in per.items():
            for c, v in cs.items():
                vals[names[k]][c].append(v)
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    res = {}
    for name, cs in vals.items():
        if "srmi" not in name:
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        rec = {c.lower(): round(v, 1) for c, v in avg.items()}
        rec["dispatches"] = len(next(iter(cs.values())))
        g = avg.get("GRBM_GUI_ACTIVE")
        mb = avg.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if dur.get(name):
            d = sorted(dur[name])[len(dur[name]) // 2]
            rec["median_us"] = round(d, 2)
            if mb is not None:
                rec["mfma_frac_at_max_clock"] = round(mb / (d * 2400.0 * 1024), 4)
            if g and d >= 300.0:
                rec["clock_mhz_est"] = round(g / 8.0 / d, 1)
        for k, fl in FLOP.items():
            if k in name:
                rec["algorithmic_mfma_simd_cycles"] = fl / 1024.0
        res[name] = rec
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
