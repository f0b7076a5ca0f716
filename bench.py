#!/usr/bin/env python3
"""Benchmark: RCAN training tiles/s on MI355X (BASELINE.json metric, config 2/3).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, RCCL)

Workload (BASELINE configs[1], weak-scaled for N>1 = configs[2]): rcan-10-20-64
training step on 2-var (SSS_SST) 48x48 -> 192x192 tiles, 64 tiles per GPU,
bf16 MFMA operands with fp32 accumulation, fp32 master weights, Adam.
One step = bicubic 1/4 of the HR batch -> RCAN forward -> RMSE -> interp
baseline RMSE -> backward -> (RCCL loss + gradient all-reduce) -> Adam ->
bf16 filter repack: exactly dual_trainer.py:310-323.
Inputs are synthetic lnorm'ed N(0,1) tiles already resident in HBM.

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel
(the fused conv1 dgrad + filter-gradient launch of the RCAB backward, re-issued
by the bench's own engines at the in-step configuration and timed with HIP
events on their streams after the timed region; conv2's fused launch and the
isolated forward conv alongside; the step-level MFMA fraction) and the CPU baseline
(the oracle, a PyTorch-CPU restatement of the reference step, timed on this
host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "super-resolution-climate_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "training tiles/sec (48→192, bf16) at 1/2/4/8 MI355X; inference MPix/sec"
PEAK_BF16_TFLOPS = 2516.6          # 256 CU x 2.4 GHz x 4096 FLOP/clk (MI355X_MICROARCH.md, dense)
PEAK_FP32_TFLOPS = 157.3           # f32-input MFMA = the f32 vector rate (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
HBM_ACHIEVABLE_GBS = 6300.0        # MI355X_MICROARCH.md: sustained streaming, not a roofline peak
RIDGE_FLOP_PER_BYTE = PEAK_BF16_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)   # 314.6
TRAIN_GFLOP_PER_TILE_C2 = 219.9    # 6 x conv MACs per tile
EDSR_TRAIN_GFLOP_PER_TILE = 27.4   # C4 EDSR x8 4-var, 6 x 4.57 G MAC
CONV64_FLOP_PER_TILE = 2 * 64 * 576 * 48 * 48   # one 64->64 3x3 conv at 48x48 (84.93 M MAC)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="tiles per GPU")
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=4, help="timed CPU oracle steps per config (median, >= 3)")
    ap.add_argument("--no-interp-loss", action="store_true")
    ap.add_argument("--no-inference", action="store_true", help="skip the C5 tiled-region inference line")
    ap.add_argument("--no-edsr", action="store_true", help="skip the C4 EDSR x8 line")
    ap.add_argument("--edsr-batch", type=int, default=64)
    ap.add_argument("--micro", type=int, default=None, help="micro-batches per step (default: trainer's choice)")
    ap.add_argument("--cu-budget", type=int, default=None, help="CUs each engine sizes its launches for")
    ap.add_argument("--infer-region", type=int, default=4096, help="C5 HR region side (BASELINE: 4096)")
    ap.add_argument("--infer-iters", type=int, default=5)
    ap.add_argument("--no-train", action="store_true", help="skip the training leg (C4 / C5 lines only)")
    ap.add_argument("--no-dp-probe", action="store_true", help="skip the dp_overhead_1rank measurement")
    ap.add_argument("--force-dp", action="store_true",
                    help="diagnostic: the DP path (RCCL group, reducer stream, bucketed all-reduce) at one rank")
    ap.add_argument("--dp-reducer-stream", action="store_true",
                    help="A/B: the DP all-reduce on a reducer stream of its own (the event-driven schedule)")
    ap.add_argument("--ca-pass", action="store_true",
                    help="A/B: the training CA forward as a pass of its own after conv2 (SRMI_FLAG_CA_PASS)")
    ap.add_argument("--du-pass", action="store_true",
                    help="A/B: the CA backward writes du for the conv2 backward to read (SRMI_FLAG_DU_PASS)")
    ap.add_argument("--no-rcab-infer", action="store_true",
                    help="A/B: inference RCABs as three launches (SRMI_FLAG_NO_RCAB_INFER)")
    return ap.parse_args()


def synthetic_hr(batch, nchan, size, seed):
    """Synthetic HR tiles ~ N(0,1) from RandomState(seed), normalised per tile and
    channel to mean 0 / std 1 (ddof 0) -- the statistics of the reference's 'lnorm'
    tiles (sres/base/source/swot/raw.py:177-181).  Same stream as
    the tests' generator, so bench inputs equal the parity-test inputs."""
    import numpy as np
    x = np.random.RandomState(seed).standard_normal((batch, nchan, size, size))
    x = (x - x.mean(axis=(2, 3), keepdims=True)) / x.std(axis=(2, 3), keepdims=True)
    return x.astype(np.float32)


def _pmc_traffic(kernel_prefix):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (FETCH_SIZE x2
    + WRITE_SIZE, gfx950-corrected; tools/pmc_traffic.sh), or None."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        for k, v in d.items():
            if kernel_prefix in k:
                return {"bytes": v.get("hbm_bytes_per_launch"), "source": os.path.relpath(f, ROOT)}
    return None


def _pmc_infer_traffic(side, flags):
    """HBM bytes per launch of the inference RCAB kernel from the newest committed
    rocprofv3 --pmc summary of the C5 leg (tools/pmc_infer.sh: FETCH_SIZE x2 +
    WRITE_SIZE, gfx950-corrected), only when that summary was taken at the same
    configuration (its "config": region side and engine flags); else None."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_infer*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        cfg = d.get("config") or {}
        if cfg.get("infer_region") != side or cfg.get("flags", 0) != flags:
            continue
        for k, v in d.items():
            if isinstance(v, dict) and "hbm_bytes_per_launch" in v and "rcab_infer_kernel" in k:
                return {"bytes": v["hbm_bytes_per_launch"], "source": os.path.relpath(f, ROOT)}
    return None


def _pmc_mfma(kernel_prefix, infer_cfg=None):
    """MFMA busy fraction of a kernel (SQ_VALU_MFMA_BUSY_CYCLES / (median duration x
    2.4 GHz x 1024 SIMDs): a lower bound, the chip runs at or below 2.4 GHz) and the
    kernel-trace median duration of the same pass, from the newest committed summary
    (tools/pmc_mfma_parse.py: profiles/rNN_pmc_mfma.json for training,
    rNN_pmc_infer_mfma.json for C5 -- the latter only at the same configuration)."""
    pat = "*pmc_infer_mfma*.json" if infer_cfg is not None else "*pmc_mfma*.json"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pat)), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if infer_cfg is not None:
            cfg = d.get("config") or {}
            if cfg.get("infer_region") != infer_cfg[0] or cfg.get("flags", 0) != infer_cfg[1]:
                continue
        for k, v in d.items():
            if isinstance(v, dict) and kernel_prefix in k and "mfma_frac_at_max_clock" in v:
                return {"mfma_frac_at_max_clock": v["mfma_frac_at_max_clock"], "median_us": v.get("median_us"),
                        "source": os.path.relpath(f, ROOT)}
    return None


def _time_launches(launch, stream, n=50, warm=5):
    for _ in range(warm):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        launch()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


ACT_BF16_PER_TILE = 48 * 48 * 64 * 2    # one bf16 48x48x64 activation
ACT_F32_PER_TILE = 48 * 48 * 64 * 4
WGRAD_OUT_BYTES = 64 * 577 * 4           # dW (64x64x9) + db, fp32, once per launch
# Algorithmic bytes per tile of the two fused RCAB-backward launches (SURVEY.md §8(d),
# DESIGN.md "Kernels"): what each must move at least, every operand once.
#  F1 = rcab_bwd_kernel<DG_ACC_CA16>: conv1's dgrad (reads dz bf16, reads + writes the
#       in-group gradient stream g -- bf16 since round 6 --, reads the CA input u bf16 for
#       the CA sums) and conv1's filter gradient (reads its input hb bf16; dz already counted)
#  F2 = rcab_bwd_kernel<DG_RELUMASK>: conv2's dgrad (reads the bf16 stream g -- du =
#       g s + dm / HW formed in LDS since round 6; before, du bf16 --, reads the ReLU output
#       t bf16 as the mask, writes dz bf16) and conv2's filter gradient (t, g already counted)
F1_BYTES_PER_TILE = 5 * ACT_BF16_PER_TILE
F2_BYTES_PER_TILE = 3 * ACT_BF16_PER_TILE
FUSED_FLOP_PER_TILE = 2 * CONV64_FLOP_PER_TILE   # one dgrad conv + one filter-gradient conv


def _pmc_step_total(step_ms):
    """Whole-step HBM traffic from the newest committed summary of
    tools/pmc_step_total.sh (profiles/rNN_pmc_step.json: FETCH_SIZE x2 + WRITE_SIZE of
    every dispatch of a run of C2 steps, / steps) over this run's step time: the bytes
    floor of the step, against the 8 TB/s peak (and the guide's ~6.3 TB/s achievable)."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_step*.json")), reverse=True):
        try:
            d = json.load(open(f))
            b = float(d["bytes_per_step"])
        except Exception:
            continue
        ach = b / (step_ms * 1e-3) / 1e9
        return {"bytes_per_step": round(b), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "frac_of_achievable": round(ach / HBM_ACHIEVABLE_GBS, 4),
                "floor_ms_at_achievable": round(b / (HBM_ACHIEVABLE_GBS * 1e9) * 1e3, 3),
                "source": os.path.relpath(f, ROOT),
                "note": "PMC bytes of one whole step (all kernels) / this run's ms_per_step"}
    return None


def _prof_in_step_us(key):
    """In-step average launch duration (us) of the fused backward kernel `key` (F1 / F2)
    from the newest committed rocprofv3 kernel-trace summary of the bench
    (tools/prof_summary.py -> profiles/rNN_prof_summary.json), or None."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*prof_summary*.json")), reverse=True):
        try:
            d = json.load(open(f))
            return {"in_step_avg_us": d["fused"][key]["in_step_avg_us"], "source": os.path.relpath(f, ROOT)}
        except Exception:
            continue
    return None


def _probe_ms(issue, streams, reps):
    """Average per-launch duration (ms) on each stream of `reps` launches issued by
    issue(reps) (after 3 warm-up launches), HIP events on those streams."""
    issue(3)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
    for k, st in enumerate(streams):
        ev[k][0].record(st)
    issue(reps)
    for k, st in enumerate(streams):
        ev[k][1].record(st)
    torch.cuda.synchronize()
    return [ev[k][0].elapsed_time(ev[k][1]) / reps for k in range(len(streams))]


def fused_rooflines(tr, step_ms, reps=20):
    # per engine and step: conv2's fused launch (F2) runs once per RCAB; conv1's
    # (F1, EPI_DG_ACC_CA) once per RCAB except the first of each residual group, whose
    # conv1 dgrad accumulates into the group-input gradient instead (EPI_DG_ACC, a
    # different kernel: engine.cpp backward_impl)
    """Roofline of the dominant kernel AT ITS IN-STEP CONFIGURATION: the bench's own
    trainer engines re-issue their fused backward launch of one RCAB
    (srmi_engine_probe: same parameters, buffers, grid and CU split as inside the step),
    HIP events on the engines' own streams.  Two measurements:
    * per launch -- the `roofline` numbers (`frac`): engine 0 alone issues `reps`
      launches, one at a time, as a rocprofv3 kernel trace of the step sees them (the
      profiler serialises the streams): achieved = algorithmic bytes of ONE launch / its
      average duration.  `rocprof_check` recomputes it from the committed kernel-trace
      summary's in-step average of the same kernel;
    * concurrent slot (`concurrent`): every micro-batch engine issues its launch on its
      own stream at once, as in the step; bytes of all launches of a slot / the slowest
      stream's average -- what the two engines move together, not one launch's roofline."""
    from srmi._lib import call
    main_st = torch.cuda.current_stream()
    n_eng = len(tr.engines)
    tiles_per_engine = tr.engines[0].batch
    out = {}
    nl, nb = tr.spec.nlayers, tr.spec.nblocks
    per_step = {1: nl * (nb - 1), 2: nl * nb}
    streams = [tr.streams[k] or main_st for k in range(n_eng)]
    for which, key, name, bpt in ((1, "F1", "rcab_bwd_kernel<EPI_DG_ACC_CA16>", F1_BYTES_PER_TILE),
                                  (2, "F2", "rcab_bwd_kernel<EPI_DG_RELUMASK>", F2_BYTES_PER_TILE)):
        def issue_all(r):
            for k, eng in enumerate(tr.engines):
                call("srmi_engine_probe", eng._h, which, r, streams[k].cuda_stream)

        def issue_one(r):
            call("srmi_engine_probe", tr.engines[0]._h, which, r, streams[0].cuda_stream)

        ms1 = _probe_ms(issue_one, streams[:1], reps)[0]
        per_stream = _probe_ms(issue_all, streams, reps)
        ms = max(per_stream)
        bytes_launch = bpt * tiles_per_engine + WGRAD_OUT_BYTES
        flop_launch = FUSED_FLOP_PER_TILE * tiles_per_engine
        ach = bytes_launch / (ms1 * 1e-3) / 1e9
        tf = flop_launch / (ms1 * 1e-3) / 1e12
        ach_slot = bytes_launch * n_eng / (ms * 1e-3) / 1e9
        tr_ = _pmc_traffic("rcab_bwd_kernel<%d" % (11 if which == 1 else 4))
        prof = _prof_in_step_us(key)
        # the roof is set by the launch's arithmetic intensity against the ridge point
        # (bf16 dense peak / HBM peak = 314.6 FLOP/B): F1 (164 FLOP/B) is HBM-bound,
        # F2 (382 FLOP/B) MFMA-bound
        ai = flop_launch / bytes_launch
        mfma_bound = ai > RIDGE_FLOP_PER_BYTE
        rc = None
        if prof:
            sec = prof["in_step_avg_us"] * 1e-6
            a = (flop_launch / sec / 1e12) if mfma_bound else (bytes_launch / sec / 1e9)
            rc = {"in_step_avg_us": prof["in_step_avg_us"], "achieved": round(a, 1),
                  "frac": round(a / (PEAK_BF16_TFLOPS if mfma_bound else HBM_PEAK_GBS), 4), "source": prof["source"]}
        budget = tr.engines[0]._cfg.cu_budget or 256
        a_main, peak = (tf, PEAK_BF16_TFLOPS) if mfma_bound else (ach, HBM_PEAK_GBS)
        out[which] = {
            "bound": "mfma" if mfma_bound else "hbm", "achieved": round(a_main, 1), "peak": peak,
            "unit": "TFLOP/s" if mfma_bound else "GB/s", "frac": round(a_main / peak, 4),
            "arithmetic_intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": round(RIDGE_FLOP_PER_BYTE, 1),
            "traffic": tr_["bytes"] if tr_ and tr_["bytes"] is not None else None,
            "traffic_source": tr_["source"] if tr_ else None,
            "kernel": "srmi::" + name, "in_step": True,
            "frac_is": f"per launch: algorithmic {'flops' if mfma_bound else 'bytes'} of one launch / its average "
                       f"duration, the launch alone (engine 0's stream, in-step grid and CU split) against the "
                       f"WHOLE chip's peak.  The launch is sized for a {budget}-CU budget ({budget} of 256 CUs, one "
                       f"workgroup per CU), so alone it can reach at most ~{budget / 256:.2f} of the chip: "
                       f"frac_of_budget = frac x 256 / {budget}",
            "cu_budget": budget, "frac_of_budget": round(a_main / peak * 256 / budget, 4),
            "config": f"one launch of {tiles_per_engine} tiles (micro-batch engine 0), in-step grid and CU split",
            "avg_launch_ms": round(ms1, 4), "bytes_per_launch": bytes_launch, "flop_per_launch": flop_launch,
            "hbm_gbs": round(ach, 1), "hbm_frac": round(ach / HBM_PEAK_GBS, 4),
            "mfma_tflops": round(tf, 1), "mfma_frac": round(tf / PEAK_BF16_TFLOPS, 4),
            "rocprof_check": rc,
            "mfma_pmc": _pmc_mfma("rcab_bwd_kernel<%d" % (11 if which == 1 else 4)),
            "concurrent": {"launches_per_slot": n_eng, "per_stream_ms": [round(x, 4) for x in per_stream],
                           "achieved": round(ach_slot, 1), "unit": "GB/s", "frac": round(ach_slot / HBM_PEAK_GBS, 4),
                           "mfma_frac": round(flop_launch * n_eng / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                           "note": "all micro-batch engines' launches at once, as in the step: bytes of the "
                                   "slot / slowest stream's average.  Not rocprof-verifiable: a kernel trace "
                                   "serialises the two streams"},
            "launches_per_engine_per_step": per_step[which],
            "share_of_step": round(ms * per_step[which] / step_ms, 3),
        }
    return out[1], out[2]


def conv_fwd_roofline(dev, batch):
    """The forward conv (fused bias + ReLU epilogue), ISOLATED: one launch over the
    bench's B tiles on the current stream (in the step it runs at the same shape,
    once per micro engine)."""
    from srmi._lib import call, ptr
    g = torch.Generator(device="cpu").manual_seed(0)
    N, H, W = batch, 48, 48
    st = torch.cuda.current_stream()
    x = torch.randn(N, H, W, 64, generator=g).to(dev).to(torch.bfloat16)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(dev)
    b = torch.zeros(64, device=dev)
    fp = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=dev)
    dp = torch.empty_like(fp)
    pb = torch.empty(64, device=dev)
    call("srmi_pack_conv", ptr(w), ptr(b), 64, 64, 0, ptr(fp), ptr(dp), ptr(pb), 0, st.cuda_stream)
    y = torch.empty_like(x)
    flop = CONV64_FLOP_PER_TILE * N
    ms_c = _time_launches(lambda: call("srmi_conv3x3", ptr(x), ptr(fp), ptr(pb), N, H, W, 64, 64, 0, 0, ptr(y), None,
                                       None, None, None, None, None, 1.0, 0, st.cuda_stream), st)
    trc = _pmc_traffic("conv64_kernel<48, 0")
    ach_c = flop / (ms_c * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(ach_c, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach_c / PEAK_BF16_TFLOPS, 4), "traffic": trc["bytes"] if trc else None,
            "kernel": "srmi::conv64_kernel<48,RELU>", "in_step": False, "config": f"isolated, {N} tiles",
            "avg_launch_ms": round(ms_c, 4), "flop_per_launch": flop,
            "bytes_per_launch": 2 * N * ACT_BF16_PER_TILE + 64 * 576 * 2}


RCAB_INFER_BYTES_PER_IMAGE = 48 * 48 * 64 * 10     # h pair in + out (3 + 3 B), t written + read (2 + 2 B)
RCAB_INFER_FLOP_PER_IMAGE = 2 * CONV64_FLOP_PER_TILE  # conv1 + conv2 (the CA MLP is negligible)


def infer_rcab_roofline(ti, side, flags, reps=20):
    """Roofline of C5's dominant kernel, the one-launch inference RCAB
    (rcab_infer_kernel: conv1 -> CA scale -> conv2 + h' = h + s u, a workgroup per
    image), at its in-region configuration: srmi_engine_probe(which = 3) re-issues RCAB
    (0, 2) of the last forward on the engine's own stream, HIP events there.  Per
    launch, the launch alone on the chip (as a rocprofv3 trace sees it): algorithmic
    bytes (RCAB_INFER_BYTES_PER_IMAGE x images) / average duration; the MFMA fraction
    of the same launch beside it.  `concurrent`: every engine's launch at once, as in the
    region.  `traffic`: PMC bytes per launch from a committed summary of the SAME
    configuration, else null."""
    from srmi._lib import call
    main_st = torch.cuda.current_stream()
    streams = [ti.streams[k] or main_st for k in range(len(ti.engs))]
    n = ti.engs[0].batch

    def issue_one(r):
        call("srmi_engine_probe", ti.engs[0]._h, 3, r, streams[0].cuda_stream)

    def issue_all(r):
        for k, e in enumerate(ti.engs):
            call("srmi_engine_probe", e._h, 3, r, streams[k].cuda_stream)

    ms1 = _probe_ms(issue_one, streams[:1], reps)[0]
    per_stream = _probe_ms(issue_all, streams, reps)
    nb = RCAB_INFER_BYTES_PER_IMAGE * n
    nf = RCAB_INFER_FLOP_PER_IMAGE * n
    ach = nb / (ms1 * 1e-3) / 1e9
    tf = nf / (ms1 * 1e-3) / 1e12
    tot = sum(e.batch for e in ti.engs)
    ach_slot = RCAB_INFER_BYTES_PER_IMAGE * tot / (max(per_stream) * 1e-3) / 1e9
    tr_ = _pmc_infer_traffic(side, flags)
    mp = _pmc_mfma("rcab_infer_kernel", (side, flags))
    rc = None
    if mp and mp.get("median_us"):
        a = nb / (mp["median_us"] * 1e-6) / 1e9
        rc = {"median_us": mp["median_us"], "achieved": round(a, 1), "frac": round(a / HBM_PEAK_GBS, 4),
              "source": mp["source"]}
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "rocprof_check": rc, "mfma_pmc": mp,
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": round(tr_["bytes"]) if tr_ else None, "traffic_source": tr_["source"] if tr_ else None,
            "kernel": "srmi::rcab_infer_kernel", "images_per_launch": n, "avg_launch_ms": round(ms1, 4),
            "bytes_per_launch": nb, "flop_per_launch": nf, "mfma_tflops": round(tf, 1),
            "mfma_frac": round(tf / PEAK_BF16_TFLOPS, 4),
            "frac_is": "per launch: algorithmic bytes (h pair in/out, t written/read: 10 B per element) / "
                       "average duration, the launch alone on the chip",
            "concurrent": {"launches": len(ti.engs), "per_stream_ms": [round(x, 4) for x in per_stream],
                           "achieved": round(ach_slot, 1), "frac": round(ach_slot / HBM_PEAK_GBS, 4)}}


def inference_bench(dev, side, iters, flags=0, info=None):
    """BASELINE config 5: RCAN inference over a full region, 1 variable, HR side x side
    cut floor-wise into 192x192 tiles (4096 -> 21 x 21 = 441 tiles, 4032^2 HR produced),
    per region: tiling + lnorm, bicubic 1/4, rcan-10-20-64 forward (bf16 MFMA), bicubic
    x4 baseline, both RMSEs, de-normalised mosaics of input/target/interp/model --
    captured once as a HIP graph and replayed (dual_trainer.process_image semantics).
    MPix/s counts produced HR pixels."""
    from srmi.engine import NetSpec
    from srmi.inference import TiledInference
    from srmi.trainer import default_init_
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4, flags=flags)
    from srmi.engine import param_table
    table = param_table(spec)
    params = torch.empty(sum(t[2] for t in table), dtype=torch.float32, device=dev)
    default_init_(params, table, 0)
    region = torch.tensor(synthetic_hr(1, 1, side, 99)[0]).to(dev)
    multi = info is not None and info.enabled
    micro = int(os.environ["SRMI_INFER_MICRO"]) if os.environ.get("SRMI_INFER_MICRO") else None  # A/B only
    ti = TiledInference(spec, params, tuple(region.shape), (192, 192), device=dev, graph=not multi, micro=micro,
                        info=info if multi else None)
    ti.process_region(region)  # builds + captures the graph
    torch.cuda.synchronize()
    if multi:
        # multi-rank: the region's tiles round-robin over the ranks,
        # mosaics and per-tile loss sums all-gathered; wall time of whole regions
        torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            ti.process_region(region)
        torch.cuda.synchronize()
        torch.distributed.barrier()
        ms = 1000 * (time.perf_counter() - t0) / iters
    else:
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            ti.replay()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / iters
    mpix = ti.n * 192 * 192 / 1e6
    roof = None
    if not multi and not (flags & 2):
        roof = infer_rcab_roofline(ti, side, flags)
    return {"metric": "inference MPix/sec (HR pixels produced)", "value": round(mpix / (ms * 1e-3), 2),
            "roofline": roof,
            "unit": "MPix/s", "ms_per_region": round(ms, 3), "tiles": ti.n, "hr_mpix_per_region": round(mpix, 3),
            "model_tflops": round(ti.n * 73.26e9 / (ms * 1e-3) / 1e12, 1),
            "mfma_frac": round(ti.n * 73.26e9 / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
            "dtype": "bf16", "data": "synthetic",
            "rcab_one_launch": not (flags & 2), "n_gpus": info.world if multi else 1,
            "config": {"workload": f"rcan-10-20-64 tiled inference, 1 var, {side}x{side} HR region, 192^2 tiles "
                                   "(floor)" + (f", tiles round-robin over {info.world} ranks + all-gather"
                                                if multi else ", graph-replayed"), "graph": not multi}}


def edsr_bench(dev, batch, steps, warmup):
    """BASELINE config 4: EDSR-style x8 (16 ResBlocks, 64 features, 3 x [conv 64->256 +
    PixelShuffle 2]), 4-variable tiles 32x32 -> 256x256, fp32 as BASELINE names it:
    the engine's exact-fp32 mode (v_mfma_f32_16x16x4_f32, fp32 activations, packs and
    gradients).  Full train step (down8, fwd, RMSE + interp RMSE, bwd, Adam) on this
    GPU; the step's MFMA fraction is against the fp32 matrix peak (157.3 TF)."""
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer
    spec = NetSpec(arch="edsr", nchannels_in=4, nchannels_out=4, nfeatures=64, nlayers=16, scale=8, dtype="fp32")
    tr = FusedTrainer(spec, batch, (32, 32), lr=1e-4, device=dev, seed=0)
    hr = torch.tensor(synthetic_hr(batch, 4, 256, 4321)).to(dev)
    for _ in range(warmup):
        tr.step(hr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(hr)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    v = batch * steps / dt
    tf = v * EDSR_TRAIN_GFLOP_PER_TILE / 1000.0
    return {"metric": "EDSR x8 training tiles/sec (32->256, 4-var, fp32)", "value": round(v, 2), "unit": "tiles/s",
            "ms_per_step": round(1000 * dt / steps, 3), "steps": steps, "warmup": warmup, "dtype": "f32",
            "data": "synthetic", "model_tflops": round(tf, 1),
            "roofline_step": {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                              "frac": round(tf / PEAK_FP32_TFLOPS, 4)},
            "config": {"workload": "edsr-16-64 x8 train step (down8 + fwd + RMSE + interp RMSE + bwd + Adam), "
                                   "4-var 32x32->256x256 tiles, exact fp32", "batch": batch}}


def dp_overhead_probe(args, reps=2):
    """dp_overhead_1rank: the data-parallel machinery's own cost on one GPU -- a
    one-rank RCCL process group (backend "nccl"), the reducer's comm stream, the
    per-residual-group events and the 11 bucketed all-reduces of the N>1 path
    (bench --force-dp) -- against the plain step.  Each leg runs as a CHILD process
    with one trainer, as a real rank does: a second trainer in this process would
    add its streams to this one's and oversubscribe the 4 hardware queues a process
    gets (GPU_MAX_HW_QUEUES), which measured -42 % for reasons that are not the DP
    path's.  `reps` interleaved rounds of plain / DP children, best of each.
    Streams per rank: one per micro-batch engine + the reducer's comm stream (+ RCCL's
    internal stream)."""
    import subprocess
    base = [sys.executable, os.path.abspath(__file__), "--no-cpu-baseline", "--no-inference", "--no-edsr",
            "--no-dp-probe", "--steps", str(args.steps), "--warmup", str(args.warmup), "--batch", str(args.batch)]
    if args.micro is not None:
        base += ["--micro", str(args.micro)]
    for flag in ("ca_pass", "du_pass", "dp_reducer_stream"):
        if getattr(args, flag):
            base += ["--" + flag.replace("_", "-")]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    best = {"plain": 0.0, "dp": 0.0}
    micro = None
    for _ in range(reps):
        for name, extra in (("plain", []), ("dp", ["--force-dp"])):
            r = subprocess.run(base + extra, env=env, capture_output=True, text=True, timeout=240)
            if r.returncode != 0:
                return {"error": f"{name} child exited {r.returncode}: {r.stderr.strip().splitlines()[-1:]}"}
            line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            best[name] = max(best[name], line["value"])
            micro = line.get("micro", micro)
    return {"tiles_per_s_plain": round(best["plain"], 2), "tiles_per_s_dp": round(best["dp"], 2),
            "overhead_frac": round(1.0 - best["dp"] / best["plain"], 4),
            "streams_per_rank": (f"{micro} engine stream(s) + 1 reducer comm stream (+ RCCL internal)"
                                 if args.dp_reducer_stream else f"{micro} engine stream(s) (+ RCCL internal)"),
            "config": f"1-rank RCCL group, {micro} micro-batch engine(s), same B={args.batch}, child process per "
                      f"leg (one trainer per process, as a rank), best of {reps} interleaved rounds of "
                      f"{args.steps} steps"}


def _log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _cpu_share():
    """CPUs this process may use: its affinity, capped by the cgroup CPU quota
    (cpu.max) -- on a GPU box the affinity lists the whole host while the quota
    holds the box's share."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except Exception:
        pass
    return n


def cpu_baseline(steps):
    """the oracle (PyTorch-CPU restatement of the reference step,
    dual_trainer.py:310-323 with array2tensor's requires_grad, the interp-loss
    metric and .item()) for C1 = rcan-10-20-64, B=4, fp32, with C=1 (as BASELINE
    words it) and C=2 (the bench workload's 2-var task), on all host cores
    available to this process (_cpu_share); warm-up 1 step, median of `steps`
    (>= 3) steps.  `value` is the C=2 number (the bench workload's shape)."""
    import statistics
    from oracle import rcan_oracle as ro
    threads = _cpu_share()
    torch.set_num_threads(threads)
    B = 4
    per = {}
    t_all = 0.0
    for C in (1, 2):
        model = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=10, nblocks=20)
        ro.init_params_numpy(model, 0)
        opt = ro.AdamOracle(list(model.parameters()), lr=1e-4)
        hr = torch.tensor(ro.synthetic_hr(B, C, 192, 1234))
        ro.train_step(model, opt, hr, 4, interp_loss=True)   # warm-up
        _log(f"cpu baseline C={C}: warm-up done")
        ts = []
        for _ in range(max(3, steps)):
            t0 = time.perf_counter()
            ro.train_step(model, opt, hr, 4, interp_loss=True)
            ts.append(time.perf_counter() - t0)
        t_all += sum(ts)
        med = statistics.median(ts)
        per[f"C{C}"] = {"tiles_per_s": round(B / med, 3), "median_s_per_step": round(med, 3), "steps": len(ts)}
    model_name = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model_name = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"value": per["C2"]["tiles_per_s"], "unit": "tiles/s", "cores": threads, "kind": "port",
            "configs": per,
            "sample": f"oracle rcan-10-20-64 fp32 train step (down4+fwd+RMSE+interp RMSE+bwd+Adam), B={B}, "
                      f"C=1 and C=2, 1 warm-up + median of {max(3, steps)} steps each ({t_all:.1f} s timed), "
                      f"torch CPU threads={threads} (this process's CPU share: affinity capped by the cgroup "
                      f"quota), cpu='{model_name}'"}


def main():
    args = parse()
    from srmi.dist import init_from_env
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer

    info = init_from_env(None, force=args.force_dp)
    world = info.world
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", info.local_rank)
    torch.cuda.set_device(dev)
    C, B = args.channels, args.batch
    if args.no_train:  # diagnostic: the C4 / C5 lines alone
        rec = {"edsr_x8": None if args.no_edsr else edsr_bench(dev, args.edsr_batch, 10, 3),
               "inference": None if args.no_inference else inference_bench(dev, args.infer_region, args.infer_iters,
                                                                           2 if args.no_rcab_infer else 0)}
        print(json.dumps(rec), flush=True)
        return
    from srmi._lib import SRMI_FLAG_CA_PASS, SRMI_FLAG_DU_PASS
    flags = (SRMI_FLAG_CA_PASS if args.ca_pass else 0) | (SRMI_FLAG_DU_PASS if args.du_pass else 0)
    spec = NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4, flags=flags)
    tr = FusedTrainer(spec, B, (48, 48), lr=1e-4, interp_loss=not args.no_interp_loss, info=info, device=dev, seed=0,
                      micro=args.micro, cu_budget=args.cu_budget, dp_reducer_stream=args.dp_reducer_stream)
    hr = torch.tensor(synthetic_hr(B, C, 192, 1234 + info.rank)).to(dev)

    micro = tr.micro
    _log(f"trainer ready (B={B}, C={C}, micro={micro}, world={world})")
    for _ in range(args.warmup):
        tr.step(hr)
    torch.cuda.synchronize()
    _log("warm-up done")
    if info.enabled:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    # per-step GPU times: an event on the main stream behind every step (the step ends
    # with the main stream joined to every engine stream); consecutive differences
    main_st = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(main_st)
    for k in range(args.steps):
        out = tr.step(hr)
        evs[k + 1].record(main_st)
    t_host = time.perf_counter() - t0  # host enqueue time of the K steps (GPU may still run)
    torch.cuda.synchronize()
    if info.enabled:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if info.enabled:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    loss = float(out["loss"])
    step_ev = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps))
    nq = len(step_ev)
    step_stats = {"median_ms": round(step_ev[nq // 2] if nq % 2 else 0.5 * (step_ev[nq // 2 - 1] + step_ev[nq // 2]), 3),
                  "min_ms": round(step_ev[0], 3), "max_ms": round(step_ev[-1], 3),
                  "p10_ms": round(step_ev[int(0.1 * (nq - 1))], 3), "p90_ms": round(step_ev[int(0.9 * (nq - 1))], 3),
                  "n": nq, "source": "HIP events on the main stream behind every timed step"}
    tiles = B * world * args.steps
    value = tiles / dt
    step_ms = 1000 * dt / args.steps
    # host cost of enqueuing ONE step onto an idle device (queue empty): the
    # back-to-back enqueue time above includes waiting on a full hardware queue
    idle = []
    for _ in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tr.step(hr)
        idle.append(time.perf_counter() - t1)
        torch.cuda.synchronize()
    host_idle_ms = 1000 * sorted(idle)[1]
    if info.rank == 0:
        roof, roof_f2 = fused_rooflines(tr, step_ms)
        step_tf = value / world * TRAIN_GFLOP_PER_TILE_C2 / 1000.0
        roof["step_mfma_tflops"] = round(step_tf, 1)
        roof["step_mfma_frac"] = round(step_tf / PEAK_BF16_TFLOPS, 4)
    del tr, hr  # the extra lines below run on their own engines
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    dp_probe = None
    if world == 1 and not info.enabled and not args.no_dp_probe:
        dp_probe = dp_overhead_probe(args)
        _log(f"dp probe: {dp_probe}")
    _log(f"timed: {value:.1f} tiles/s")
    infer_dp = None
    if world > 1 and not args.no_inference:  # every rank takes part (collectives)
        infer_dp = inference_bench(dev, args.infer_region, args.infer_iters, 2 if args.no_rcab_infer else 0, info)
        _log("multi-rank inference done")
    if info.rank == 0:
        roof_conv = conv_fwd_roofline(dev, B)
        _log("rooflines done")
        edsr = None
        if not args.no_edsr and world == 1:
            edsr = edsr_bench(dev, args.edsr_batch, 10, 3)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            _log("edsr done")
        infer = None
        if not args.no_inference and world == 1:
            infer = inference_bench(dev, args.infer_region, args.infer_iters, 2 if args.no_rcab_infer else 0)
            _log("inference done")
        if world > 1:
            infer = infer_dp
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_steps)
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "tiles/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * dt / args.steps, 3), "step_times": step_stats,
            "ca_pass": bool(args.ca_pass), "du_pass": bool(args.du_pass),
            "host_enqueue_ms_per_step": round(1000 * t_host / args.steps, 3),
            "host_enqueue_idle_ms_per_step": round(host_idle_ms, 3), "micro": micro, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": "rcan-10-20-64 train step (down4 + fwd + RMSE + interp RMSE + bwd + Adam), "
                                   f"{C}-var 48x48->192x192 tiles",
                       "global_batch": B * world, "per_gpu_batch": B, "tile": "48->192",
                       "parallelism": f"dp{world}"},
            "model_tflops": round(value * TRAIN_GFLOP_PER_TILE_C2 / 1000.0, 1),
            "loss": loss,
            "roofline": roof,
            "roofline_f2": roof_f2,
            "step_traffic": _pmc_step_total(step_ms),
            "roofline_conv_fwd": roof_conv,
            "dp_overhead_1rank": dp_probe,
            "cpu_baseline": cpu,
            "inference": infer,
            "edsr_x8": edsr,
        }
        print(json.dumps(rec), flush=True)
    if info.enabled:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
