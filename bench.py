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
(the 64->64 3x3 conv, measured live with HIP events) and the CPU baseline
(the oracle, a PyTorch-CPU restatement of the reference step, timed on this
host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
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
HBM_PEAK_GBS = 8000.0
TRAIN_GFLOP_PER_TILE_C2 = 219.9    # 6 x conv MACs per tile
CONV64_FLOP_PER_TILE = 2 * 64 * 576 * 48 * 48   # one 64->64 3x3 conv at 48x48 (84.93 M MAC)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="tiles per GPU")
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-interp-loss", action="store_true")
    return ap.parse_args()


def conv_roofline(dev, batch):
    """Average duration of the dominant kernel (64->64 3x3 conv, fused bias+ReLU
    epilogue, B tiles of 48x48) from HIP events on its launch stream."""
    from srmi._lib import call, ptr
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(batch, 48, 48, 64, generator=g).to(dev).to(torch.bfloat16)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(dev)
    b = torch.zeros(64, device=dev)
    fp = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=dev)
    dp = torch.empty_like(fp)
    pb = torch.empty(64, device=dev)
    st = torch.cuda.current_stream()
    call("srmi_pack_conv", ptr(w), ptr(b), 64, 64, 0, ptr(fp), ptr(dp), ptr(pb), st.cuda_stream)
    y = torch.empty(batch, 48, 48, 64, dtype=torch.bfloat16, device=dev)

    def launch():
        call("srmi_conv3x3", ptr(x), ptr(fp), ptr(pb), batch, 48, 48, 64, 64, 0, 0, ptr(y), None, None, None, None,
             None, None, 1.0, st.cuda_stream)

    for _ in range(5):
        launch()
    n = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        launch()
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / n
    flop = CONV64_FLOP_PER_TILE * batch
    achieved = flop / (ms * 1e-3) / 1e12
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "conv3x3_pmc.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    return {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
            "kernel": "srmi::conv3x3_kernel<48,EPI_RELU_BF16>", "avg_launch_ms": round(ms, 4),
            "flop_per_launch": flop}


def cpu_baseline(channels, steps):
    """Oracle (PyTorch-CPU restatement of the reference step) on this host's cores."""
    from oracle import rcan_oracle as ro
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count() or 1
    threads = max(1, min(16, avail))
    torch.set_num_threads(threads)
    B = 4
    model = ro.RCANOracle(nchannels_in=channels, nchannels_out=channels, nlayers=10, nblocks=20)
    ro.init_params_numpy(model, 0)
    opt = ro.AdamOracle(list(model.parameters()), lr=1e-4)
    hr = torch.tensor(ro.synthetic_hr(B, channels, 192, 1234))
    ro.train_step(model, opt, hr, 4, interp_loss=True)   # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        ro.train_step(model, opt, hr, 4, interp_loss=True)
    dt = time.perf_counter() - t0
    model_name = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model_name = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"value": round(B * steps / dt, 3), "unit": "tiles/s", "cores": threads, "kind": "port",
            "sample": f"oracle rcan-10-20-64 fp32 train step (down4+fwd+RMSE+interp RMSE+bwd+Adam), "
                      f"B={B}, C={channels}, 1 warm-up + {steps} timed steps, {dt:.1f} s, torch CPU threads="
                      f"{threads}, cpu='{model_name}'"}


def main():
    args = parse()
    from srmi.dist import init_from_env
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer
    from oracle import rcan_oracle as ro  # synthetic inputs only (same generator as the tests)

    info = init_from_env()
    world = info.world
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", info.local_rank)
    torch.cuda.set_device(dev)
    C, B = args.channels, args.batch
    spec = NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)
    tr = FusedTrainer(spec, B, (48, 48), lr=1e-4, interp_loss=not args.no_interp_loss, info=info, device=dev, seed=0)
    hr = torch.tensor(ro.synthetic_hr(B, C, 192, 1234 + info.rank)).to(dev)

    for _ in range(args.warmup):
        tr.step(hr)
    torch.cuda.synchronize()
    if info.enabled:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = tr.step(hr)
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
    tiles = B * world * args.steps
    value = tiles / dt
    if info.rank == 0:
        roof = conv_roofline(dev, B)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(C, args.cpu_steps)
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "tiles/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": "rcan-10-20-64 train step (down4 + fwd + RMSE + interp RMSE + bwd + Adam), "
                                   f"{C}-var 48x48->192x192 tiles",
                       "global_batch": B * world, "per_gpu_batch": B, "tile": "48->192",
                       "parallelism": f"dp{world}"},
            "model_tflops": round(value * TRAIN_GFLOP_PER_TILE_C2 / 1000.0, 1),
            "loss": round(loss, 6),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if info.enabled:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
