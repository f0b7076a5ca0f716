"""Times the upsampler's Cin=256 unshuffle dgrad (generic conv3x3_kernel) at the C2 in-step shapes.

    python tools/kbench_unshuf.py [--batch 32] [--iters 30]      (SRMI_LIB selects a build)

96x96 (second upsampler stage, EPI_PLAIN -> bf16) and 48x48 (first stage, EPI_DG_ACC into the
fp32 gradient stream), one engine's B=32 launch, HIP events on the launch stream.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]

import torch  # noqa: E402

from srmi._lib import call, ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    S = lambda: torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(0)
    w = (torch.randn(256, 64, 3, 3, generator=g) * 0.05).to(d)
    b = torch.zeros(256, device=d)
    fp = torch.empty(256 * 64 * 9, dtype=torch.bfloat16, device=d)
    dp = torch.empty_like(fp)
    pb = torch.empty(256, device=d)
    call("srmi_pack_conv", ptr(w), ptr(b), 256, 64, 1, ptr(fp), ptr(dp), ptr(pb), 0, S())
    res = {}
    for H, epi in ((96, 6), (48, 5)):
        N = a.batch
        dyp = torch.randn(N, 2 * H, 2 * H, 64, generator=g).to(d).to(torch.bfloat16)
        yb = torch.empty(N, H, H, 64, dtype=torch.bfloat16, device=d)
        yf = torch.zeros(N, H, H, 64, device=d)
        def f():
            if epi == 6:
                call("srmi_conv3x3", ptr(dyp), ptr(dp), None, N, H, H, 256, 64, 1, 6, ptr(yb), None, None, None,
                     None, None, None, 1.0, 0, S())
            else:
                call("srmi_conv3x3", ptr(dyp), ptr(dp), None, N, H, H, 256, 64, 1, 5, ptr(yb), ptr(yf), ptr(yf),
                     None, None, None, None, 1.0, 0, S())
        for _ in range(3):
            f()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.iters):
            f()
        e1.record(st)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / a.iters
        flop = 2.0 * N * H * H * 64 * 256 * 9
        res[f"unshuf_dgrad_{H}"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
