"""Launch the bench's roofline kernels in isolation (for rocprofv3 --pmc passes).

    python tools/roofline_driver.py [--batch 64] [--iters 20]

wgrad3x3 (slab-only: the MFMA kernel without its reduction) and the 64->64 conv
with the fused bias+ReLU epilogue, both at BASELINE config 2 shapes (B tiles of
48x48x64, bf16).  Inputs are re-used across launches, as in a training step
where x and dY were just produced.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]

import torch  # noqa: E402

from srmi._lib import call, ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    N, H, W = a.batch, 48, 48
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(N, H, W, 64, generator=g).to(d).to(torch.bfloat16)
    dy = torch.randn(N, H, W, 64, generator=g).to(d).to(torch.bfloat16)
    slab = torch.empty(N * 12 * 64 * 577 + 64, dtype=torch.float32, device=d)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(d)
    b = torch.zeros(64, device=d)
    fp = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=d)
    dp = torch.empty_like(fp)
    pb = torch.empty(64, device=d)
    call("srmi_pack_conv", ptr(w), ptr(b), 64, 64, 0, ptr(fp), ptr(dp), ptr(pb), 0, st)
    y = torch.empty_like(x)
    for _ in range(a.iters):
        call("srmi_wgrad3x3", ptr(x), ptr(dy), N, H, W, 64, 0, 0, ptr(slab), slab.numel() * 4, 0, 1.0, None, None,
             0, st)
    for _ in range(a.iters):
        call("srmi_conv3x3", ptr(x), ptr(fp), ptr(pb), N, H, W, 64, 64, 0, 0, ptr(y), None, None, None, None, None,
             None, 1.0, 0, st)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
