"""Diagnostic driver for PMC passes: the 64-channel conv kernel (epilogues 0, 1, 4) at
the C2 shape, a few launches each (tools/pmc_lds.sh)."""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
from srmi._lib import call, ptr  # noqa: E402

d = torch.device("cuda", 0)
N, H, W = 64, 48, 48
S = torch.cuda.current_stream().cuda_stream
x = torch.randn(N, H, W, 64, device=d).to(torch.bfloat16)
t = torch.randn(N, H, W, 64, device=d).clamp_min(0).to(torch.bfloat16)
w = torch.randn(64, 64, 3, 3, device=d) * 0.05
b = torch.zeros(64, device=d)
fp = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=d)
dp = torch.empty_like(fp)
pb = torch.empty(64, device=d)
call("srmi_pack_conv", ptr(w), ptr(b), 64, 64, 0, ptr(fp), ptr(dp), ptr(pb), 0, S)
yb = torch.empty_like(x)
ns = call("srmi_conv3x3_nstrips", H, W)
part = torch.zeros(N, ns, 128, device=d)
for _ in range(5):
    call("srmi_conv3x3", ptr(x), ptr(fp), ptr(pb), N, H, W, 64, 64, 0, 0, ptr(yb), None, None, None, None, None, None,
         1.0, 0, S)
    call("srmi_conv3x3", ptr(x), ptr(dp), None, N, H, W, 64, 64, 0, 4, ptr(yb), None, None, None, None, ptr(t), None,
         1.0, 0, S)
torch.cuda.synchronize()
print("done")
