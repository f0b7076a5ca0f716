"""Debug: per-tensor gradients of one small FusedTrainer step (and the plugin-module
dy path), saved for comparison across library builds (SRMI_LIB).
    python tools/debug_grads.py TAG"""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT, os.path.join(ROOT, "tests")]
from bench import synthetic_hr  # noqa: E402
from srmi.engine import Engine, NetSpec, downsample  # noqa: E402
from srmi.trainer import FusedTrainer, default_init_  # noqa: E402

d = torch.device("cuda", 0)
spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=2, nblocks=2, cbottleneck=2, scale=4)
tr = FusedTrainer(spec, 2, (48, 48), device=d, seed=0, micro=1)
hr = torch.tensor(synthetic_hr(2, 2, 192, 1234)).to(d)
tr.step(hr)
torch.cuda.synchronize()
out = {"grads": tr.grads.cpu().clone(), "sr": tr.sr.cpu().clone()}
# dy path (plugin module): backward with an explicit upstream gradient
eng = tr.eng
lr = downsample(hr, 4)
sr = eng.forward(tr.params, lr)
dy = torch.randn(sr.shape, generator=torch.Generator().manual_seed(5)).to(d) * 1e-3
g2 = torch.zeros_like(tr.grads)
eng.backward(tr.params, lr, g2, dy=dy)
torch.cuda.synchronize()
out["grads_dy"] = g2.cpu()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
torch.save(out, os.path.join(ROOT, "gpurun_out", f"dg_{sys.argv[1]}.pt"))
print("ok")
