"""Debug: forward outputs of one engine configuration saved for comparison across
library builds (SRMI_LIB).   python tools/debug_ca.py TAG B NL NB CU"""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "super-resolution-climate_amd"))
from srmi.engine import Engine, NetSpec  # noqa: E402
from srmi.trainer import default_init_  # noqa: E402

tag, B, NL, NB, CU = sys.argv[1], *map(int, sys.argv[2:6])
dev = torch.device("cuda", 0)
spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=NL, nblocks=NB, cbottleneck=2,
               scale=4)
eng = Engine(spec, B, (48, 48), train=True, device=dev, cu_budget=CU)
p = torch.empty(eng.n_params, device=dev)
default_init_(p, eng.table, 0)
eng.pack(p)
lr = torch.randn(B, 2, 48, 48, generator=torch.Generator().manual_seed(3)).to(dev)
out = eng.forward(p, lr)
torch.cuda.synchronize()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
torch.save(out.cpu(), os.path.join(ROOT, "gpurun_out", f"dbg_{tag}.pt"))
print(tag, float(out.double().norm()))
