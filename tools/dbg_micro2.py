"""Diagnostic: per-tensor micro=1 vs micro=2 gradient differences (fused CA forward)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
import torch  # noqa: E402
from oracle import rcan_oracle as ro  # noqa: E402
from srmi._lib import SRMI_FLAG_CA_PASS  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer, default_init_  # noqa: E402

d = torch.device("cuda", 0)
hr = torch.tensor(ro.synthetic_hr(16, 2, 192, 17)).to(d)
for flags in (0, SRMI_FLAG_CA_PASS):
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=2, nblocks=3, flags=flags)
    table = param_table(spec)
    flat = torch.empty(sum(x[2] for x in table), device=d)
    default_init_(flat, table, seed=5)
    g = []
    for micro in (1, 2):
        tr = FusedTrainer(spec, 16, (48, 48), device=d, params=flat, micro=micro)
        tr.step(hr)
        torch.cuda.synchronize()
        g.append(tr.grads.clone())
        del tr
    print("flags", flags, flush=True)
    for name, off, n, shape in table:
        a, b = g[0][off:off + n], g[1][off:off + n]
        print(f"  {name:40s} rel {float((a - b).norm() / b.norm()):.3e}  norm {float(b.norm()):.3e}")
