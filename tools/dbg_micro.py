"""Diagnostic: micro=1 vs micro=2 gradient agreement per engine variant (flags)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
import torch  # noqa: E402
from oracle import rcan_oracle as ro  # noqa: E402
from srmi._lib import SRMI_FLAG_CA_PASS, SRMI_FLAG_WGRAD_FULL_CO  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer, default_init_  # noqa: E402

d = torch.device("cuda", 0)
for flags in (0, SRMI_FLAG_WGRAD_FULL_CO, SRMI_FLAG_CA_PASS, SRMI_FLAG_WGRAD_FULL_CO | SRMI_FLAG_CA_PASS):
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=2, nblocks=3, flags=flags)
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=5)
    hr = torch.tensor(ro.synthetic_hr(16, 2, 192, 17)).to(d)
    res = []
    for micro in (1, 2, 1):
        tr = FusedTrainer(spec, 16, (48, 48), device=d, params=flat, micro=micro)
        out = tr.step(hr)
        res.append((float(out["loss"]), tr.grads.clone(), tr.sr.clone()))
        del tr
    g1, g2, g3 = res[0][1], res[1][1], res[2][1]
    rl = lambda a, b: float((a - b).double().norm() / b.double().norm())
    worst = []
    for name, off, n, shape in table:
        worst.append((rl(g2[off:off + n], g1[off:off + n]), name))
    worst.sort(reverse=True)
    print(flags, "loss", res[0][0], res[1][0], "sr equal", torch.equal(res[0][2], res[1][2]), "rerun equal",
          torch.equal(g1, g3), "grad rel", rl(g2, g1), worst[:3], flush=True)
