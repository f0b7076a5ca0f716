"""Diagnostic: per-tensor gradient error of the fp32 (and bf16) RCAN engine against the
fp64 oracle at several CA bottlenecks, and run-to-run bit identity
(python tools/diag/dbg_f32_cb.py CB... ; CB:NL:NB:B picks the model shape and batch)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
from oracle import rcan_oracle as ro  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402

d = torch.device("cuda", 0)
for arg in sys.argv[1:]:
    cb, nl, nb, B = ([int(v) for v in arg.split(":")] + [2, 3, 2])[:4] if ":" in arg else (int(arg), 2, 3, 2)
    model = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=nl, nblocks=nb, nfeatures=64, cbottleneck=cb)
    ro.init_params_numpy(model, 9)
    hr = ro.synthetic_hr(B, 2, 192, 13)
    md = model.double()
    h = torch.tensor(hr, dtype=torch.float64)
    md.zero_grad()
    ro.l2loss(md(ro.downsample(h, 4)), h).backward()
    g = {n: p.grad for n, p in md.named_parameters()}
    for dt in ("fp32",):
        spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=nl, nblocks=nb,
                       cbottleneck=cb, scale=4, dtype=dt)
        table = param_table(spec)
        flat = torch.cat([dict(md.named_parameters())[n].detach().float().reshape(-1) for n, _, _, _ in table])
        runs = []
        for rep in range(2):
            tr = FusedTrainer(spec, B, (48, 48), device=d, params=flat.to(d), micro=1)
            tr.step(torch.tensor(hr, device=d))
            torch.cuda.synchronize()
            runs.append(tr.grads.cpu().clone())
            del tr
        errs = []
        for name, off, n, shape in table:
            e = float((runs[0][off:off + n].view(shape).double() - g[name]).norm() / g[name].norm())
            errs.append((e, name))
        errs.sort(reverse=True)
        print(arg, dt, "identical" if torch.equal(runs[0], runs[1]) else "DIFFER", errs[:4], flush=True)
