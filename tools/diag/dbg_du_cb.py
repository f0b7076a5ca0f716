"""Diagnostic: which gradient tensors differ between the fused CA backward and the du pass
at a given CA bottleneck (python tools/diag/dbg_du_cb.py CB)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
from srmi._lib import SRMI_FLAG_DU_PASS  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer, default_init_  # noqa: E402

d = torch.device("cuda", 0)


def run(cb):
    C, nl, nb, B, h, w = 2, 2, 4, 6, 48, 48
    specs = [NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=nl, nblocks=nb, cbottleneck=cb,
                     scale=4, flags=f) for f in (0, SRMI_FLAG_DU_PASS)]
    table = param_table(specs[0])
    flat = torch.empty(sum(t[2] for t in table))
    default_init_(flat, table, seed=21)
    g = torch.Generator().manual_seed(5)
    hr = torch.randn(B, C, 4 * h, 4 * w, generator=g, dtype=torch.float64)
    trs = [FusedTrainer(sp, B, (h, w), device=d, params=flat.to(d), micro=1) for sp in specs]
    for t in trs:
        t.step(hr.float().to(d))
    torch.cuda.synchronize()
    ga, gb = trs[0].grads.cpu(), trs[1].grads.cpu()
    nd = 0
    for name, off, n, shape in table:
        a, b = ga[off:off + n], gb[off:off + n]
        if not torch.equal(a, b):
            nd += 1
            diff = (a - b).abs()
            print(f"{name}: {int((diff > 0).sum())} of {n} differ, max {float(diff.max()):.3e}, rel {float((a - b).norm() / b.norm()):.3e}")
    print("differing tensors:", nd)
    covered = torch.zeros(ga.numel(), dtype=torch.bool)
    for name, off, n, shape in table:
        covered[off:off + n] = True
    print("whole vector equal:", torch.equal(ga, gb), "elements", ga.numel(), "covered by the table", int(covered.sum()))
    bad = (ga != gb).nonzero().flatten()
    print("differing indices (first 10):", bad[:10].tolist(), "all outside the table:", bool((~covered[bad]).all()) if len(bad) else None)
    print("values there:", ga[bad[:5]].tolist(), gb[bad[:5]].tolist())


for cb in [int(x) for x in sys.argv[1:]] or [8]:
    print("== cb", cb)
    run(cb)
