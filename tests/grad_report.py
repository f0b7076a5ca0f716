"""Dev tool: per-tensor gradient deviation of the engine vs the fp64 golden / oracle (full rcan-10-20-64, 1 tile)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
from oracle import rcan_oracle as ro
from srmi.engine import NetSpec, param_table
from srmi.trainer import FusedTrainer

d = torch.device("cuda", 0)
gd = np.load(os.path.join(ROOT, "tests", "golden", "rcan_full_c2_f64.npz"))
model = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20)
ro.init_params_numpy(model, int(gd["seed_w"]))
spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20)
table = param_table(spec)
sd = dict(model.named_parameters())
flat = torch.cat([sd[n].detach().reshape(-1) for n, _, _, _ in table]).float()
tr = FusedTrainer(spec, 1, (48, 48), lr=1e-4, device=d, params=flat.to(d))
hr_np = ro.synthetic_hr(1, 2, 192, int(gd["seed_x"]))
tr.step(torch.tensor(hr_np).to(d)); torch.cuda.synchronize()
g = tr.grads.cpu()
# fp64 oracle grads on CPU
m64 = model.double(); m64.zero_grad()
h = torch.tensor(hr_np, dtype=torch.float64, requires_grad=True)
loss = ro.l2loss(m64(ro.downsample(h, 4)), h); loss.backward()
rows = []
for i, (n, off, k, shp) in enumerate(table):
    ref = sd[n].grad.double().reshape(-1)
    mine = g[off:off + k].double()
    rel = float((mine - ref).norm() / ref.norm())
    rows.append((rel, float(mine.norm() / ref.norm()), n, float(ref.norm())))
rows.sort(reverse=True)
print("loss", float(loss), "engine", float(tr.loss4[3]))
for r in rows[:40]:
    print(f"relL2 {r[0]:.3e} ratio {r[1]:.4f} |g|={r[3]:.3e} {r[2]}")
fam = {}
for r in rows:
    key = r[2].split(".")[-2] if "conv_du" not in r[2] else "ca." + r[2].split(".")[-2] + "." + r[2].split(".")[-1]
    key = ("w" if r[2].endswith("weight") else "b") + ":" + key
    fam.setdefault(key, []).append(r[0])
for k, v in sorted(fam.items()):
    print(f"{k:20s} n={len(v):4d} median relL2 {np.median(v):.3e} max {np.max(v):.3e}")
