"""Diagnostic: compare the saved forward state (u maps, CA records) of two engine
variants / micro-batch splits from the engine workspaces (carve order of engine.cpp)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
import torch  # noqa: E402
from oracle import rcan_oracle as ro  # noqa: E402
from srmi._lib import SRMI_FLAG_CA_PASS  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer, default_init_  # noqa: E402

NL, NB, B = 2, 3, 16


def views(eng):
    ws = eng.workspace
    base = (ws.data_ptr() + 255) & ~255
    off = [base - ws.data_ptr()]
    n = eng.batch
    m = n * 48 * 48 * 64

    def take(nbytes):
        o = (off[0] + 255) & ~255
        off[0] = o + nbytes
        return o
    take(m * 4); take(m * 4); take(m * 4)
    nhb = NL * (NB + 1) + 1
    hb_off = take(m * 2 * nhb)
    t_off = take(m * 2 * NL * NB)
    u_off = take(m * 2 * NL * NB)
    res_off = take(m * 2)
    ps0_off = take((m << 2) * 2); ps1_off = take((m << 4) * 2)
    rec_off = take(NL * NB * n * 160 * 4)
    global EXTRA
    EXTRA = {"hb": ws[hb_off:hb_off + m * 2 * nhb].view(torch.bfloat16).view(nhb, n, -1),
             "res": ws[res_off:res_off + m * 2].view(torch.bfloat16).view(1, n, -1),
             "ps0": ws[ps0_off:ps0_off + (m << 2) * 2].view(torch.bfloat16).view(1, n, -1),
             "ps1": ws[ps1_off:ps1_off + (m << 4) * 2].view(torch.bfloat16).view(1, n, -1)}
    u = ws[u_off:u_off + m * 2 * NL * NB].view(torch.bfloat16).view(NL * NB, n, 48, 48, 64)
    t = ws[t_off:t_off + m * 2 * NL * NB].view(torch.bfloat16).view(NL * NB, n, 48, 48, 64)
    rec = ws[rec_off:rec_off + NL * NB * n * 160 * 4].view(torch.float32).view(NL * NB, n, 160)
    return t, u, rec


d = torch.device("cuda", 0)
hr = torch.tensor(ro.synthetic_hr(B, 2, 192, 17)).to(d)
out = {}
for flags in (0, SRMI_FLAG_CA_PASS):
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=NL, nblocks=NB, flags=flags)
    table = param_table(spec)
    flat = torch.empty(sum(x[2] for x in table), device=d)
    default_init_(flat, table, seed=5)
    for micro in (1, 2):
        tr = FusedTrainer(spec, B, (48, 48), device=d, params=flat, micro=micro)
        tr.step(hr)
        torch.cuda.synchronize()
        parts, extras = [], []
        for e in tr.engines:
            parts.append(views(e))
            extras.append({k: v.clone() for k, v in EXTRA.items()})
        ex = {k: torch.cat([x[k] for x in extras], 1) for k in extras[0]}
        t = torch.cat([p[0] for p in parts], 1).clone()
        u = torch.cat([p[1] for p in parts], 1).clone()
        rec = torch.cat([p[2] for p in parts], 1).clone()
        out[(flags, micro)] = (t, u, rec, tr.grads.clone(), ex)
        del tr
for a, b in (((0, 1), (0, 2)), ((4, 1), (4, 2)), ((0, 1), (4, 1))):
    ta, ua, ra, ga, ea = out[a]
    tb, ub, rb, gb, eb = out[b]
    for k in ea:
        if not torch.equal(ea[k], eb[k]):
            dd = (ea[k].float() - eb[k].float()).abs()
            print("   ", k, "differs: max", float(dd.max()), "count", int((dd > 0).sum()), "per slot/image",
                  dd.amax(dim=2).cpu().numpy().round(4).tolist()[:12])
        else:
            print("   ", k, "equal")
    print(a, b, "t equal", torch.equal(ta, tb), "u equal", torch.equal(ua, ub),
          "u maxdiff", float((ua.float() - ub.float()).abs().max()),
          "rec m/z1/s maxdiff", [float((ra[..., sl] - rb[..., sl]).abs().max()) for sl in
                                 (slice(0, 64), slice(64, 96), slice(96, 160))],
          "grad rel", float((ga - gb).norm() / gb.norm()), flush=True)
    if not torch.equal(ua, ub):
        diff = (ua.float() - ub.float()).abs().amax(dim=(2, 3, 4))
        print("   u diff per (rcab, image):", diff.cpu().numpy().round(4).tolist())
