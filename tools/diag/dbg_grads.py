"""Per-tensor gradient error of one small-model step against the fp64 oracle (the
check of tests/test_gpu_model.py test_small_model_step_vs_golden, every tensor
printed instead of stopping at the first over its bound).  Debug aid.
    python tools/dbg_grads.py [rcan|edsr]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_model as t  # noqa: E402


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "rcan"
    if arch == "rcan":
        C, nl, nb, scale, S, B, gname = 1, 2, 2, 4, 192, 2, "rcan_small_c1_f64.npz"
    else:
        C, nl, nb, scale, S, B, gname = 4, 2, 0, 8, 256, 1, "edsr_small_c4_f64.npz"
    d = t.dev()
    gd = np.load(os.path.join(t.GOLDEN, gname))
    kw = dict(nchannels_in=C, nchannels_out=C, nlayers=nl, nfeatures=64)
    model = t.ro.RCANOracle(nblocks=nb, cbottleneck=2, **kw) if arch == "rcan" else \
        t.ro.EDSROracle(downscale_factors=[2, 2, 2], **kw)
    t.ro.init_params_numpy(model, int(gd["seed_w"]))
    model = model.double()
    hr = t.ro.synthetic_hr(B, C, S, int(gd["seed_x"]))
    spec = t.spec_of(arch, C, nl, nb, scale)
    tr = t.FusedTrainer(spec, B, (S // scale, S // scale), lr=float(gd["lr"]), interp_loss=True, device=d,
                        params=t.flat_from_model(model, t._table(spec)).to(d))
    _, _, g_ref = t.oracle_grads(model, hr, scale)
    res = tr.step(torch.tensor(hr).to(d))
    torch.cuda.synchronize()
    print("loss", float(res["loss"]), "golden", float(gd["loss0"]))
    grads = tr.grads.cpu()
    bound = t.drift_bounds(model, hr, scale, g_ref)
    for name, off, n, shape in tr.eng.table:
        r = t.rel_l2(grads[off:off + n].view(shape), g_ref[name])
        print(f"{name:40s} {r:.3e} bound {bound[name]:.3e} {'FAIL' if r > bound[name] else ''}")


if __name__ == "__main__":
    main()
