"""Parity at the headline configurations themselves (BASELINE configs 2 and 5), not
scaled-down stand-ins:

* C2: FusedTrainer(B=64, micro=2) on rcan-10-20-64, 2-var 48->192 tiles -- the
  bench's exact shape (two micro-batch engines on two streams, side streams, the
  ring of 4 DU/DZ buffers) -- one step against the oracle run on the GPU in fp32
  with the same weights and inputs.  Tolerances: loss rel <= 1e-3 (north-star),
  output rel-L2 <= 2e-2 (SURVEY.md §8(c) bf16 output drift), and per parameter
  tensor a gradient bound DERIVED in the test from the reference's own bf16
  drift: the oracle with bf16-rounded conv operands (tests/gpu_oracle.py, the
  engine's precision model) is run on the same step, and the engine's rel-L2
  distance from the fp32 gradient must stay within 3x that drift (+1e-3).
* the fp64 golden's gradient SAMPLES of rcan-10-20-64 at B=1
  (tests/golden/rcan_full_c2_f64.npz, made from the imported reference).
* C5: TiledInference over a 4096^2 region with rcan-10-20-64 (441 tiles, HIP
  graph on) against oracle.process_region on the GPU in fp32.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gpu_oracle import bf16_operand_emulation, conv_params, exact_fp32  # noqa: E402
from oracle import rcan_oracle as ro  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
# fixed per-tensor gradient rel-L2 bars vs the fp32 oracle at C2, independent of the
# emulation (bf16 drift ~2e-2): every conv tensor within 2e-2; the CA
# bottleneck MLP's tensors (64 -> 2 -> 64, conv_du.*: a few ReLU units whose gradient
# sums cancel) within 1e-1 -- the emulated-bf16 oracle alone drifts 5.4e-2 there
# (profiles/r06_c2_parity.json); the whole gradient vector within 1e-2
GRAD_CAP_C2 = 2e-2
GRAD_CAP_C2_CA = 1e-1


def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def rel_l2(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double().to(a.device)
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _full_spec(C):
    return NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)


def _oracle(C, seed, d):
    m = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=10, nblocks=20, nfeatures=64, cbottleneck=2)
    ro.init_params_numpy(m, seed)
    return m.to(d)


def _flat(params_by_name, table):
    return torch.cat([params_by_name[n].detach().reshape(-1).float() for n, _, _, _ in table])


def _oracle_step(model, hr):
    """loss, output and gradients of one reference step (dual_trainer.py:310-322)."""
    model.zero_grad(set_to_none=True)
    lr_in = ro.downsample(hr, 4)
    out = model(lr_in)
    loss = ro.l2loss(out, hr)
    loss.backward()
    g = {n: p.grad.detach().clone() for n, p in conv_params(model).items()}
    return float(loss), out.detach(), g


@pytest.mark.timeout(900)
def test_c2_full_shape_step_vs_fp32_oracle():
    d = dev()
    C, B = 2, 64
    spec = _full_spec(C)
    table = param_table(spec)
    hr = torch.tensor(ro.synthetic_hr(B, C, 192, 1234), device=d)
    with exact_fp32():
        model = _oracle(C, 0, d)
        flat = _flat(dict(model.named_parameters()), table)
        l32, out32, g32 = _oracle_step(model, hr)
        emul = bf16_operand_emulation(_oracle(C, 0, d))
        le, oute, ge = _oracle_step(emul, hr)
        del model, emul
    torch.cuda.empty_cache()
    out32_sub = out32[:, :, ::2, ::2].clone()
    oute_sub = oute[:, :, ::2, ::2].clone()
    del out32, oute
    tr = FusedTrainer(spec, B, (48, 48), lr=1e-4, device=d, params=flat, micro=2)
    assert tr.micro == 2 and tr.engines[0].batch == 32
    res = tr.step(hr)
    torch.cuda.synchronize()
    loss = float(res["loss"])
    assert abs(loss - l32) / l32 < 1e-3, (loss, l32)
    assert rel_l2(tr.sr[:, :, ::2, ::2], out32_sub) < 2e-2
    grads = tr.grads
    worst, report = 0.0, []
    for name, off, n, shape in table:
        e_eng = rel_l2(grads[off:off + n].view(shape), g32[name])
        e_emu = rel_l2(ge[name], g32[name])
        bound = 3.0 * e_emu + 1e-3
        report.append((name, e_eng, e_emu))
        worst = max(worst, e_eng / bound)
    report.sort(key=lambda r: -r[1] / (3.0 * r[2] + 1e-3))
    print("\nC2 grads: emulated-bf16 drift vs engine (worst 5):", report[:5])
    out_rel, emu_out_rel = rel_l2(tr.sr[:, :, ::2, ::2], out32_sub), rel_l2(oute_sub, out32_sub)
    print(f"C2 loss: engine {loss:.7f} fp32 {l32:.7f} emulated {le:.7f}; output rel-L2 "
          f"{out_rel:.3e} (emulated {emu_out_rel:.3e})")
    g_all = torch.cat([g32[name].reshape(-1) for name, _, _, _ in table])
    whole = rel_l2(grads, g_all)
    path = os.environ.get("SRMI_PARITY_REPORT")
    if path:  # the committed per-tensor report (profiles/rNN_c2_parity.json)
        import json
        eng = np.array([r[1] for r in report])
        json.dump({"config": "C2: rcan-10-20-64, 2-var, B=64, micro=2, one step from the same weights and tiles",
                   "reference": "oracle/rcan_oracle.py in exact fp32 on the GPU (TF32 off)",
                   "emulation": "tests/gpu_oracle.py: the oracle with the engine's bf16 operands, pair stream, bf16 u",
                   "loss": {"engine": loss, "fp32": l32, "emulated": le, "rel": abs(loss - l32) / l32},
                   "output_rel_l2": {"engine": out_rel, "emulated": emu_out_rel},
                   "grad_rel_l2_whole_vector": whole,
                   "grad_rel_l2_caps": {"conv": GRAD_CAP_C2, "ca_mlp": GRAD_CAP_C2_CA, "whole": 1e-2},
                   "grad_rel_l2_per_tensor": {"max": float(eng.max()), "median": float(np.median(eng)),
                                              "p90": float(np.percentile(eng, 90))},
                   "tensors": [{"name": n_, "engine_vs_fp32": a_, "emulated_vs_fp32": b_, "bound": 3 * b_ + 1e-3}
                               for n_, a_, b_ in report]}, open(path, "w"), indent=1)
    assert worst <= 1.0, report[:5]
    # a fixed bar as well (bf16 drift ~2e-2 element-wise): the bound above
    # follows the emulation, this one does not move with the engine's precision model
    assert max(r[1] for r in report if "conv_du" not in r[0]) <= GRAD_CAP_C2, report[:5]
    assert max(r[1] for r in report if "conv_du" in r[0]) <= GRAD_CAP_C2_CA, report[:5]
    assert whole <= 1e-2, whole


def test_full_rcan_grad_samples_vs_golden_b1():
    """rcan-10-20-64, one tile: the engine's gradient at the golden's sample indices
    (48 per tensor) against the fp64 reference, and the per-tensor norms."""
    d = dev()
    gd = np.load(os.path.join(GOLDEN, "rcan_full_c2_f64.npz"))
    spec = _full_spec(2)
    table = param_table(spec)
    m = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20, nfeatures=64, cbottleneck=2)
    ro.init_params_numpy(m, int(gd["seed_w"]))
    flat = _flat(dict(m.named_parameters()), table).to(d)
    tr = FusedTrainer(spec, 1, (48, 48), lr=float(gd["lr"]), device=d, params=flat)
    hr = torch.tensor(ro.synthetic_hr(1, 2, 192, int(gd["seed_x"])), device=d)
    tr.step(hr)
    torch.cuda.synchronize()
    g = tr.grads.double().cpu().numpy()
    samples, off_s = [], 0
    for name, off, n, shape in table:
        idx = np.unique(np.linspace(0, n - 1, min(n, 48)).astype(np.int64))
        samples.append(g[off + idx])
    eng = np.concatenate(samples)
    ref = gd["grad_sample"]
    assert eng.shape == ref.shape
    # all samples together: the bf16 element drift of SURVEY.md §8(c)
    r_all = np.linalg.norm(eng - ref) / np.linalg.norm(ref)
    print(f"\ngrad samples rel-L2 {r_all:.3e}")
    assert r_all < 3e-2
    # per tensor: 48 samples each; medians tight, the worst tensors (CA bottleneck
    # ReLU flips at one tile, see test_gpu_model) allowed a loose bound
    per, k = [], 0
    for name, off, n, shape in table:
        m_ = min(n, 48)
        idx = np.unique(np.linspace(0, n - 1, m_).astype(np.int64)).size
        a, b = eng[k:k + idx], ref[k:k + idx]
        per.append(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
        k += idx
    per = np.array(per)
    assert np.median(per) < 2e-2, np.median(per)
    assert np.mean(per < 8e-2) > 0.97


@pytest.mark.timeout(900)
def test_c5_full_region_vs_fp32_oracle():
    from srmi.inference import TiledInference
    d = dev()
    spec = _full_spec(1)
    table = param_table(spec)
    with exact_fp32():
        model = _oracle(1, 5, d)
        flat = _flat(dict(model.named_parameters()), table)
        region = torch.tensor(ro.synthetic_hr(1, 1, 4096, 99)[0], device=d) * 2.0 + 0.5
        tiles, mean, std, ids, grid = ro.region_to_tiles(region.double().cpu().numpy(), 192, 192)
        assert grid == (21, 21) and len(ids) == 441
        target = torch.tensor(tiles, dtype=torch.float32, device=d)
        lr_in = ro.downsample(target, 4)
        with torch.no_grad():
            sr_ref = model(lr_in)
        interp_ref = ro.upsample(lr_in, 4)
        bm = ro.batch_losses(sr_ref, target, 36)
        bi = ro.batch_losses(interp_ref, target, 36)
        del model
    ti = TiledInference(spec, flat, tuple(region.shape), (192, 192), device=d, graph=True, batch_size=36)
    assert ti.n == 441
    images, losses = ti.process_region(region)
    torch.cuda.synchronize()
    img_model = images["model"].clone()
    ref_model = torch.tensor(ro.assemble(sr_ref.double().cpu().numpy(), mean, std, ids, grid), device=d)
    ref_interp = torch.tensor(ro.assemble(interp_ref.double().cpu().numpy(), mean, std, ids, grid), device=d)
    assert rel_l2(images["target"], region[:, :4032, :4032]) < 1e-6
    assert rel_l2(images["interpolated"], ref_interp) < 1e-5
    assert rel_l2(img_model, ref_model) < 2e-2
    assert abs(float(losses["interpolated"]) - np.mean(bi)) < 1e-5 * np.mean(bi)
    assert abs(float(losses["model"]) - np.mean(bm)) < 1e-3 * np.mean(bm)
    b = ti.batch_losses()
    assert b["model"].numel() == 13
    np.testing.assert_allclose(b["interpolated"].cpu().numpy(), bi, rtol=1e-5)
    np.testing.assert_allclose(b["model"].cpu().numpy(), bm, rtol=2e-3)
    # replaying the captured graph on the same region is bit-stable
    ti.replay()
    torch.cuda.synchronize()
    assert torch.equal(images["model"], img_model)
