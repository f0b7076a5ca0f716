"""Model-level parity of the HIP engine against the oracle and the golden vectors
generated from the reference (tests/golden/make_golden.py).

Tolerances: the engine computes conv operands in bf16 with
fp32 accumulation and a 16-bit pair residual stream inside each residual group
(emulated by tests/gpu_oracle.py), so element-wise outputs are
compared by relative L2 (<= 2e-2), the loss within 2e-3 relative (the
north-star "results within 1e-3 rel" is met for the loss at full size, see
test_full_rcan_loss_parity), gradients by relative L2 per tensor family.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import rcan_oracle as ro  # noqa: E402
from srmi.engine import Engine, NetSpec  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def flat_from_model(model, table):
    sd = dict(model.named_parameters())
    flat = torch.empty(sum(t[2] for t in table), dtype=torch.float32)
    for name, off, n, shape in table:
        flat[off:off + n] = sd[name].detach().float().reshape(-1)
    return flat


def spec_of(arch, C, nl, nb=0, scale=4, rs=1.0, cb=2):
    return NetSpec(arch=arch, nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=nl, nblocks=nb, cbottleneck=cb,
                   scale=scale, res_scale=rs)


def oracle_grads(model, hr, scale):
    model.zero_grad()
    h = torch.tensor(hr, dtype=torch.float64, requires_grad=True)
    out = model(ro.downsample(h, scale))
    loss = ro.l2loss(out, h)
    loss.backward()
    return float(loss), out.detach(), {conv_key(n): p.grad.detach().clone() for n, p in model.named_parameters()}


def conv_key(n):
    return n.replace(".conv.", ".")


def drift_bounds(model, hr, scale, g_ref):
    """Per-tensor gradient bounds DERIVED from the reference's own bf16 drift
    (SURVEY.md §8(c)): the same fp64 oracle step with bf16-rounded conv operands
    (tests/gpu_oracle.py, the engine's precision model); the engine may sit at
    most 3x that drift (+1e-3) from the exact gradient."""
    import copy
    from gpu_oracle import bf16_operand_emulation
    emul = bf16_operand_emulation(copy.deepcopy(model))
    _, _, g_emu = oracle_grads(emul, hr, scale)
    return {n: 3.0 * rel_l2(g_emu[n], g_ref[n]) + 1e-3 for n in g_ref}


@pytest.mark.parametrize("arch,C,nl,nb,scale,S,B,gname", [
    ("rcan", 1, 2, 2, 4, 192, 2, "rcan_small_c1_f64.npz"),
    ("rcan", 2, 2, 2, 4, 192, 2, "rcan_small_c2_f64.npz"),
    ("edsr", 4, 2, 0, 8, 256, 1, "edsr_small_c4_f64.npz"),
])
def test_small_model_step_vs_golden(arch, C, nl, nb, scale, S, B, gname):
    d = dev()
    gd = np.load(os.path.join(GOLDEN, gname))
    kw = dict(nchannels_in=C, nchannels_out=C, nlayers=nl, nfeatures=64)
    if arch == "rcan":
        model = ro.RCANOracle(nblocks=nb, cbottleneck=2, **kw)
    else:
        model = ro.EDSROracle(downscale_factors=[2, 2, 2], **kw)
    ro.init_params_numpy(model, int(gd["seed_w"]))
    model = model.double()
    hr = ro.synthetic_hr(B, C, S, int(gd["seed_x"]))
    spec = spec_of(arch, C, nl, nb, scale)
    tr = FusedTrainer(spec, B, (S // scale, S // scale), lr=float(gd["lr"]), interp_loss=True, device=d,
                      params=flat_from_model(model, _table(spec)).to(d))
    # oracle reference gradients (fp64, same weights)
    l_ref, out_ref, g_ref = oracle_grads(model, hr, scale)
    assert abs(l_ref - float(gd["loss0"])) < 1e-10  # oracle pinned to the reference
    hr_d = torch.tensor(hr).to(d)
    res = tr.step(hr_d)
    torch.cuda.synchronize()
    loss0 = float(res["loss"])
    iloss0 = float(res["interp_loss"])
    assert abs(loss0 - float(gd["loss0"])) / float(gd["loss0"]) < 2e-3, (loss0, float(gd["loss0"]))
    assert abs(iloss0 - float(gd["iloss0"])) / float(gd["iloss0"]) < 1e-5
    # SR output of that forward
    assert rel_l2(tr.sr[:B].cpu()[:, :, ::4, ::4], gd["out_sub"]) < 2e-2
    # gradients, per tensor, within the bound derived from the bf16-operand drift
    grads = tr.grads.cpu()
    bound = drift_bounds(model, hr, scale, g_ref)
    for name, off, n, shape in tr.eng.table:
        r = rel_l2(grads[off:off + n].view(shape), g_ref[name])
        assert r <= bound[name], (name, r, bound[name])
    gl2 = np.array([float(grads[off:off + n].norm()) for _, off, n, _ in tr.eng.table])
    rtol = np.array([bound[nm] for nm, _, _, _ in tr.eng.table])
    assert np.all(np.abs(gl2 - gd["grad_l2"]) <= rtol * np.abs(gd["grad_l2"]))
    # second step: loss after one Adam update
    res = tr.step(hr_d)
    torch.cuda.synchronize()
    loss1 = float(res["loss"])
    assert abs(loss1 - float(gd["loss1"])) / float(gd["loss1"]) < 2e-3, (loss1, float(gd["loss1"]))


@pytest.mark.parametrize("factors,lr,C", [([2], 48, 2), ([2, 2, 2], 32, 2), ([2, 2], 48, 3), ([2, 2], 32, 4)])
def test_rcan_other_scales_vs_oracle(factors, lr, C):
    """RCAN at downscale_factors [2] and [2, 2, 2] (the headline is [2, 2]: one and three
    pixel-shuffle stages in the upsampler, sres/model/common/common.py Upsampler), and at
    x4 with 3 and 4 variables (the goldens hold 1 and 2), against the fp64 oracle on the
    same weights and tiles (no golden file: the oracle itself is pinned by the goldens
    above): loss and every gradient tensor within the bf16 drift bounds."""
    d = dev()
    scale, nl, nb, B = int(np.prod(factors)), 2, 2, 2
    model = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=nl, nblocks=nb, nfeatures=64, cbottleneck=2,
                          downscale_factors=factors)
    ro.init_params_numpy(model, 3)
    model = model.double()
    hr = ro.synthetic_hr(B, C, lr * scale, 11)
    spec = spec_of("rcan", C, nl, nb, scale)
    tr = FusedTrainer(spec, B, (lr, lr), device=d, params=flat_from_model(model, _table(spec)).to(d))
    l_ref, _, g_ref = oracle_grads(model, hr, scale)
    res = tr.step(torch.tensor(hr).to(d))
    torch.cuda.synchronize()
    assert abs(float(res["loss"]) - l_ref) / l_ref < 2e-3, (float(res["loss"]), l_ref)
    grads = tr.grads.cpu()
    bound = drift_bounds(model, hr, scale, g_ref)
    for name, off, n, shape in tr.eng.table:
        r = rel_l2(grads[off:off + n].view(shape), g_ref[name])
        assert r <= bound[name], (name, r, bound[name])


def _table(spec):
    from srmi.engine import param_table
    return param_table(spec)


def test_full_rcan_forward_vs_golden():
    """rcan-10-20-64, 2-var, one tile: output and loss vs the reference (fp64 golden)."""
    d = dev()
    gd = np.load(os.path.join(GOLDEN, "rcan_full_c2_f64.npz"))
    model = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20, nfeatures=64, cbottleneck=2)
    ro.init_params_numpy(model, int(gd["seed_w"]))
    spec = spec_of("rcan", 2, 10, 20)
    table = _table(spec)
    flat = flat_from_model(model, table).to(d)
    eng = Engine(spec, 1, (48, 48), train=False, device=d)
    eng.pack(flat)
    hr = torch.tensor(ro.synthetic_hr(1, 2, 192, int(gd["seed_x"]))).to(d)
    from srmi.engine import downsample
    lr = downsample(hr, 4)
    out = eng.forward(flat, lr)
    torch.cuda.synchronize()
    assert rel_l2(out.cpu()[:, :, ::4, ::4], gd["out_sub"]) < 2e-2
    loss = float(((out - hr) ** 2).mean().sqrt())
    assert abs(loss - float(gd["loss0"])) / float(gd["loss0"]) < 1e-3


def test_full_rcan_loss_parity_and_grads():
    """rcan-10-20-64 train step at one tile vs the fp64 golden: loss within 1e-3 rel,
    gradient norms per tensor within 10 %."""
    d = dev()
    gd = np.load(os.path.join(GOLDEN, "rcan_full_c2_f64.npz"))
    model = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20, nfeatures=64, cbottleneck=2)
    ro.init_params_numpy(model, int(gd["seed_w"]))
    spec = spec_of("rcan", 2, 10, 20)
    table = _table(spec)
    tr = FusedTrainer(spec, 1, (48, 48), lr=float(gd["lr"]), device=d, params=flat_from_model(model, table).to(d))
    hr = torch.tensor(ro.synthetic_hr(1, 2, 192, int(gd["seed_x"]))).to(d)
    res = tr.step(hr)
    torch.cuda.synchronize()
    assert abs(float(res["loss"]) - float(gd["loss0"])) / float(gd["loss0"]) < 1e-3
    grads = tr.grads.cpu()
    gl2 = np.array([float(grads[off:off + n].norm()) for _, off, n, _ in table])
    ratio = gl2 / gd["grad_l2"]
    # CA bottleneck (conv_du.0) grads hinge on 32 per-tile ReLU decisions of the pooled
    # pre-activation; with ONE tile a channel sitting at ~0 flips under bf16 activation
    # noise (weight and bias rows then move by the same ratio).  Everything else: 10 %.
    ca0 = np.array([".conv_du.0." in n for n, _, _, _ in table])
    assert np.all(np.abs(ratio[~ca0] - 1) < 0.1), (ratio[~ca0].min(), ratio[~ca0].max())
    assert np.mean(np.abs(ratio[ca0] - 1) < 0.1) > 0.97
    assert np.median(np.abs(ratio - 1)) < 0.01


def test_batch_invariance_and_determinism():
    """Full-size property checks at B=64 (BASELINE config 2): a tile's output does not
    depend on its batch mates, and a train step is bitwise reproducible."""
    d = dev()
    spec = spec_of("rcan", 2, 10, 20)
    table = _table(spec)
    from srmi.trainer import default_init_
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=3)
    hr = torch.tensor(ro.synthetic_hr(64, 2, 192, 99)).to(d)
    from srmi.engine import downsample
    lr = downsample(hr, 4)
    e64 = Engine(spec, 64, (48, 48), train=False, device=d)
    e64.pack(flat)
    o64 = e64.forward(flat, lr)
    e2 = Engine(spec, 2, (48, 48), train=False, device=d)
    e2.pack(flat)
    o2 = e2.forward(flat, lr[5:7].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(o64[5:7], o2)
    del e64, e2
    losses = []
    for rep in range(2):
        tr = FusedTrainer(spec, 64, (48, 48), device=d, params=flat)
        out = [float(tr.step(hr)["loss"]) for _ in range(3)]
        losses.append((out, tr.params.clone()))
        del tr
    assert losses[0][0] == losses[1][0]
    assert torch.equal(losses[0][1], losses[1][1])
    assert all(math.isfinite(x) for x in losses[0][0])
    assert losses[0][0][2] < losses[0][0][0]   # the loss goes down on a fixed batch


def test_plugin_module_reference_style_step():
    """The drop-in nn.Module: torch.optim.Adam + the reference's l2loss step, against the oracle."""
    d = dev()
    from srmi.config import ConfigContext
    from srmi.model.rcan.network import get_model
    torch.manual_seed(0)  # the module draws its default init from the global generator, as nn.Conv2d does
    with ConfigContext("sres", dict(model="rcan-10-20-64", task="SSS_SST-tiles-48"), **{"model.nlayers": 2,
                                                                                         "model.nblocks": 2}):
        net = get_model(nchannels_in=2, nchannels_out=2, device=d).to(d)
    meta = json.load(open(os.path.join(GOLDEN, "keys.json")))
    oracle = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=2, nblocks=2)
    assert [k for k, _ in net.named_parameters()] == [k for k, _ in oracle.named_parameters()]
    oracle.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
    oracle = oracle.double()
    net.train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    hr = torch.tensor(ro.synthetic_hr(2, 2, 192, 1234)).to(d)
    from srmi.engine import downsample
    opt.zero_grad()
    x = downsample(hr, 4).requires_grad_(True)
    out = net(x)
    loss = torch.sqrt(((out - hr) ** 2).mean())
    loss.backward()
    l_ref, out_ref, g_ref = oracle_grads(oracle, hr.cpu().numpy(), 4)
    bound = drift_bounds(oracle, hr.cpu().numpy(), 4, g_ref)
    assert abs(loss.item() - l_ref) / l_ref < 2e-3
    for name, p in net.named_parameters():
        assert p.grad is not None
        assert rel_l2(p.grad, g_ref[name]) <= bound[name], (name, rel_l2(p.grad, g_ref[name]), bound[name])
    opt.step()
    # state_dict round trip through the tolerant loader
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    net.load_state_dict(sd)
    assert len(meta["keys"]["rcan_small_c2"]) == len(sd)


@pytest.mark.parametrize("cb", [2, 8])
def test_micro_batch_step_matches_single_engine(cb):
    """FusedTrainer(micro=2) -- two half-batch engines on two streams -- computes the
    same step as one engine: the loss comes from per-tile parts summed in tile order
    (srmi_tile_loss_parts / srmi_loss_from_parts), so it is bit-identical whatever the
    split, and the gradients agree up to fp32 summation order.  (A 1-ulp loss
    difference would scale the bf16 gradient maps and flip roundings: 4e-5.)  cb: the
    CA bottleneck (CR = 32, 8; the engines' record slots at a narrower CR)."""
    d = dev()
    spec = spec_of("rcan", 2, 2, 3, cb=cb)
    table = _table(spec)
    from srmi.trainer import default_init_
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=5)
    hr = torch.tensor(ro.synthetic_hr(16, 2, 192, 17)).to(d)
    res = []
    for micro in (1, 2):
        tr = FusedTrainer(spec, 16, (48, 48), device=d, params=flat, micro=micro)
        out = tr.step(hr)
        res.append((float(out["loss"]), float(out["interp_loss"]), tr.grads.clone(), tr.params.clone()))
        del tr
    (l1, i1, g1, p1), (l2, i2, g2, p2) = res
    assert l1 == l2 and i1 == i2
    assert rel_l2(g2, g1) < 1e-5
    assert rel_l2(p2 - flat, p1 - flat) < 1e-4


def test_checkpoint_resume_matches_uninterrupted():
    """FusedTrainer.checkpoint() -> torch.save / torch.load(weights_only) ->
    load_checkpoint() resumes bit-exactly (reference checkpoint layout, §8f row 4)."""
    import io
    d = dev()
    spec = spec_of("rcan", 2, 2, 3)
    table = _table(spec)
    from srmi.trainer import default_init_
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=9)
    hr = torch.tensor(ro.synthetic_hr(8, 2, 192, 21)).to(d)
    a = FusedTrainer(spec, 8, (48, 48), device=d, params=flat, micro=1, lr=2e-4)
    for _ in range(3):
        a.step(hr)
    b = FusedTrainer(spec, 8, (48, 48), device=d, params=flat, micro=1, lr=2e-4)
    for _ in range(2):
        b.step(hr)
    buf = io.BytesIO()
    torch.save(b.checkpoint(epoch=1, itime=2, loss=0.5), buf)
    buf.seek(0)
    state = torch.load(buf, weights_only=True)
    c = FusedTrainer(spec, 8, (48, 48), device=d, params=torch.zeros_like(flat), micro=1, lr=1.0)
    c.load_checkpoint(state)
    assert c.t == 2 and c.lr == 2e-4
    c.step(hr)
    torch.cuda.synchronize()
    assert torch.equal(a.params, c.params)
    assert torch.equal(a.m, c.m) and torch.equal(a.v, c.v)


def _engine_variants_agree(lr_hw, flags, grad_tol, fwd_tol=None, cb=2):
    """One training step of the same weights and tiles through two engine variants
    (srmi_model_config.flags): the forward is untouched (fwd_tol None: bit-identical
    output and loss; else output rel. L2 and loss within fwd_tol), the gradients agree
    to grad_tol (rel. L2 of the whole vector, 3e-2 per tensor; 0: bit-identical) and
    both sit within the drift bounds of the fp64 oracle."""
    from srmi.trainer import default_init_
    d = dev()
    h, w = lr_hw
    C, nl, nb, B = 2, 2, 4, 6
    specs = [NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=nl, nblocks=nb,
                     cbottleneck=cb, scale=4, flags=f) for f in flags]
    table = _table(specs[0])
    flat = torch.empty(sum(t[2] for t in table))
    default_init_(flat, table, seed=21)
    g = torch.Generator().manual_seed(5)
    hr = torch.randn(B, C, 4 * h, 4 * w, generator=g, dtype=torch.float64)
    trs = [FusedTrainer(sp, B, (h, w), device=d, params=flat.to(d), micro=1) for sp in specs]
    outs = [t.step(hr.float().to(d)) for t in trs]
    torch.cuda.synchronize()
    if fwd_tol is None:
        assert torch.equal(trs[0].sr, trs[1].sr)
        assert float(outs[0]["loss"]) == float(outs[1]["loss"])
    else:
        assert rel_l2(trs[0].sr, trs[1].sr) < fwd_tol
        assert abs(float(outs[0]["loss"]) - float(outs[1]["loss"])) < fwd_tol * float(outs[1]["loss"])
    ga, gb = trs[0].grads.cpu(), trs[1].grads.cpu()
    if grad_tol == 0:
        assert torch.equal(ga, gb)
    else:
        assert rel_l2(ga, gb) < grad_tol
    model = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=nl, nblocks=nb, nfeatures=64, cbottleneck=cb).double()
    sd = dict(model.named_parameters())
    with torch.no_grad():
        for name, off, n, shape in table:
            sd[name].copy_(flat[off:off + n].view(shape).double())
    _, _, g_ref = oracle_grads(model, hr.numpy(), 4)
    bound = drift_bounds(model, hr.numpy(), 4, g_ref)
    for name, off, n, shape in table:
        ra = rel_l2(ga[off:off + n].view(shape), g_ref[name])
        rb = rel_l2(gb[off:off + n].view(shape), g_ref[name])
        assert ra <= bound[name] and rb <= bound[name], (name, ra, rb, bound[name])
        assert rel_l2(ga[off:off + n], gb[off:off + n]) < 3e-2, name
    return trs


@pytest.mark.parametrize("lr_hw", [(48, 48), (32, 48), (8, 48), (24, 96)])
def test_ca_forward_in_conv2_matches_ca_pass(lr_hw):
    """The training CA forward inside conv2's launch (the default: conv1 writes t, the
    per-strip sums of the bf16 t and per workgroup its rows' share of mean(u) -- the
    matvec on conv2's bf16 filter image, SRMI_CA_MPART; every conv2 workgroup sums the
    shares, runs the CA MLP and writes u and h' = h + s bf16(u); engine.cpp ca_fwd_mode)
    against the CA pass of its own (SRMI_FLAG_CA_PASS: conv2 + pool writing u, then
    ca_fwd).  mean(u) differs only in fp32 summation order, so the forward agrees far
    below bf16 noise and the gradients (the backward reads the same stored u and record)
    to that order; both sit within the oracle's drift bounds.  Three tile heights move
    the border rows between runs; the 96-wide tiles put columns 0 and W-1 (and the
    corners) in different workgroups."""
    from srmi._lib import SRMI_FLAG_CA_PASS
    _engine_variants_agree(lr_hw, (0, SRMI_FLAG_CA_PASS), 5e-3, fwd_tol=1e-3)


@pytest.mark.parametrize("lr_hw", [(48, 48), (32, 48), (8, 48), (24, 96)])
def test_du_from_g_matches_du_pass(lr_hw):
    """The CALayer backward's du = bf16(g s + dm / HW) formed by the fused conv2 backward
    on its input rings in LDS, from the bf16 gradient stream g (the default: the dgrad's
    ring groups and the filter gradient's dY rows, each wave on its own DMA pieces) against
    du written by the CA backward and read back (SRMI_FLAG_DU_PASS): the same fma and
    rounding, so the whole step is bit-identical.  Three tile heights change the runs'
    and row bands' boundaries (and the image-border halo rows the transform must leave
    zero); the 96-wide tiles take the unfused launches in both engines."""
    from srmi._lib import SRMI_FLAG_DU_PASS, call
    trs = _engine_variants_agree(lr_hw, (0, SRMI_FLAG_DU_PASS), 0)
    # the default engine really took the fused path (srmi_engine_probe which = 4), the
    # du-pass one did not; 96-wide tiles are unfusable in both
    fused = [call("srmi_engine_probe", t.engines[0]._h, 4, 1, None) for t in trs]
    assert fused == ([0, 0] if lr_hw[1] == 96 else [1, 0]), fused


@pytest.mark.parametrize("cb", [8, 16])
def test_du_from_g_matches_du_pass_other_bottlenecks(cb):
    """As above at CA bottlenecks of 64 / 8 = 8 and 64 / 16 = 4 channels (the reference's
    default is 32): the MLP's thread mapping (ca_bwd.hpp) at every CR the fused path takes.
    The oracle check also pins the CA parameter gradients of RCABs 2..nb at CR < 32: the
    batched kernel once stepped between RCABs by N x (2C + CR) floats instead of the
    engine's N x 160 / N x 224 slots, reading uninitialised memory (bit-different between
    two engines, and wrong in both)."""
    from srmi._lib import SRMI_FLAG_DU_PASS, call
    trs = _engine_variants_agree((48, 48), (0, SRMI_FLAG_DU_PASS), 0, cb=cb)
    assert [call("srmi_engine_probe", t.engines[0]._h, 4, 1, None) for t in trs] == [1, 0]


@pytest.mark.parametrize("arch", ["rcan", "edsr"])
def test_backward_stages_one_at_a_time_and_order_checked(arch):
    """srmi_backward_stages run one stage per call gives the gradients of one
    srmi_backward bit for bit; a stage skipped, repeated or out of order -- or a whole
    backward while a staged one is half-way -- is refused (SRMI_ERR_ARG), since the
    gradient-stream buffers and slab parity carry over from stage to stage."""
    from srmi._lib import SrmiError
    from srmi.trainer import default_init_
    d = dev()
    # RCAN 4x 48 -> 192, 2 variables; EDSR 8x 32 -> 256, 4 variables (C4's shapes)
    spec, C, T = (spec_of("rcan", 2, 2, 2), 2, 192) if arch == "rcan" else (spec_of("edsr", 4, 2, scale=8), 4, 256)
    table = _table(spec)
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=4)
    hr = torch.tensor(ro.synthetic_hr(2, C, T, 8)).to(d)
    tr = FusedTrainer(spec, 2, (T // spec.scale,) * 2, device=d, params=flat, micro=1)
    tr.step(hr)  # the engine's last forward, loss4 and sr
    eng = tr.eng
    ns = eng.stage_count
    assert ns == (spec.nlayers + 2 if arch == "rcan" else 1)
    kw = dict(sr=tr.sr, hr=hr, loss4=tr.loss4)
    g_full = torch.zeros_like(tr.grads)
    eng.backward(tr.params, tr.lrbuf, g_full, **kw)
    g_st = torch.zeros_like(tr.grads)
    for s in range(ns):
        eng.backward(tr.params, tr.lrbuf, g_st, stages=(s, s), **kw)
    torch.cuda.synchronize()
    assert torch.equal(g_full, g_st)
    if arch == "rcan":
        with pytest.raises(SrmiError):  # stage 1 before stage 0
            eng.backward(tr.params, tr.lrbuf, g_st, stages=(1, 1), **kw)
        eng.backward(tr.params, tr.lrbuf, g_st, stages=(0, 0), **kw)
        with pytest.raises(SrmiError):  # stage 0 again
            eng.backward(tr.params, tr.lrbuf, g_st, stages=(0, 0), **kw)
        with pytest.raises(SrmiError):  # stage 2 skips stage 1
            eng.backward(tr.params, tr.lrbuf, g_st, stages=(2, 2), **kw)
        with pytest.raises(SrmiError):  # a whole backward half-way through
            eng.backward(tr.params, tr.lrbuf, g_st, **kw)
        eng.backward(tr.params, tr.lrbuf, g_st, stages=(1, ns - 1), **kw)
        torch.cuda.synchronize()
        assert torch.equal(g_full, g_st)
