"""Pin the CPU oracle (oracle/rcan_oracle.py) against the golden vectors that
tests/golden/make_golden.py produced from the real reference.  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import rcan_oracle as ro
from conftest import GOLDEN


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def _sample_idx(n, k=48):
    return np.unique(np.linspace(0, n - 1, min(n, k)).astype(np.int64))


def test_downsample_closed_form_matches_reference():
    g = _load("ops.npz")
    x = g["down4_in"].astype(np.float64)
    # torch path of the oracle
    y = ro.downsample(torch.tensor(x), 4).numpy()
    np.testing.assert_allclose(y, g["down4_out"], rtol=0, atol=1e-12)
    # the closed-form separable [-3,19,19,-3]/32 filter the HIP kernel implements
    y2 = ro.downsample_explicit(x, 4)
    np.testing.assert_allclose(y2, g["down4_out"], rtol=0, atol=1e-12)
    x8 = g["down8_in"].astype(np.float64)
    np.testing.assert_allclose(ro.downsample_explicit(x8, 8), g["down8_out"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(ro.downsample(torch.tensor(x8), 8).numpy(), g["down8_out"], atol=1e-12)


def test_upsample_and_l2loss():
    g = _load("ops.npz")
    u = ro.upsample(torch.tensor(g["up4_in"].astype(np.float64)), 4).numpy()
    np.testing.assert_allclose(u, g["up4_out"], atol=1e-12)
    p = torch.tensor(g["l2_p"], requires_grad=True)
    lv = ro.l2loss(p, torch.tensor(g["l2_t"]))
    lv.backward()
    assert abs(lv.item() - float(g["l2_val"])) < 1e-14
    np.testing.assert_allclose(p.grad.numpy(), g["l2_grad"], atol=1e-15)


def test_pixelshuffle_and_adam():
    g = _load("ops.npz")
    ps = torch.nn.PixelShuffle(2)(torch.tensor(g["ps_in"])).numpy()
    np.testing.assert_array_equal(ps, g["ps_out"])
    # out[c, 2h+i, 2w+j] = in[4c+2i+j, h, w]
    inp = g["ps_in"][0]
    for c in range(2):
        for i in range(2):
            for j in range(2):
                np.testing.assert_array_equal(g["ps_out"][0, c, i::2, j::2], inp[4 * c + 2 * i + j])
    p = torch.tensor(g["adam_p0"]).clone()
    p.grad = None
    opt = ro.AdamOracle([p], lr=1e-3)
    for k in range(3):
        p.grad = torch.tensor(g["adam_g"][k])
        opt.step()
    np.testing.assert_allclose(p.numpy(), g["adam_p3"], rtol=0, atol=1e-14)


def test_ca_and_rcab_blocks():
    g = _load("ops.npz")
    ca = ro._CA(64, 2).double()
    with torch.no_grad():
        flat = torch.tensor(g["ca_params"])
        off = 0
        for q in ca.parameters():
            q.copy_(flat[off:off + q.numel()].view_as(q))
            off += q.numel()
    x = torch.tensor(g["ca_x"], requires_grad=True)
    y = ca(x)
    y.backward(torch.tensor(g["ca_gy"]))
    np.testing.assert_allclose(y.detach().numpy(), g["ca_y"], atol=1e-13)
    np.testing.assert_allclose(x.grad.numpy(), g["ca_gx"], atol=1e-13)
    pg = np.concatenate([q.grad.numpy().ravel() for q in ca.parameters()])
    np.testing.assert_allclose(pg, g["ca_pgrads"], atol=1e-12)
    rcab = ro._RCAB(64, 3, 2).double()
    ro.init_params_numpy(rcab, 22)
    xr = torch.tensor(g["rcab_x"], requires_grad=True)
    yr = rcab(xr)
    yr.backward(torch.tensor(g["rcab_gy"]))
    np.testing.assert_allclose(yr.detach().numpy(), g["rcab_y"], atol=1e-12)
    np.testing.assert_allclose(xr.grad.numpy(), g["rcab_gx"], atol=1e-12)
    l2 = np.array([np.sqrt((q.grad.numpy() ** 2).sum()) for q in rcab.parameters()])
    np.testing.assert_allclose(l2, g["rcab_pgrad_l2"], rtol=1e-11)


def test_state_dict_keys_match_reference():
    meta = json.load(open(os.path.join(GOLDEN, "keys.json")))
    m = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20, nfeatures=64, cbottleneck=2)
    got = [[k, list(v.shape)] for k, v in m.named_parameters()]
    assert got == meta["keys"]["rcan-10-20-64_c2"]
    assert sum(p.numel() for p in m.parameters()) == 16313602
    m1 = ro.RCANOracle(nchannels_in=1, nchannels_out=1, nlayers=10, nblocks=20)
    assert sum(p.numel() for p in m1.parameters()) == 16312449
    e = ro.EDSROracle(nchannels_in=4, nchannels_out=4, nlayers=2, downscale_factors=[2, 2, 2])
    assert [[k, list(v.shape)] for k, v in e.named_parameters()] == meta["keys"]["edsr_small_c4"]


def _model_case(name, model, C, dtype, steps, atol_out, rtol_grad):
    g = _load(name)
    B, C_, S = [int(v) for v in g["shape"]]
    assert C_ == C
    hr = ro.synthetic_hr(B, C, S, int(g["seed_x"]))
    assert abs(hr.astype(np.float64).sum() - float(g["hr_sum"])) < 1e-6
    np.testing.assert_array_equal(hr[:, :, ::8, ::8], g["hr_sub"])
    ro.init_params_numpy(model, int(g["seed_w"]))
    model = model.to(dtype)
    opt = ro.AdamOracle(list(model.parameters()), lr=float(g["lr"]))
    scale = model.parms["scale"]
    for step in range(steps):
        opt.zero_grad()
        h = torch.tensor(hr, dtype=dtype, requires_grad=True)
        lr_in = ro.downsample(h, scale)
        out = model(lr_in)
        loss = ro.l2loss(out, h)
        loss.backward()
        assert abs(loss.item() - float(g[f"loss{step}"])) <= 1e-12 + 1e-7 * (dtype == torch.float32)
        with torch.no_grad():
            il = ro.l2loss(h, ro.upsample(lr_in, scale)).item()
        assert abs(il - float(g[f"iloss{step}"])) < 1e-6
        if step == 0:
            o = out.detach().double().numpy()
            np.testing.assert_allclose(o[:, :, ::4, ::4], g["out_sub"], atol=atol_out)
            gl2 = np.array([np.sqrt((p.grad.double() ** 2).sum().item()) for p in model.parameters()])
            np.testing.assert_allclose(gl2, g["grad_l2"], rtol=rtol_grad)
            gs = np.concatenate([p.grad.double().numpy().ravel()[_sample_idx(p.numel())] for p in model.parameters()])
            np.testing.assert_allclose(gs, g["grad_sample"], rtol=rtol_grad, atol=rtol_grad * np.abs(gs).max())
        opt.step()
        if step == 0:
            ps = np.concatenate([p.detach().double().numpy().ravel()[_sample_idx(p.numel())] for p in model.parameters()])
            np.testing.assert_allclose(ps, g["p1_sample"], atol=1e-10 if dtype == torch.float64 else 1e-6)


@pytest.mark.parametrize("C", [1, 2])
def test_rcan_small_train_step_f64(C):
    m = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=2, nblocks=2, nfeatures=64, cbottleneck=2)
    _model_case(f"rcan_small_c{C}_f64.npz", m, C, torch.float64, 2, 1e-12, 1e-9)


def test_rcan_small_train_step_f32():
    m = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=2, nblocks=2, nfeatures=64, cbottleneck=2)
    _model_case("rcan_small_c2_f32.npz", m, 2, torch.float32, 2, 1e-5, 1e-3)


def test_edsr_small_train_step_f64():
    m = ro.EDSROracle(nchannels_in=4, nchannels_out=4, nlayers=2, nfeatures=64, downscale_factors=[2, 2, 2])
    _model_case("edsr_small_c4_f64.npz", m, 4, torch.float64, 2, 1e-12, 1e-9)


@pytest.mark.slow
def test_rcan_full_train_step_f64():
    m = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20, nfeatures=64, cbottleneck=2)
    _model_case("rcan_full_c2_f64.npz", m, 2, torch.float64, 1, 1e-11, 1e-8)
