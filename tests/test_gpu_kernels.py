"""Kernel-level parity of the HIP conv / wgrad / CA / resampling / Adam kernels
against fp64 references of the same op (on the same bf16-rounded operands)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu

from srmi import _lib  # noqa: E402
from srmi._lib import call, ptr  # noqa: E402


def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda", 0)


def S():
    return torch.cuda.current_stream().cuda_stream


def rel_l2(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def bf(t):
    return t.to(torch.bfloat16)


def pack(w, b, ps=0):
    Cout, Cin = w.shape[0], w.shape[1]
    fp = torch.empty(Cout * Cin * 9, dtype=torch.bfloat16, device=w.device)
    dp = torch.empty_like(fp)
    pb = torch.empty(Cout, dtype=torch.float32, device=w.device)
    call("srmi_pack_conv", ptr(w), ptr(b), Cout, Cin, ps, ptr(fp), ptr(dp), ptr(pb), S())
    return fp, dp, pb


def nchw(t):  # NHWC -> NCHW
    return t.permute(0, 3, 1, 2)


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def ps_perm(Cout):
    # packed channel c'' = 64 q + c  <- torch channel 4 c + q
    return torch.tensor([4 * (cp % 64) + cp // 64 for cp in range(Cout)])


SHAPES = [(2, 48, 48), (1, 8, 96), (1, 4, 32), (2, 12, 64), (64, 48, 48), (16, 96, 96), (8, 32, 32)]


def conv(x, fp, pb, N, H, W, Cin, Cout, epi, unshuf=0, yb=None, yf=None, r1=None, r2=None, r3=None, aux=None,
         part=None, alpha=1.0):
    call("srmi_conv3x3", ptr(x), ptr(fp), ptr(pb), N, H, W, Cin, Cout, unshuf, epi, ptr(yb), ptr(yf), ptr(r1), ptr(r2),
         ptr(r3), ptr(aux), ptr(part), float(alpha), S())


@pytest.mark.parametrize("N,H,W", SHAPES)
def test_conv_forward_epilogues(N, H, W):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(1)
    x = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.06).to(d)
    b = (torch.randn(64, generator=g) * 0.1).to(d)
    fp, dp, pb = pack(w, b)
    ref = Fn.conv2d(nchw(x).double().cpu(), bf(w).double().cpu(), b.double().cpu(), padding=1)
    ref = nhwc(ref)
    # relu -> bf16
    yb = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=d)
    conv(x, fp, pb, N, H, W, 64, 64, 0, yb=yb)
    assert rel_l2(yb.float(), ref.clamp_min(0)) < 4e-3
    # pool: bf16 + per-strip channel sums
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, 64, device=d)
    conv(x, fp, pb, N, H, W, 64, 64, 1, yb=yb, part=part)
    assert rel_l2(yb.float(), ref) < 4e-3
    np.testing.assert_allclose(part.sum(1).double().cpu().numpy(), ref.sum((1, 2)).numpy(), rtol=1e-4, atol=1e-3)
    # resid: alpha*(conv+b) + r1 -> fp32 exact-ish
    r1 = torch.randn(N, H, W, 64, generator=g).to(d)
    yf = torch.empty(N, H, W, 64, device=d)
    conv(x, fp, pb, N, H, W, 64, 64, 2, yb=yb, yf=yf, r1=r1, alpha=0.5)
    exp = 0.5 * ref + r1.double().cpu()
    np.testing.assert_allclose(yf.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=2e-5)
    assert rel_l2(yb.float(), exp) < 4e-3


@pytest.mark.parametrize("N,H,W", [(2, 48, 48), (1, 4, 96)])
def test_conv_pixelshuffle_forward(N, H, W):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(2)
    x = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    w = (torch.randn(256, 64, 3, 3, generator=g) * 0.06).to(d)
    b = (torch.randn(256, generator=g) * 0.1).to(d)
    fp, dp, pb = pack(w, b, ps=1)
    y = torch.empty(N, 2 * H, 2 * W, 64, dtype=torch.bfloat16, device=d)
    conv(x, fp, pb, N, H, W, 64, 256, 3, yb=y)
    ref = Fn.pixel_shuffle(Fn.conv2d(nchw(x).double().cpu(), bf(w).double().cpu(), b.double().cpu(), padding=1), 2)
    assert rel_l2(y.float(), nhwc(ref)) < 4e-3


@pytest.mark.parametrize("N,H,W", SHAPES)
def test_conv_dgrad_epilogues(N, H, W):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(3)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.06).to(d)
    b = torch.zeros(64, device=d)
    fp, dp, pb = pack(w, b)
    dy = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    ref = torch.nn.grad.conv2d_input((N, 64, H, W), bf(w).double().cpu(), nchw(dy).double().cpu(), padding=1)
    ref = nhwc(ref)
    out = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=d)
    conv(dy, dp, None, N, H, W, 64, 64, 6, yb=out)
    assert rel_l2(out.float(), ref) < 4e-3
    # relu mask with t
    t = bf(torch.randn(N, H, W, 64, generator=g).clamp_min(0)).to(d)
    conv(dy, dp, None, N, H, W, 64, 64, 4, yb=out, aux=t, alpha=2.0)
    exp = 2.0 * ref * (t.double().cpu() > 0)
    assert rel_l2(out.float(), exp) < 4e-3
    # acc: g = acc + r1 + r2 + r3, with G / ds partial sums
    r1, r2, r3 = [torch.randn(N, H, W, 64, generator=g).to(d) for _ in range(3)]
    u = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, 128, device=d)
    yf = r1.clone()
    conv(dy, dp, None, N, H, W, 64, 64, 5, yb=out, yf=yf, r1=yf, r2=r2, r3=r3, aux=u, part=part)
    exp = ref + r1.double().cpu() + r2.double().cpu() + r3.double().cpu()
    np.testing.assert_allclose(yf.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=5e-5)
    assert rel_l2(out.float(), exp) < 4e-3
    Gs = part[:, :, :64].sum(1).double().cpu()
    ds = part[:, :, 64:].sum(1).double().cpu()
    np.testing.assert_allclose(Gs.numpy(), exp.sum((1, 2)).numpy(), rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(ds.numpy(), (exp * u.double().cpu()).sum((1, 2)).numpy(), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("N,H,W", [(2, 48, 48), (1, 4, 96)])
def test_conv_dgrad_unshuffle(N, H, W):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(4)
    w = (torch.randn(256, 64, 3, 3, generator=g) * 0.06).to(d)
    b = torch.zeros(256, device=d)
    fp, dp, pb = pack(w, b, ps=1)
    dyp = bf(torch.randn(N, 2 * H, 2 * W, 64, generator=g)).to(d)   # grad wrt PS output
    dy_log = Fn.pixel_unshuffle(nchw(dyp).double().cpu(), 2)          # grad wrt conv output (torch order)
    ref = nhwc(torch.nn.grad.conv2d_input((N, 64, H, W), bf(w).double().cpu(), dy_log, padding=1))
    out = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=d)
    conv(dyp, dp, None, N, H, W, 256, 64, 6, unshuf=1, yb=out)
    assert rel_l2(out.float(), ref) < 4e-3


@pytest.mark.parametrize("N,H,W,rs", [(2, 48, 48, 0), (2, 48, 48, 1), (1, 8, 96, 0), (1, 4, 32, 0), (3, 12, 64, 3),
                                       (64, 48, 48, 0), (4, 96, 96, 0), (3, 12, 48, 3), (2, 48, 48, 12), (1, 8, 48, 2),
                                       (2, 24, 48, 2)])
def test_wgrad(N, H, W, rs):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(5)
    x = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    dy = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    slab = torch.empty(64 << 20, dtype=torch.float32, device=d)
    gw = torch.empty(64, 64, 3, 3, device=d)
    gb = torch.empty(64, device=d)
    call("srmi_wgrad3x3", ptr(x), ptr(dy), N, H, W, 64, 0, rs, ptr(slab), slab.numel() * 4, 0, 1.0, ptr(gw), ptr(gb),
         S())
    ref = torch.nn.grad.conv2d_weight(nchw(x).double().cpu(), (64, 64, 3, 3), nchw(dy).double().cpu(), padding=1)
    assert rel_l2(gw, ref) < 1e-5
    np.testing.assert_allclose(gb.double().cpu().numpy(), dy.double().cpu().sum((0, 1, 2)).numpy(), rtol=1e-4,
                               atol=1e-3)


@pytest.mark.parametrize("N,H,W", [(2, 48, 48), (1, 4, 96)])
def test_wgrad_pixelshuffle(N, H, W):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(6)
    x = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    dyp = bf(torch.randn(N, 2 * H, 2 * W, 64, generator=g)).to(d)
    slab = torch.empty(64 << 20, dtype=torch.float32, device=d)
    gw = torch.empty(256, 64, 3, 3, device=d)
    gb = torch.empty(256, device=d)
    call("srmi_wgrad3x3", ptr(x), ptr(dyp), N, H, W, 256, 1, 0, ptr(slab), slab.numel() * 4, 1, 1.0, ptr(gw), ptr(gb),
         S())
    dy_log = Fn.pixel_unshuffle(nchw(dyp).double().cpu(), 2)
    ref = torch.nn.grad.conv2d_weight(nchw(x).double().cpu(), (256, 64, 3, 3), dy_log, padding=1)
    assert rel_l2(gw, ref) < 1e-5
    np.testing.assert_allclose(gb.double().cpu().numpy(), dy_log.sum((0, 2, 3)).numpy(), rtol=1e-4, atol=1e-3)


def test_channel_attention_fwd_bwd():
    d = dev()
    N, H, W, Cc, R = 2, 48, 48, 64, 2
    g = torch.Generator(device="cpu").manual_seed(7)
    u = bf(torch.randn(N, H, W, Cc, generator=g)).to(d)
    h_in = torch.randn(N, H, W, Cc, generator=g).to(d)
    w1 = (torch.randn(Cc // R, Cc, generator=g) * 0.1).to(d)
    b1 = (torch.randn(Cc // R, generator=g) * 0.1).to(d)
    w2 = (torch.randn(Cc, Cc // R, generator=g) * 0.1).to(d)
    b2 = (torch.randn(Cc, generator=g) * 0.1).to(d)
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, Cc, device=d)
    part[:, 0, :] = u.float().sum((1, 2))
    h_out = torch.empty_like(h_in)
    hb = torch.empty(N, H, W, Cc, dtype=torch.bfloat16, device=d)
    rec = torch.empty(N, 160, device=d)
    call("srmi_ca_forward", ptr(u), ptr(part), ns, ptr(w1), ptr(b1), ptr(w2), ptr(b2), N, H * W, Cc, R, ptr(h_in),
         ptr(h_out), ptr(hb), ptr(rec), S())
    # torch reference (fp64 on CPU)
    U = u.double().cpu().requires_grad_(True)
    W1, B1, W2, B2 = [t.double().cpu().requires_grad_(True) for t in (w1, b1, w2, b2)]
    m = U.mean((1, 2))
    z1 = m @ W1.T + B1
    s = torch.sigmoid(torch.relu(z1) @ W2.T + B2)
    y = U * s[:, None, None, :] + h_in.double().cpu()
    np.testing.assert_allclose(h_out.double().cpu().numpy(), y.detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(rec[:, 96:].double().cpu().numpy(), s.detach().numpy(), rtol=1e-5, atol=1e-6)
    # backward: g -> du, brec
    gy = torch.randn(N, H, W, Cc, generator=g).to(d)
    y.backward(gy.double().cpu())
    bpart = torch.zeros(N, ns, 2 * Cc, device=d)
    bpart[:, 0, :Cc] = gy.sum((1, 2))
    bpart[:, 0, Cc:] = (gy * u.float()).sum((1, 2))
    du = torch.empty(N, H, W, Cc, dtype=torch.bfloat16, device=d)
    brec = torch.empty(N * 224, device=d)  # [N][160] then dm[N][64]
    call("srmi_ca_backward", ptr(gy), ptr(bpart), ns, ptr(rec), ptr(w1), ptr(w2), N, H * W, Cc, R, ptr(du), ptr(brec),
         S())
    assert rel_l2(du.float(), U.grad) < 4e-3
    # conv2-bias grad path: sum_p du = s*G + dm
    np.testing.assert_allclose(brec[:N * 160].view(N, 160)[:, 96:].double().cpu().numpy(), U.grad.sum((1, 2)).numpy(), rtol=1e-4, atol=1e-3)


def test_downsample_upsample_match_reference():
    import os
    d = dev()
    gd = np.load(os.path.join(os.path.dirname(__file__), "golden", "ops.npz"))
    x = torch.tensor(gd["down4_in"]).to(d)
    y = torch.empty(2, 2, 48, 48, device=d)
    call("srmi_downsample", ptr(x), 2, 2, 192, 192, 4, ptr(y), S())
    np.testing.assert_allclose(y.double().cpu().numpy(), gd["down4_out"], rtol=1e-5, atol=1e-6)
    x8 = torch.tensor(gd["down8_in"]).to(d)
    y8 = torch.empty(1, 1, 32, 32, device=d)
    call("srmi_downsample", ptr(x8), 1, 1, 256, 256, 8, ptr(y8), S())
    np.testing.assert_allclose(y8.double().cpu().numpy(), gd["down8_out"], rtol=1e-5, atol=1e-6)
    u = torch.tensor(gd["up4_in"]).to(d)
    up = torch.empty(1, 2, 96, 96, device=d)
    call("srmi_upsample", ptr(u), 1, 2, 24, 24, 4, ptr(up), S())
    np.testing.assert_allclose(up.double().cpu().numpy(), gd["up4_out"], rtol=1e-5, atol=1e-5)


def test_adam_matches_reference():
    import os
    d = dev()
    gd = np.load(os.path.join(os.path.dirname(__file__), "golden", "ops.npz"))
    p = torch.tensor(gd["adam_p0"], dtype=torch.float32).to(d)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for k in range(3):
        gk = torch.tensor(gd["adam_g"][k], dtype=torch.float32).to(d)
        call("srmi_adam_step", ptr(p), ptr(gk), ptr(m), ptr(v), p.numel(), k + 1, 1e-3, 0.9, 0.999, 1e-8, 0.0, S())
    np.testing.assert_allclose(p.double().cpu().numpy(), gd["adam_p3"], rtol=0, atol=2e-6)


@pytest.mark.parametrize("C,H,W", [(1, 8, 192), (2, 12, 192), (4, 8, 256), (3, 4, 96)])
def test_tail_forward(C, H, W):
    """Tail conv 64 -> C (network.py:16 / EDSR tail) through srmi_tail_forward: MFMA
    implicit GEMM with bf16 operands vs an fp64 conv of the same bf16 input."""
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(12)
    N = 2
    x = bf(torch.randn(N, H, W, 64, generator=g)).to(d)
    w = (torch.randn(C, 64, 3, 3, generator=g) * 0.05).to(d)
    b = (torch.randn(C, generator=g) * 0.1).to(d)
    y = torch.empty(N, C, H, W, device=d)
    call("srmi_tail_forward", ptr(x), ptr(w), ptr(b), N, C, H, W, ptr(y), S())
    ref = Fn.conv2d(nchw(x).double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
    assert rel_l2(y, ref) < 4e-3
