"""Kernel-level parity of the HIP conv / wgrad / CA / resampling / Adam kernels
against fp64 references of the same op, in both engine operand types: bf16
(references on the same bf16-rounded operands; bf16 outputs within 4e-3 rel-L2)
and exact fp32 (SRMI_DTYPE_F32: outputs within 1e-5 rel-L2 of fp64, the
north-star's fp32 tolerance)."""
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


DTS = ["bf16", "fp32"]
TORCH_DT = {"bf16": torch.bfloat16, "fp32": torch.float32}
ABI_DT = {"bf16": _lib.SRMI_DTYPE_BF16, "fp32": _lib.SRMI_DTYPE_F32}
TOL = {"bf16": 4e-3, "fp32": 1e-5}   # rel-L2 of operand-type outputs vs fp64


def bf(t):
    return t.to(torch.bfloat16)


def op(t, dt):
    """an operand in the engine's storage type"""
    return t.to(TORCH_DT[dt])


def pack(w, b, ps=0, dt="bf16"):
    Cout, Cin = w.shape[0], w.shape[1]
    fp = torch.empty(Cout * Cin * 9, dtype=TORCH_DT[dt], device=w.device)
    dp = torch.empty_like(fp)
    pb = torch.empty(Cout, dtype=torch.float32, device=w.device)
    call("srmi_pack_conv", ptr(w), ptr(b), Cout, Cin, ps, ptr(fp), ptr(dp), ptr(pb), ABI_DT[dt], S())
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
         part=None, alpha=1.0, dt="bf16"):
    call("srmi_conv3x3", ptr(x), ptr(fp), ptr(pb), N, H, W, Cin, Cout, unshuf, epi, ptr(yb), ptr(yf), ptr(r1), ptr(r2),
         ptr(r3), ptr(aux), ptr(part), float(alpha), ABI_DT[dt], S())


def wref(w, dt):
    """the filter as the kernel sees it (bf16-rounded in the bf16 mode)"""
    return (bf(w) if dt == "bf16" else w).double().cpu()


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("N,H,W", SHAPES)
def test_conv_forward_epilogues(N, H, W, dt):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(1)
    x = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.06).to(d)
    b = (torch.randn(64, generator=g) * 0.1).to(d)
    fp, dp, pb = pack(w, b, dt=dt)
    ref = Fn.conv2d(nchw(x).double().cpu(), wref(w, dt), b.double().cpu(), padding=1)
    ref = nhwc(ref)
    # relu -> operand type
    yb = torch.empty(N, H, W, 64, dtype=TORCH_DT[dt], device=d)
    conv(x, fp, pb, N, H, W, 64, 64, 0, yb=yb, dt=dt)
    assert rel_l2(yb.float(), ref.clamp_min(0)) < TOL[dt]
    # pool: + per-strip channel sums
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, 64, device=d)
    conv(x, fp, pb, N, H, W, 64, 64, 1, yb=yb, part=part, dt=dt)
    assert rel_l2(yb.float(), ref) < TOL[dt]
    np.testing.assert_allclose(part.sum(1).double().cpu().numpy(), ref.sum((1, 2)).numpy(), rtol=1e-4, atol=1e-3)
    # resid: alpha*(conv+b) + r1 -> fp32 exact-ish
    r1 = torch.randn(N, H, W, 64, generator=g).to(d)
    yf = torch.empty(N, H, W, 64, device=d)
    conv(x, fp, pb, N, H, W, 64, 64, 2, yb=yb, yf=yf, r1=r1, alpha=0.5, dt=dt)
    exp = 0.5 * ref + r1.double().cpu()
    np.testing.assert_allclose(yf.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=2e-5)
    assert rel_l2(yb.float(), exp) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("N,H,W", [(2, 48, 48), (1, 4, 96), (2, 8, 32)])
def test_conv_pixelshuffle_forward(N, H, W, dt):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(2)
    x = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    w = (torch.randn(256, 64, 3, 3, generator=g) * 0.06).to(d)
    b = (torch.randn(256, generator=g) * 0.1).to(d)
    fp, dp, pb = pack(w, b, ps=1, dt=dt)
    y = torch.empty(N, 2 * H, 2 * W, 64, dtype=TORCH_DT[dt], device=d)
    conv(x, fp, pb, N, H, W, 64, 256, 3, yb=y, dt=dt)
    ref = Fn.pixel_shuffle(Fn.conv2d(nchw(x).double().cpu(), wref(w, dt), b.double().cpu(), padding=1), 2)
    assert rel_l2(y.float(), nhwc(ref)) < TOL[dt]


def test_conv_pixelshuffle_bf16_at_32bit_boundary():
    """The output-range guard sizes the map from the bytes actually stored: a bf16
    pixel-shuffle output of 456 x 192^2 x 64 elements is 2.15 GB (< 2^32 bytes) and
    must run, although the same map in fp32 would be refused.  The last image -- the
    far end of the buffer resource -- equals that image convolved alone."""
    d = dev()
    N, H, W = 456, 96, 96
    assert N * H * W * 256 * 4 >= 2 ** 32 > N * H * W * 256 * 2
    g = torch.Generator(device="cpu").manual_seed(9)
    w = (torch.randn(256, 64, 3, 3, generator=g) * 0.06).to(d)
    b = (torch.randn(256, generator=g) * 0.1).to(d)
    fp, dp, pb = pack(w, b, ps=1)
    x = torch.randn(N, H, W, 64, device=d, dtype=torch.bfloat16)
    y = torch.empty(N, 2 * H, 2 * W, 64, dtype=torch.bfloat16, device=d)
    conv(x, fp, pb, N, H, W, 64, 256, 3, yb=y)
    y1 = torch.empty(1, 2 * H, 2 * W, 64, dtype=torch.bfloat16, device=d)
    conv(x[N - 1:].contiguous(), fp, pb, 1, H, W, 64, 256, 3, yb=y1)
    torch.cuda.synchronize()
    assert torch.equal(y[N - 1:], y1)
    assert float(y1.float().abs().sum()) > 0


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("N,H,W", SHAPES)
def test_conv_dgrad_epilogues(N, H, W, dt):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(3)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.06).to(d)
    b = torch.zeros(64, device=d)
    fp, dp, pb = pack(w, b, dt=dt)
    dy = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    ref = torch.nn.grad.conv2d_input((N, 64, H, W), wref(w, dt), nchw(dy).double().cpu(), padding=1)
    ref = nhwc(ref)
    out = torch.empty(N, H, W, 64, dtype=TORCH_DT[dt], device=d)
    conv(dy, dp, None, N, H, W, 64, 64, 6, yb=out, dt=dt)
    assert rel_l2(out.float(), ref) < TOL[dt]
    # relu mask with t
    t = op(torch.randn(N, H, W, 64, generator=g).clamp_min(0), dt).to(d)
    conv(dy, dp, None, N, H, W, 64, 64, 4, yb=out, aux=t, alpha=2.0, dt=dt)
    exp = 2.0 * ref * (t.double().cpu() > 0)
    assert rel_l2(out.float(), exp) < TOL[dt]
    # acc: g = acc + r1 + r2 + r3, with G / ds partial sums
    r1, r2, r3 = [torch.randn(N, H, W, 64, generator=g).to(d) for _ in range(3)]
    u = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, 128, device=d)
    yf = r1.clone()
    conv(dy, dp, None, N, H, W, 64, 64, 5, yb=out, yf=yf, r1=yf, r2=r2, r3=r3, aux=u, part=part, dt=dt)
    exp = ref + r1.double().cpu() + r2.double().cpu() + r3.double().cpu()
    np.testing.assert_allclose(yf.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=5e-5)
    assert rel_l2(out.float(), exp) < TOL[dt]
    Gs = part[:, :, :64].sum(1).double().cpu()
    ds = part[:, :, 64:].sum(1).double().cpu()
    np.testing.assert_allclose(Gs.numpy(), exp.sum((1, 2)).numpy(), rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(ds.numpy(), (exp * u.double().cpu()).sum((1, 2)).numpy(), rtol=1e-4, atol=2e-3)
    # the RCAB form (epi 7): g += dx in place, sums of g and g*u, nothing else
    yf = r1.clone()
    part.zero_()
    conv(dy, dp, None, N, H, W, 64, 64, 7, yf=yf, r1=yf, aux=u, part=part, dt=dt)
    exp = ref + r1.double().cpu()
    np.testing.assert_allclose(yf.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=5e-5)
    Gs = part[:, :, :64].sum(1).double().cpu()
    ds = part[:, :, 64:].sum(1).double().cpu()
    np.testing.assert_allclose(Gs.numpy(), exp.sum((1, 2)).numpy(), rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(ds.numpy(), (exp * u.double().cpu()).sum((1, 2)).numpy(), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("N,H,W", [(2, 48, 48), (1, 4, 96), (2, 8, 32)])
def test_conv_dgrad_unshuffle(N, H, W, dt):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(4)
    w = (torch.randn(256, 64, 3, 3, generator=g) * 0.06).to(d)
    b = torch.zeros(256, device=d)
    fp, dp, pb = pack(w, b, ps=1, dt=dt)
    dyp = op(torch.randn(N, 2 * H, 2 * W, 64, generator=g), dt).to(d)  # grad wrt PS output
    dy_log = Fn.pixel_unshuffle(nchw(dyp).double().cpu(), 2)          # grad wrt conv output (torch order)
    ref = nhwc(torch.nn.grad.conv2d_input((N, 64, H, W), wref(w, dt), dy_log, padding=1))
    out = torch.empty(N, H, W, 64, dtype=TORCH_DT[dt], device=d)
    conv(dyp, dp, None, N, H, W, 256, 64, 6, unshuf=1, yb=out, dt=dt)
    assert rel_l2(out.float(), ref) < TOL[dt]


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 48, 48, 128, 128), (1, 8, 96, 192, 64), (2, 8, 32, 128, 64),
                                             (3, 12, 48, 256, 128)])
def test_conv_generic_multichunk(N, H, W, Cin, Cout):
    """The generic conv (Cin > 64, plain input): the K stream of Cin/64 chunks x 9
    filter slices with its three-slice register prefetch and the chunk-boundary
    halo reload, at 2, 3 and 4 chunks and one or two output-channel blocks."""
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(9)
    x = bf(torch.randn(N, H, W, Cin, generator=g)).to(d)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.04).to(d)
    b = (torch.randn(Cout, generator=g) * 0.1).to(d)
    fp, dp, pb = pack(w, b)
    ref = nhwc(Fn.conv2d(nchw(x).double().cpu(), wref(w, "bf16"), b.double().cpu(), padding=1))
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=d)
    conv(x, fp, pb, N, H, W, Cin, Cout, 6, yb=y)
    assert rel_l2(y.float(), ref) < TOL["bf16"]
    conv(x, fp, pb, N, H, W, Cin, Cout, 0, yb=y)
    assert rel_l2(y.float(), ref.clamp_min(0)) < TOL["bf16"]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("N,H,W,rs", [(2, 48, 48, 0), (2, 48, 48, 1), (1, 8, 96, 0), (1, 4, 32, 0), (3, 12, 64, 3),
                                       (64, 48, 48, 0), (4, 96, 96, 0), (3, 12, 48, 3), (2, 48, 48, 12), (1, 8, 48, 2),
                                       (2, 24, 48, 2), (4, 32, 32, 4), (2, 16, 128, 2), (2, 8, 144, 1),
                                       (32, 96, 96, 1)])
def test_wgrad(N, H, W, rs, dt):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(5)
    x = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    dy = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    slab = torch.empty(64 << 20, dtype=torch.float32, device=d)
    gw = torch.empty(64, 64, 3, 3, device=d)
    gb = torch.empty(64, device=d)
    call("srmi_wgrad3x3", ptr(x), ptr(dy), N, H, W, 64, 0, rs, ptr(slab), slab.numel() * 4, 0, 1.0, ptr(gw), ptr(gb),
         ABI_DT[dt], S())
    ref = torch.nn.grad.conv2d_weight(nchw(x).double().cpu(), (64, 64, 3, 3), nchw(dy).double().cpu(), padding=1)
    assert rel_l2(gw, ref) < 1e-5
    np.testing.assert_allclose(gb.double().cpu().numpy(), dy.double().cpu().sum((0, 1, 2)).numpy(), rtol=1e-4,
                               atol=1e-3)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("N,H,W", [(2, 48, 48), (1, 4, 96), (2, 8, 32), (2, 96, 96)])
def test_wgrad_pixelshuffle(N, H, W, dt):
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(6)
    x = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    dyp = op(torch.randn(N, 2 * H, 2 * W, 64, generator=g), dt).to(d)
    slab = torch.empty(64 << 20, dtype=torch.float32, device=d)
    gw = torch.empty(256, 64, 3, 3, device=d)
    gb = torch.empty(256, device=d)
    call("srmi_wgrad3x3", ptr(x), ptr(dyp), N, H, W, 256, 1, 0, ptr(slab), slab.numel() * 4, 1, 1.0, ptr(gw), ptr(gb),
         ABI_DT[dt], S())
    dy_log = Fn.pixel_unshuffle(nchw(dyp).double().cpu(), 2)
    ref = torch.nn.grad.conv2d_weight(nchw(x).double().cpu(), (256, 64, 3, 3), dy_log, padding=1)
    assert rel_l2(gw, ref) < 1e-5
    np.testing.assert_allclose(gb.double().cpu().numpy(), dy_log.sum((0, 2, 3)).numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dt", DTS)
def test_channel_attention_fwd_bwd(dt):
    d = dev()
    N, H, W, Cc, R = 2, 48, 48, 64, 2
    g = torch.Generator(device="cpu").manual_seed(7)
    u = op(torch.randn(N, H, W, Cc, generator=g), dt).to(d)
    h_in = torch.randn(N, H, W, Cc, generator=g).to(d)
    w1 = (torch.randn(Cc // R, Cc, generator=g) * 0.1).to(d)
    b1 = (torch.randn(Cc // R, generator=g) * 0.1).to(d)
    w2 = (torch.randn(Cc, Cc // R, generator=g) * 0.1).to(d)
    b2 = (torch.randn(Cc, generator=g) * 0.1).to(d)
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, Cc, device=d)
    part[:, 0, :] = u.float().sum((1, 2))
    h_out = torch.empty_like(h_in)
    hb = torch.empty(N, H, W, Cc, dtype=TORCH_DT[dt], device=d)
    rec = torch.empty(N, 160, device=d)
    call("srmi_ca_forward", ptr(u), ptr(part), ns, ptr(w1), ptr(b1), ptr(w2), ptr(b2), N, H * W, Cc, R, ptr(h_in),
         ptr(h_out), ptr(hb), ptr(rec), ABI_DT[dt], S())
    # torch reference (fp64 on CPU)
    U = u.double().cpu().requires_grad_(True)
    W1, B1, W2, B2 = [t.double().cpu().requires_grad_(True) for t in (w1, b1, w2, b2)]
    m = U.mean((1, 2))
    z1 = m @ W1.T + B1
    s = torch.sigmoid(torch.relu(z1) @ W2.T + B2)
    y = U * s[:, None, None, :] + h_in.double().cpu()
    np.testing.assert_allclose(h_out.double().cpu().numpy(), y.detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(rec[:, 96:].double().cpu().numpy(), s.detach().numpy(), rtol=1e-5, atol=1e-6)
    assert rel_l2(hb.float(), y.detach()) < TOL[dt]
    # backward: g -> du, brec
    gy = torch.randn(N, H, W, Cc, generator=g).to(d)
    y.backward(gy.double().cpu())
    bpart = torch.zeros(N, ns, 2 * Cc, device=d)
    bpart[:, 0, :Cc] = gy.sum((1, 2))
    bpart[:, 0, Cc:] = (gy * u.float()).sum((1, 2))
    du = torch.empty(N, H, W, Cc, dtype=TORCH_DT[dt], device=d)
    brec = torch.empty(N * 224, device=d)  # [N][160] then dm[N][64]
    call("srmi_ca_backward", ptr(gy), ptr(bpart), ns, ptr(rec), ptr(w1), ptr(w2), N, H * W, Cc, R, ptr(du), ptr(brec),
         ABI_DT[dt], S())
    assert rel_l2(du.float(), U.grad) < TOL[dt]
    # conv2-bias grad path: sum_p du = s*G + dm
    np.testing.assert_allclose(brec[:N * 160].view(N, 160)[:, 96:].double().cpu().numpy(), U.grad.sum((1, 2)).numpy(), rtol=1e-4, atol=1e-3)


def lo8_decode(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """The residual pair's value (csrc/common.hpp pair_decode4, include/srmi.h
    srmi_ca_forward_pair): fp32 bits ((hi << 16) | 0x80) + (sext8(lo) << 8)."""
    hb = hi.cpu().view(torch.int16).to(torch.int64) & 0xFFFF
    q = lo.cpu().view(torch.int8).to(torch.int64)
    bits = (((hb << 16) | 0x80) + (q << 8)) & 0xFFFFFFFF
    bits = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
    return bits.view(torch.float32).double()


def test_channel_attention_forward_residual_pair():
    """The bf16 engine's residual stream as a pair (hi bf16, lo int8 remainder): the
    group's first CALayer add takes the fp32 group input, the next ones the pair, in
    place.  hi is h to bf16 precision and the pair keeps h to 16 significant bits
    (2^-16 rel-L2) over a chain of adds."""
    d = dev()
    N, H, W, Cc, R = 2, 48, 48, 64, 2
    g = torch.Generator(device="cpu").manual_seed(8)
    w1 = (torch.randn(Cc // R, Cc, generator=g) * 0.1).to(d)
    b1 = (torch.randn(Cc // R, generator=g) * 0.1).to(d)
    w2 = (torch.randn(Cc, Cc // R, generator=g) * 0.1).to(d)
    b2 = (torch.randn(Cc, generator=g) * 0.1).to(d)
    ns = call("srmi_conv3x3_nstrips", H, W)
    h_in = torch.randn(N, H, W, Cc, generator=g).to(d)
    h_ref = h_in.double().cpu()
    hi = [torch.empty(N, H, W, Cc, dtype=torch.bfloat16, device=d) for _ in range(2)]
    lo = torch.empty(N, H, W, Cc, dtype=torch.uint8, device=d)
    rec = torch.empty(N, 160, device=d)
    for step in range(6):
        u = bf(torch.randn(N, H, W, Cc, generator=g)).to(d)
        part = torch.zeros(N, ns, Cc, device=d)
        part[:, 0, :] = u.float().sum((1, 2))
        first = step == 0
        call("srmi_ca_forward_pair", ptr(u), ptr(part), ns, ptr(w1), ptr(b1), ptr(w2), ptr(b2), N, H * W, Cc, R,
             ptr(h_in if first else None), ptr(None if first else hi[(step + 1) % 2]), ptr(None if first else lo),
             ptr(hi[step % 2]), ptr(lo), ptr(rec), S())
        torch.cuda.synchronize()
        m = u.double().cpu().mean((1, 2))
        s = torch.sigmoid(torch.relu(m @ w1.double().cpu().T + b1.double().cpu()) @ w2.double().cpu().T + b2.double().cpu())
        h_ref = h_ref + u.double().cpu() * s[:, None, None, :]
        got = lo8_decode(hi[step % 2], lo)
        # the pair keeps h to within 128 fp32 steps of its binade: a rounding error of
        # 2^-16 of each element (the fp32 arithmetic of the adds is in the same range)
        assert rel_l2(got, h_ref) < 2 ** -16
        assert float((got - h_ref).abs().max()) <= 2 ** -14 * float(h_ref.abs().max())
        # hi is within half a bf16 ulp (plus lo's rounding) of h: the conv operand
        assert rel_l2(hi[step % 2], h_ref) < 2 ** -8


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


def test_downsample_upsample_beyond_grid_y_planes():
    """N * C above the 65535 grid.y limit (a large batch of tiles x channels): the
    resampling kernels stride over the planes instead of refusing the shape; every
    plane equals the same plane resampled in a small batch, bit for bit."""
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(7)
    n = 70001
    x = torch.randn(n, 1, 8, 8, generator=g).to(d)
    y = torch.empty(n, 1, 2, 2, device=d)
    call("srmi_downsample", ptr(x), n, 1, 8, 8, 4, ptr(y), S())
    up = torch.empty(n, 1, 8, 8, device=d)
    call("srmi_upsample", ptr(y), n, 1, 2, 2, 4, ptr(up), S())
    for sl in (slice(0, 3), slice(65534, 65537), slice(n - 3, n)):
        ys = torch.empty(3, 1, 2, 2, device=d)
        call("srmi_downsample", ptr(x[sl].contiguous()), 3, 1, 8, 8, 4, ptr(ys), S())
        us = torch.empty(3, 1, 8, 8, device=d)
        call("srmi_upsample", ptr(ys), 3, 1, 2, 2, 4, ptr(us), S())
        torch.cuda.synchronize()
        assert torch.equal(y[sl], ys) and torch.equal(up[sl], us)


INTERP_CASES = ["down_linear_4", "down_linear_8", "down_linear_3", "down_linear_1p5", "down_cubic_3",
                "down_cubic_1p5", "down_cubic_6", "up_linear_4", "up_linear_4b"]


@pytest.mark.parametrize("case", INTERP_CASES)
def test_interpolate_modes_match_reference(case):
    """srmi_interpolate (through srmi.engine.downsample / upsample) against the
    reference's own downsample / upsample under task.downsample_mode /
    upsample_mode 'linear' / 'cubic' (array.py:37-41, :72-76, :84-87) at the model
    scale and at odd / fractional data_downsample factors: golden vectors of
    tests/golden/make_golden_interp.py (fp64 reference on the fp32 inputs)."""
    import os
    from oracle import rcan_oracle as ro
    from srmi.engine import downsample, upsample
    d = dev()
    gd = np.load(os.path.join(os.path.dirname(__file__), "golden", "interp.npz"))
    B, C, T = (int(v) for v in gd[f"{case}_shape"][:3])
    x = ro.synthetic_hr(B, C, T, int(gd[f"{case}_seed"]))
    assert abs(x.astype(np.float64).sum() - float(gd[f"{case}_in_sum"])) < 1e-6
    sf = float(gd[f"{case}_sf"])
    mode = "bilinear" if "linear" in case else "bicubic"
    xt = torch.tensor(x).to(d)
    y = downsample(xt, sf, mode=mode) if case.startswith("down") else upsample(xt, int(sf), mode=mode)
    torch.cuda.synchronize()
    ref = gd[f"{case}_out"]
    assert tuple(y.shape) == ref.shape
    np.testing.assert_allclose(y.double().cpu().numpy(), ref, rtol=1e-5, atol=2e-6)


def test_batch_losses_beyond_1024_tiles_one_batch():
    """Per-tile sums of more than 1024 tiles (a multi-rank tiled-inference rank's
    share, srmi.inference._process_region_ranks): one batch of all tiles keeps the
    mean pass within its 1024-batch bound while `work` holds every tile's sum."""
    d = dev()
    n, te = 1500, 48
    g = torch.Generator(device="cpu").manual_seed(3)
    y = torch.randn(n, te, generator=g).to(d)
    t = torch.randn(n, te, generator=g).to(d)
    work = torch.zeros(n, device=d)
    out = torch.zeros(2, device=d)
    call("srmi_batch_losses", ptr(y), ptr(t), n, te, n, _lib.SRMI_LOSS_RMSE, 1e-6, ptr(work), ptr(out), S())
    torch.cuda.synchronize()
    ref = ((y.double() - t.double()) ** 2).sum(dim=1)
    assert rel_l2(work, ref) < 1e-6
    assert abs(float(out[0]) - math.sqrt(float(ref.sum()) / (n * te))) < 1e-5
    with pytest.raises(_lib.SrmiError):  # batches of one tile exceed the bound
        call("srmi_batch_losses", ptr(y), ptr(t), n, te, 1, _lib.SRMI_LOSS_RMSE, 1e-6, ptr(work), ptr(out), S())


@pytest.mark.parametrize("te", [50, 4 * (2 * 4096 + 777)])  # the scalar kernel; the float4 one past its unrolled loop
@pytest.mark.parametrize("kind", [0, 1])
def test_tile_loss_sums_both_kernels(te, kind):
    d = dev()
    n = 7
    g = torch.Generator(device="cpu").manual_seed(5)
    y = torch.randn(n, te, generator=g).to(d)
    t = torch.randn(n, te, generator=g).to(d)
    work = torch.zeros(n, device=d)
    out = torch.zeros(1 + n, device=d)
    call("srmi_batch_losses", ptr(y), ptr(t), n, te, 1, kind, 1e-6, ptr(work), ptr(out), S())
    torch.cuda.synchronize()
    dd = y.double() - t.double()
    ref = (dd * dd).sum(dim=1) if kind == 0 else torch.sqrt(dd * dd + 1e-6).sum(dim=1)
    assert rel_l2(work, ref) < 1e-6


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


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("C,H,W", [(1, 8, 192), (2, 12, 192), (4, 8, 256), (3, 4, 96), (2, 192, 288), (3, 192, 256)])
def test_tail_forward(C, H, W, dt):
    """Tail conv 64 -> C (network.py:16 / EDSR tail) through srmi_tail_forward: bf16 =
    MFMA implicit GEMM with bf16 operands (and bf16 filters) vs an fp64 conv of the
    same bf16 input; fp32 = the exact fp32 form.  The two large shapes have more
    strips (576, 768) than the persistent bf16 grid has workgroups (512), so each
    workgroup walks several strips with the next strip's halo prefetched."""
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(12)
    N = 2
    x = op(torch.randn(N, H, W, 64, generator=g), dt).to(d)
    w = (torch.randn(C, 64, 3, 3, generator=g) * 0.05).to(d)
    b = (torch.randn(C, generator=g) * 0.1).to(d)
    y = torch.empty(N, C, H, W, device=d)
    call("srmi_tail_forward", ptr(x), ptr(w), ptr(b), N, C, H, W, ptr(y), ABI_DT[dt], S())
    ref = Fn.conv2d(nchw(x).double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
    assert rel_l2(y, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTS)
def test_head_forward(dt):
    """Head conv C -> 64 (network.py:13): fp32 arithmetic, fp32 stream + operand copy."""
    d = dev()
    g = torch.Generator(device="cpu").manual_seed(13)
    N, C, H, W = 2, 3, 48, 48
    lr = torch.randn(N, C, H, W, generator=g).to(d)
    w = (torch.randn(64, C, 3, 3, generator=g) * 0.2).to(d)
    b = (torch.randn(64, generator=g) * 0.1).to(d)
    x0f = torch.empty(N, H, W, 64, device=d)
    x0b = torch.empty(N, H, W, 64, dtype=TORCH_DT[dt], device=d)
    call("srmi_head_forward", ptr(lr), ptr(w), ptr(b), N, C, H, W, ptr(x0f), ptr(x0b), ABI_DT[dt], S())
    ref = nhwc(Fn.conv2d(lr.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1))
    assert rel_l2(x0f, ref) < 1e-6
    assert rel_l2(x0b.float(), ref) < TOL[dt]
