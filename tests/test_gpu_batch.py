"""Device batch preparation (srmi_batch_prep through the C ABI) against the
oracle's restatement of norm 'lnorm' + xyflip + downsample (SURVEY.md §8f row 2;
xyflip pinned by the reference's golden vectors in test_batch_oracle.py).
Tolerance (kernel: fp64 statistics, fp32 outputs; oracle fp64): 1e-6 absolute
on the unit-variance HR tiles (fp32 rounding), 4e-6 on the fp32-filtered LR
tiles, 1e-6 relative on mean / std."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import rcan_oracle as ro  # noqa: E402
from srmi._lib import SrmiError  # noqa: E402
from srmi.batch import prep_batch  # noqa: E402
from srmi.engine import downsample  # noqa: E402


def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def _raw(B, C, T, seed):
    rng = np.random.RandomState(seed)
    # climate-like: large offset per channel, O(1) variability, one smooth ramp
    ramp = np.linspace(-2, 2, T)[None, None, :, None] * np.linspace(0, 1, T)[None, None, None, :]
    return (rng.randn(B, C, T, T) + 3 * ramp + 280.0 + 10 * np.arange(C)[None, :, None, None]).astype(np.float32)


def _check(raw, f, scale):
    d = dev()
    out = prep_batch(torch.tensor(raw, device=d), f, scale)
    torch.cuda.synchronize()
    hr, lr, mean, std = ro.prep_batch(raw.astype(np.float64), f, scale)
    np.testing.assert_allclose(out["hr"].cpu().numpy(), hr, atol=1e-6, rtol=0)
    np.testing.assert_allclose(out["lr"].cpu().numpy(), lr, atol=4e-6, rtol=0)
    np.testing.assert_allclose(out["mean"].cpu().numpy()[:, :, 0, 0], mean, rtol=1e-6)
    np.testing.assert_allclose(out["std"].cpu().numpy()[:, :, 0, 0], std, rtol=1e-6)
    assert out["xyflip"] == f
    # the fused LR equals srmi's own downsample of the fused HR to fp32 rounding
    lr2 = downsample(out["hr"], scale)
    torch.cuda.synchronize()
    assert float((out["lr"] - lr2).abs().max()) < 1e-6
    return out


@pytest.mark.parametrize("f", range(8))
def test_batch_prep_all_flips(f):
    _check(_raw(3, 2, 48, 10 + f), f, 4)


def test_batch_prep_c2_shape_lds_path():
    # BASELINE C2 tiles: 192^2 HR, 2 channels (the LDS-resident path)
    _check(_raw(16, 2, 192, 1), 6, 4)


def test_batch_prep_edsr_x8_global_path():
    # C4 tiles: 256^2 HR, 4 channels, scale 8 (too big for LDS -> L2 path)
    _check(_raw(2, 4, 256, 2), 3, 8)


def test_batch_prep_ragged_row_and_no_lr():
    # T % 4 == 2: float4 loads straddle rows
    d = dev()
    raw = _raw(2, 1, 10, 3)
    out = prep_batch(torch.tensor(raw, device=d), 5, 4, with_lr=False)
    hr = ro.xyflip(ro.lnorm(raw.astype(np.float64)), 5)
    np.testing.assert_allclose(out["hr"].cpu().numpy(), hr, atol=1e-6, rtol=0)
    assert "lr" not in out


def test_batch_prep_deterministic_and_batch_invariant():
    d = dev()
    raw = torch.tensor(_raw(8, 2, 192, 4), device=d)
    a = prep_batch(raw, 2, 4)
    b = prep_batch(raw, 2, 4)
    c = prep_batch(raw[3:5].contiguous(), 2, 4)
    torch.cuda.synchronize()
    for k in ("hr", "lr", "mean", "std"):
        assert torch.equal(a[k], b[k])
        assert torch.equal(a[k][3:5], c[k])


def test_batch_prep_rejects_bad_args():
    d = dev()
    raw = torch.zeros(1, 1, 48, 48, device=d)
    with pytest.raises(SrmiError):
        prep_batch(raw, 8, 4)
    with pytest.raises(SrmiError):
        prep_batch(torch.zeros(1, 1, 50, 50, device=d), 0, 4)  # 50 % 4
    with pytest.raises(ValueError):
        prep_batch(torch.zeros(1, 1, 48, 40, device=d), 0, 4)
