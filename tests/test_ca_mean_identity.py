"""The identity the one-launch inference RCAB (rcab_infer.hip v2, ca_infer.hpp
ca_scale_from_t) rests on, checked in fp64 on the CPU: the CALayer's pooled mean of
u = conv2(t) + b2 (sres/model/rcan/network.py:44-47, 54-57; same padding) follows
from t's channel totals, its four border lines and four corners, without u:

    mean_p u[c] = b2[c] + (1/HW) sum_{tap, ci} W2[c][ci][tap] S_tap[ci]
    S_tap[ci]   = T[ci] - (row tap (dy, dx) never reads) - (column it never reads)
                        + (their corner)

The GPU tests check the kernel against the three-launch path and the oracle
(tests/test_gpu_inference.py); this pins the algebra itself, shapes included."""
import numpy as np
import pytest
import torch


def _stats_mean(t, w, b):
    """t [C, H, W], w [Co, C, 3, 3], b [Co] -> mean over pixels of conv2(t) + b, from
    t's statistics as ca_scale_from_t forms them."""
    C, H, W = t.shape
    T = t.sum(axis=(1, 2))
    rows = {0: t[:, 0, :].sum(axis=1), H - 1: t[:, H - 1, :].sum(axis=1)}
    cols = {0: t[:, :, 0].sum(axis=1), W - 1: t[:, :, W - 1].sum(axis=1)}
    m = b.astype(np.float64).copy()
    for ky in range(3):
        for kx in range(3):
            dy, dx = ky - 1, kx - 1
            s = T.copy()
            if dy == -1:
                s -= rows[H - 1]  # output row y reads input row y - 1: row H-1 is never read
            if dy == 1:
                s -= rows[0]
            if dx == -1:
                s -= cols[W - 1]
            if dx == 1:
                s -= cols[0]
            if dy != 0 and dx != 0:
                s += t[:, H - 1 if dy == -1 else 0, W - 1 if dx == -1 else 0]
            m += w[:, :, ky, kx] @ s / (H * W)
    return m


@pytest.mark.parametrize("C,H,W", [(64, 48, 48), (8, 4, 48), (5, 7, 3)])
def test_pooled_mean_from_t_statistics(C, H, W):
    rng = np.random.RandomState(C + H + W)
    t = np.maximum(rng.randn(C, H, W), 0.0)  # a ReLU output, as in the RCAB
    w = rng.randn(C, C, 3, 3) / np.sqrt(9 * C)
    b = rng.randn(C)
    u = torch.nn.functional.conv2d(torch.tensor(t)[None], torch.tensor(w), torch.tensor(b), padding=1)[0]
    ref = u.mean(dim=(1, 2)).numpy()
    np.testing.assert_allclose(_stats_mean(t, w, b), ref, rtol=1e-12, atol=1e-12)
