"""The identity the CA scale (csrc/ca_scale.hpp: ca_scale_finish in the inference RCAB,
conv1's partial means ca_matvec in the training forward) rests on, checked in fp64 on
the CPU: the CALayer's pooled mean of
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
    t's statistics as ca_scale_finish forms them."""
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


def _partial_share(t, w, y0, y1, x0, x1):
    """The share of sum_{tap, ci} W2 S_tap of the rows y0..y1-1 and columns x0..x1-1 of t,
    as one conv1 workgroup forms it in the training forward (conv64_body, SRMI_CA_MPART):
    T over its tile, the image's column 0 / W-1 restricted to its rows (only when its
    tile holds them), rows 0 / H-1 and the corners only where its tile holds them."""
    C, H, W = t.shape
    tile = t[:, y0:y1, x0:x1]
    T = tile.sum(axis=(1, 2))
    z = np.zeros(C)
    row0 = t[:, 0, x0:x1].sum(axis=1) if y0 == 0 else z
    rowH = t[:, H - 1, x0:x1].sum(axis=1) if y1 == H else z
    col0 = t[:, y0:y1, 0].sum(axis=1) if x0 == 0 else z
    colW = t[:, y0:y1, W - 1].sum(axis=1) if x1 == W else z
    corner = {(0, 0): t[:, 0, 0], (0, 1): t[:, 0, W - 1], (1, 0): t[:, H - 1, 0], (1, 1): t[:, H - 1, W - 1]}
    owns = {(0, 0): y0 == 0 and x0 == 0, (0, 1): y0 == 0 and x1 == W, (1, 0): y1 == H and x0 == 0,
            (1, 1): y1 == H and x1 == W}
    a = np.zeros(w.shape[0])
    for ky in range(3):
        for kx in range(3):
            dy, dx = ky - 1, kx - 1
            s = T.copy()
            if dy == -1:
                s -= rowH
            if dy == 1:
                s -= row0
            if dx == -1:
                s -= colW
            if dx == 1:
                s -= col0
            if dy != 0 and dx != 0:
                key = (1 if dy == -1 else 0, 1 if dx == -1 else 0)
                if owns[key]:
                    s += corner[key]
            a += w[:, :, ky, kx] @ s
    return a


@pytest.mark.parametrize("C,H,W,tw,rows_per_run", [(64, 48, 48, 48, 12), (8, 48, 96, 48, 16), (5, 12, 6, 3, 4),
                                                   (4, 8, 48, 48, 8)])
def test_pooled_mean_from_partial_shares(C, H, W, tw, rows_per_run):
    """The training forward's partial means: each conv1 workgroup's share (its rows of
    one column tile) summed over the image's workgroups gives the same mean (linearity);
    one run covering the whole image is the inference form."""
    rng = np.random.RandomState(C * H + W)
    t = np.maximum(rng.randn(C, H, W), 0.0)
    w = rng.randn(C, C, 3, 3) / np.sqrt(9 * C)
    b = rng.randn(C)
    total = np.zeros(C)
    for x0 in range(0, W, tw):
        for y0 in range(0, H, rows_per_run):
            total += _partial_share(t, w, y0, min(H, y0 + rows_per_run), x0, min(W, x0 + tw))
    np.testing.assert_allclose(b + total / (H * W), _stats_mean(t, w, b), rtol=1e-12, atol=1e-12)
