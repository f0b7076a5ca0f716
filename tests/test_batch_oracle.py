"""CPU checks of the batch-preparation restatement:
oracle.xyflip against golden vectors produced by the reference's own xyflip
(sres/base/source/batch.py:37-49, tests/golden/make_golden_batch.py), and
prep_batch's lnorm/downsample composition (lnorm pinned by restatement: the
reference's norm() needs xarray)."""
import os
import random

import numpy as np
import torch

from oracle import rcan_oracle as ro
from srmi.batch import xyflip_index


def test_xyflip_matches_reference_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "xyflip.npz"))
    x = g["input"]
    for f in range(8):
        np.testing.assert_array_equal(ro.xyflip(x, f), g[f"flip{f}"])
        assert int(g[f"attr{f}"]) == f
    np.testing.assert_array_equal(ro.xyflip(x, 0), g["disabled"])
    assert int(g["attr_disabled"]) == 0
    # the 8 variants are the 8 distinct elements of the dihedral group
    assert len({g[f"flip{f}"].tobytes() for f in range(8)}) == 8


def test_prep_batch_oracle_composition():
    rng = np.random.RandomState(3)
    raw = rng.randn(3, 2, 16, 16) * 4 + 280.0
    for f in (0, 5, 7):
        hr, lr, mean, std = ro.prep_batch(raw, f, 4)
        assert hr.shape == raw.shape and lr.shape == (3, 2, 4, 4)
        np.testing.assert_allclose(hr.mean(axis=(2, 3)), 0, atol=1e-12)
        np.testing.assert_allclose(hr.std(axis=(2, 3)), 1, atol=1e-12)
        np.testing.assert_allclose(mean, raw.mean(axis=(2, 3)), rtol=1e-14)
        # lr is the reference's bicubic downsample of the flipped target
        ref_lr = ro.downsample(torch.tensor(hr), 4).numpy()
        np.testing.assert_allclose(lr, ref_lr, atol=1e-12)


def test_xyflip_index_draw():
    assert xyflip_index(False) == 0
    r = random.Random(5)
    draws = [xyflip_index(True, r) for _ in range(400)]
    assert set(draws) == set(range(8))
