"""CPU checks of the tiled-inference restatement (oracle/rcan_oracle.py:
region_to_tiles / assemble / process_region) against direct slicing of the
reference's semantics (raw.py:216-233 tile order, dual_trainer.py:482-512 mosaic)."""
import numpy as np
import torch

from oracle import rcan_oracle as ro


def test_tile_order_and_round_trip():
    rng = np.random.RandomState(0)
    region = rng.randn(1, 2 * 8 + 3, 3 * 6 + 5)  # floor tiling drops the ragged edge
    tiles, mean, std, ids, grid = ro.region_to_tiles(region, 8, 6)
    assert grid == (2, 3) and list(ids) == list(range(6))
    for tid in ids:
        y, x = tid // 3, tid % 3
        raw = region[0, y * 8:(y + 1) * 8, x * 6:(x + 1) * 6]
        np.testing.assert_allclose(tiles[tid, 0], (raw - raw.mean()) / raw.std(), atol=1e-12)
    back = ro.assemble(tiles, mean, std, ids, grid)
    np.testing.assert_allclose(back, region[:, :16, :18], atol=1e-12)


def test_nonfinite_tiles_dropped_and_nan_in_mosaic():
    rng = np.random.RandomState(1)
    region = rng.randn(1, 16, 18)
    region[0, 9, 13] = np.nan  # tile (1, 2) -> id 5
    tiles, mean, std, ids, grid = ro.region_to_tiles(region, 8, 6)
    assert list(ids) == [0, 1, 2, 3, 4]
    img = ro.assemble(tiles, mean, std, ids, grid)
    assert np.isnan(img[0, 8:16, 12:18]).all()
    assert np.isfinite(img[0, :8]).all() and np.isfinite(img[0, 8:16, :12]).all()


def test_process_region_small_model():
    model = ro.RCANOracle(nchannels_in=1, nchannels_out=1, nlayers=1, nblocks=1).double()
    ro.init_params_numpy(model, 3)
    region = np.random.RandomState(2).randn(1, 2 * 32, 3 * 32)
    images, losses = ro.process_region(model, region, 32, 32, 4)
    assert images["input"].shape == (1, 16, 24) and images["model"].shape == (1, 64, 96)
    np.testing.assert_allclose(images["target"], region, atol=1e-12)
    assert losses["interpolated"] > 0 and np.isfinite(losses["model"])
