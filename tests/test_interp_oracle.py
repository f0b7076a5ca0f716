"""CPU: the oracle's resampling (F.interpolate with the task's mode) against golden
vectors of the reference's own downsample / upsample under task.downsample_mode /
upsample_mode (tests/golden/make_golden_interp.py, array.py:37-41, :72-76, :84-87),
and the config mapping of those keys (srmi.config.interp_mode)."""
import os

import numpy as np
import pytest
import torch

from oracle import rcan_oracle as ro
from srmi.config import check_fused_task, data_downsample_factor, interp_mode

CASES = ["down_linear_4", "down_linear_8", "down_linear_3", "down_linear_1p5", "down_cubic_3", "down_cubic_1p5",
         "down_cubic_6", "up_linear_4", "up_linear_4b"]


@pytest.mark.parametrize("case", CASES)
def test_oracle_interp_matches_reference_goldens(case):
    gd = np.load(os.path.join(os.path.dirname(__file__), "golden", "interp.npz"))
    B, C, T = (int(v) for v in gd[f"{case}_shape"][:3])
    x = ro.synthetic_hr(B, C, T, int(gd[f"{case}_seed"]))
    assert abs(x.astype(np.float64).sum() - float(gd[f"{case}_in_sum"])) < 1e-6
    mode = "bilinear" if "linear" in case else "bicubic"
    sf = float(gd[f"{case}_sf"])
    t = torch.tensor(x, dtype=torch.float64)
    y = ro.downsample(t, sf, mode) if case.startswith("down") else ro.upsample(t, int(sf), mode)
    np.testing.assert_allclose(y.numpy(), gd[f"{case}_out"], rtol=0, atol=1e-12)


def test_interp_mode_mapping_and_refusals():
    """torch_interp_mode (array.py:37-41): 'linear' -> bilinear, 'cubic' -> bicubic,
    absent -> cubic (every reference task yaml); anything the engine does not run
    raises instead of silently resampling bicubic."""
    assert interp_mode(None, True) == "bicubic"
    assert interp_mode({}, False) == "bicubic"
    assert interp_mode({"downsample_mode": "linear"}, True) == "bilinear"
    assert interp_mode({"downsample_mode": "linear"}, False) == "bicubic"
    assert interp_mode({"upsample_mode": "linear"}, False) == "bilinear"
    assert interp_mode({"upsample_mode": "bicubic"}, False) == "bicubic"
    for bad in ("nearest", "area", "trilinear"):
        with pytest.raises(NotImplementedError, match="mode"):
            interp_mode({"downsample_mode": bad}, True)
        with pytest.raises(NotImplementedError, match="mode"):
            check_fused_task({"upsample_mode": bad}, 1, 1)
    from srmi.engine import NetSpec
    from srmi.inference import TiledInference
    from srmi.trainer import FusedTrainer
    with pytest.raises(NotImplementedError, match="downsample_mode"):  # before any device work
        FusedTrainer(NetSpec(), 2, device=torch.device("cpu"), task={"downsample_mode": "nearest"})
    with pytest.raises(NotImplementedError, match="upsample_mode"):
        TiledInference(NetSpec(), torch.empty(0), (1, 384, 384), device=torch.device("cpu"),
                       task={"upsample_mode": "area"})


def test_data_downsample_any_factor():
    """apply_network's data_downsample (dual_trainer.py:561-563) acts for any value
    > 1 (F.interpolate at scale_factor 1/ds): integers come back as int, other
    factors as float; <= 1 is a no-op."""
    assert data_downsample_factor({"data_downsample": 0.5}) == 1
    assert data_downsample_factor({"data_downsample": 3}) == 3
    assert isinstance(data_downsample_factor({"data_downsample": 3.0}), int)
    assert data_downsample_factor({"data_downsample": 1.5}) == 1.5
    assert check_fused_task({"data_downsample": 3}, 1, 1) is None
