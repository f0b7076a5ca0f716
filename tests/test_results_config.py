"""CPU tests: the inference result files (sres/data/inference.py:10-50), the
ConfigContext identity keys (sres/base/util/config.py:51, :82-84) that name the
checkpoint and loss-history files, and the fused trainer's refusal of the
apply_network features it does not implement (dual_trainer.py:557-571).

The NetCDF layout's parity against xarray's own writer is unpinned (xarray and
netCDF4 are not installed); what is tested is the reference's naming, variable /
dimension / coordinate layout and a scipy round trip."""
import os

import numpy as np
import pytest
import torch

from srmi import results as R
from srmi.config import ConfigContext, cfg, check_fused_task, data_downsample_factor
from srmi.harness import CheckpointStore, LossRecords


def test_results_path_naming(tmp_path):
    root = str(tmp_path)
    p = R.results_path(root, "swot", "SST-tiles-48", "SST", 3, "image")
    assert p == f"{root}/inference/swot/SST-tiles-48/SST-3.image.nc"
    assert os.path.isdir(os.path.dirname(p))
    p = R.results_path(root, "swot", "SST-tiles-48", "SST", 3, "tiles", data_downsample=2)
    assert p.endswith("/SST-3.tiles_ds-2.00.nc")
    with pytest.raises(ValueError):
        R.results_path(root, "swot", "t", "SST", 0, "mosaic")
    open(R.results_path(root, "swot", "t", "SST", 7, "tiles"), "w").close()
    open(R.results_path(root, "swot", "t", "SST", 12, "tiles"), "w").close()
    assert sorted(R.time_indices(root, "swot", "t", "SST", "tiles")) == [7, 12]


def test_image_results_round_trip(tmp_path):
    rng = np.random.RandomState(0)
    C, H, W, s = 2, 2 * 192, 3 * 192, 4
    images = {"input": rng.randn(C, H // s, W // s).astype(np.float32),
              "target": rng.randn(C, H, W).astype(np.float32),
              "interpolated": rng.randn(C, H, W).astype(np.float32),
              "model": rng.randn(C, H, W).astype(np.float32)}
    images["model"][1, :192, :192] = np.nan  # a dropped tile
    per_var = R.image_results(images, ["SSS", "SST"])
    losses = {"model": 0.125, "interpolated": 0.5}
    path = R.save_inference_results(R.results_path(str(tmp_path), "swot", "SSS_SST-tiles-48", "SST", 0, "image"),
                                    per_var["SST"], losses)
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as f:
        assert f.version_byte == 2
        assert f.variables["input"].dimensions == ("ys", "xs")
        for k in ("target", "interpolated", "model"):
            assert f.variables[k].dimensions == ("y", "x")
        assert f.dimensions["ys"] == H // s and f.dimensions["x"] == W
        np.testing.assert_allclose(f.variables["y"][:], np.arange(0.0, 100.0, 100.0 / H))
        np.testing.assert_allclose(f.variables["ys"][:], np.arange(0.0, 100.0, 100.0 / (H // s)))
        assert np.isnan(f.variables["model"]._FillValue)
    back, bl = R.load_inference_results(path)
    assert bl == losses
    assert back["input"].dims == ("y", "x")
    for k, v in images.items():
        np.testing.assert_array_equal(back[k].values, v[1].astype(np.float64))
    assert np.isnan(back["model"].values[:192, :192]).all()


@pytest.mark.parametrize("nvars", [1, 2])
def test_tiles_results_round_trip(tmp_path, nvars):
    rng = np.random.RandomState(1)
    n, s = 6, 4
    res = {"input": torch.tensor(rng.randn(n, nvars, 48, 48), dtype=torch.float32)}
    for k in ("target", "model", "interpolated"):
        res[k] = torch.tensor(rng.randn(n, nvars, 192, 192), dtype=torch.float32)
    names = ["SST"] if nvars == 1 else ["SSS", "SST"]
    per_var = R.tiles_results(res, names)
    v = names[-1]
    path = R.save_inference_results(R.results_path(str(tmp_path), "swot", "t", v, 5, "tiles"), per_var[v],
                                    {"model": 1.0, "interpolated": 2.0})
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as f:
        assert f.variables["input"].dimensions == ("tiles", "ys", "xs")
        assert f.variables["model"].dimensions == ("tiles", "y", "x")
        assert f.variables["tiles"].typecode() == "i"  # netCDF-3 has no int64: int32
        if nvars == 1:  # squeeze() keeps channels as a scalar coordinate
            assert b"".join(f.variables["channels"][:].tolist()) == b"SST"
            assert f.variables["model"].coordinates == b"channels"
        else:
            assert "channels" not in f.variables
    back, bl = R.load_inference_results(path)
    assert bl == {"model": 1.0, "interpolated": 2.0}
    for k in res:
        np.testing.assert_array_equal(back[k].values, res[k][:, len(names) - 1].numpy())
    if nvars == 1:
        assert back["model"].scalar_coords["channels"] == "SST"


def test_config_identity_keys_and_derived_paths(tmp_path, monkeypatch):
    """training_version = '-'.join([name, model, dataset, task]) (config.py:51, :84),
    task.name / task.dataset (:82-83); the checkpoint and loss-CSV file names a
    reference run writes (checkpoints.py:60-66, manager.py:185-212)."""
    plat = tmp_path / "cfg" / "platform"
    plat.mkdir(parents=True)
    (plat / "box.yaml").write_text(f'root: "{tmp_path}/data"\nresults: "${{.root}}/results"\n'
                                   "processed: '${.root}/processed'\n")
    monkeypatch.setenv("SRMI_CONFIG_PATH", str(tmp_path / "cfg"))
    conf = dict(model="rcan-10-20-64", task="SSS_SST-tiles-48", dataset="swot", platform="box")
    with ConfigContext("sres", conf) as c:
        assert c.task.training_version == "sres-rcan-10-20-64-swot-SSS_SST-tiles-48"
        assert c.task.name == "SSS_SST-tiles-48" and c.task.dataset == "swot"
        assert c.platform.results == f"{tmp_path}/data/results"
        store = CheckpointStore.from_config()
        assert store.path("train") == f"{tmp_path}/data/results/checkpoints/sres-rcan-10-20-64-swot-SSS_SST-tiles-48.train.pt"
        assert store.path("test", backup=True).endswith("sres-rcan-10-20-64-swot-SSS_SST-tiles-48.valid.backup.pt")
    cc = ConfigContext("sres", conf)
    assert cc.cid == "sres-rcan-10-20-64-swot-SSS_SST-tiles-48"
    with cc:
        rec = LossRecords.from_context(cc)
        assert rec.result_file_path() == (f"{tmp_path}/data/processed/SSS_SST-tiles-48_result_recs/"
                                          "swot_SSS_SST-tiles-48_rcan-10-20-64_losses.csv")


def test_fused_trainer_apply_network_target_selection_and_refusals():
    """apply_network (dual_trainer.py:557-571): data_downsample only acts when > 1
    (any factor: srmi.engine.downsample runs the general F.interpolate kernel for
    the odd / fractional ones); the target is index_selected only when
    the batch has more channels than target_variables, in the INPUT's order
    (np.in1d(channels, targets)); equal counts in another order are a no-op."""
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer
    assert check_fused_task({"data_downsample": 1, "input_variables": {"SST": "x"}, "target_variables": ["SST"]},
                            1, 1) is None
    assert check_fused_task({"data_downsample": 0.5}, 1, 1) is None  # <= 1: a no-op in the reference
    assert check_fused_task({"data_downsample": 2.0}, 1, 1) is None  # the trainer downsamples by 2 first
    assert data_downsample_factor({"data_downsample": 0.5}) == 1
    assert data_downsample_factor({"data_downsample": 4}) == 4
    for ok in (3, 1.5):  # odd and fractional factors: the general interpolation kernel
        assert check_fused_task({"data_downsample": ok}, 1, 1) is None
    with pytest.raises(NotImplementedError, match="subset"):
        check_fused_task({}, 2, 1)
    two = {"input_variables": {"SSS": "a", "SST": "b"}}
    assert check_fused_task(dict(two, target_variables=["SST"]), 2, 1) == [1]
    assert check_fused_task(dict(two, target_variables=["SSS"]), 2, 1) == [0]
    assert check_fused_task(dict(two, target_variables=["SST", "SSS"]), 2, 2) is None  # same set, other order
    with pytest.raises(ValueError):
        check_fused_task(dict(two, target_variables=["SST"]), 2, 2)  # model outputs do not match the target
    with pytest.raises(ValueError):
        check_fused_task(dict(two, target_variables=["U"]), 2, 1)  # selects nothing
    # the trainer checks before it touches a device
    with pytest.raises(NotImplementedError):
        FusedTrainer(NetSpec(nchannels_in=2, nchannels_out=1), 2, device=torch.device("cpu"))
    with pytest.raises(ValueError, match="broadcast"):  # a 2-of-3 target cannot meet the 3-channel interp input
        FusedTrainer(NetSpec(nchannels_in=3, nchannels_out=2), 2, device=torch.device("cpu"),
                     task={"input_variables": ["A", "B", "C"], "target_variables": ["A", "C"]})
    from srmi.inference import TiledInference
    with pytest.raises(ValueError, match="divisible"):  # floor(384 / 5) = 76 is no multiple of the scale 4
        TiledInference(NetSpec(), torch.empty(0), (1, 384, 384), device=torch.device("cpu"),
                       task={"data_downsample": 5})
    with ConfigContext("sres", dict(model="rcan-10-20-64", task="SST-tiles-48"),
                       **{"task.downsample_mode": "nearest"}):
        assert cfg().task.downsample_mode == "nearest"
        with pytest.raises(NotImplementedError):  # (read from the active context)
            FusedTrainer(NetSpec(), 2, device=torch.device("cpu"))


def test_partial_context_has_no_training_version_and_legacy_stem_warns(tmp_path, monkeypatch):
    """A context without a dataset gets no training_version (the reference's join
    raises there), so no checkpoint is named from it; a resume that finds only a
    checkpoint under the pre-round-3 '{cname}-{model}' stem warns instead of
    silently starting over."""
    import warnings as W
    plat = tmp_path / "cfg" / "platform"
    plat.mkdir(parents=True)
    (plat / "box.yaml").write_text(f'root: "{tmp_path}"\nresults: "${{.root}}/results"\n')
    monkeypatch.setenv("SRMI_CONFIG_PATH", str(tmp_path / "cfg"))
    with ConfigContext("sres", dict(model="rcan-10-20-64", task="SST-tiles-48", platform="box")) as c:
        assert "training_version" not in c.task
        with pytest.raises(ValueError, match="training_version"):
            CheckpointStore.from_config()
    conf = dict(model="rcan-10-20-64", task="SST-tiles-48", dataset="swot", platform="box")
    with ConfigContext("sres", conf):
        store = CheckpointStore.from_config()
        old = tmp_path / "results" / "checkpoints" / "sres-rcan-10-20-64.train.pt"
        old.parent.mkdir(parents=True, exist_ok=True)
        old.write_bytes(b"x")
        with pytest.warns(UserWarning, match="pre-round-3"):
            assert store.load(None, "train") == {}
        old.unlink()
        with W.catch_warnings():
            W.simplefilter("error")
            assert store.load(None, "train") == {}
