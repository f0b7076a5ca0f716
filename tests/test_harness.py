"""Host-side checks of the training harness (srmi.harness) and the loss semantics
of the oracle: CheckpointManager file layout with its .backup copy
(sres/controller/checkpoints.py:18-67), ResultsAccumulator CSV rows
(sres/model/manager.py:103-112, :208-212), evaluate's validation-checkpoint policy
(sres/controller/dual_trainer.py:534-539), TileBatchIterator order
(sres/data/tiles.py:48-74) and the per-batch loss means (dual_trainer.py:443-446)."""
import csv
import os
import random

import numpy as np
import pytest
import torch

from oracle import rcan_oracle as ro


class _FakeTrainer:
    def __init__(self, v):
        self.v = v
        self.loaded = None

    def checkpoint(self, epoch=0, itime=0, loss=0.0):
        return dict(epoch=epoch, itime=itime, model_state_dict={"w": torch.tensor([self.v])},
                    optimizer_state_dict={"state": {}, "param_groups": []}, loss=loss)

    def load_checkpoint(self, state):
        self.loaded = state


def test_checkpoint_store_paths_backup_and_load(tmp_path):
    from srmi.harness import CheckpointStore
    st = CheckpointStore(str(tmp_path), "sres-rcan-10-20-64-swot-SST-tiles-48")
    assert st.path("train").endswith("checkpoints/sres-rcan-10-20-64-swot-SST-tiles-48.train.pt")
    assert st.path("validation").endswith(".valid.pt") and st.path("test") == st.path("valid")
    assert st.path("train", backup=True).endswith(".train.backup.pt")
    assert st.load(_FakeTrainer(0.0), "train") == {}
    st.save(_FakeTrainer(1.0), 1, 0, "train", 0.5)
    assert not os.path.exists(st.path("train", backup=True))
    st.save(_FakeTrainer(2.0), 1, 1, "train", 0.4)
    bk = torch.load(st.path("train", backup=True), weights_only=True)
    cur = torch.load(st.path("train"), weights_only=True)
    assert float(bk["model_state_dict"]["w"]) == 1.0 and float(cur["model_state_dict"]["w"]) == 2.0
    tr = _FakeTrainer(0.0)
    s = st.load(tr, "train", update_model=True)
    assert s == {"epoch": 1, "itime": 1, "loss": 0.4} and tr.loaded is not None
    with open(st.path("valid"), "wb") as f:
        f.write(b"not a checkpoint")
    assert st.load(tr, "valid") is None  # unreadable -> None (checkpoints.py:45-48)
    st.clear()
    assert not os.path.exists(st.path("train"))


def test_loss_records_csv_format(tmp_path):
    from srmi.harness import LossRecords
    r = LossRecords(str(tmp_path), "swot", "SSS_SST-tiles-48", "rcan-10-20-64")
    assert r.result_file_path().endswith("SSS_SST-tiles-48_result_recs/swot_SSS_SST-tiles-48_rcan-10-20-64_losses.csv")
    r.record_losses("train", 0.0, 0.123456789, 0.5)
    r.record_losses("validation", 1.0 / 3.0, 0.1, 0.25, flush=True)
    r.record_losses("train", 2.0, 0.05, 0.2)
    r.flush()
    with open(r.result_file_path(), newline="") as f:
        rows = list(csv.reader(f))
    assert rows == [["train", "0.000", "0.123457", "0.500000"], ["valid", "0.333", "0.100000", "0.250000"],
                    ["train", "2.000", "0.050000", "0.200000"]]
    assert r.load_results() == rows
    r.refresh_state()
    assert r.load_results() == []


def test_validation_checkpoint_policy():
    from srmi.harness import ValidationCheckpoint
    saved = []
    v = ValidationCheckpoint()
    save = lambda m, i: saved.append((m, i))  # noqa: E731
    assert v.update(0.5, 0.9, save) and saved == [(0.5, 0.9)]  # first evaluation: inf -> save
    assert not v.update(0.6, 0.9, save) and v.validation_loss == 0.5
    assert v.update(0.4, 0.9, save) and v.validation_loss == 0.4
    assert not v.update(0.3, 0.9, save, update_checkpoint=False) and v.validation_loss == 0.3
    z = ValidationCheckpoint(0.0)  # a zero best loss: always replaced, never saved
    assert not z.update(0.7, 0.9, save) and z.validation_loss == 0.7


def test_batch_starts_tilebatchiterator():
    from srmi.harness import batch_starts
    assert batch_starts(100, 36, False) == [0, 36, 72]
    s = batch_starts(100, 36, True, random.Random(3))
    assert sorted(s) == [0, 36, 72]


def test_unknown_loss_fn_raises():
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer
    with pytest.raises(ValueError, match="Unknown single-product loss function"):
        FusedTrainer(NetSpec(), 2, loss_fn="l1", device=torch.device("cpu"))


def test_oracle_batch_loss_mean_and_evaluate():
    model = ro.RCANOracle(nchannels_in=1, nchannels_out=1, nlayers=1, nblocks=1).double()
    ro.init_params_numpy(model, 3)
    rng = np.random.RandomState(4)
    region = rng.randn(1, 2 * 32, 3 * 32)
    imgs, l = ro.process_region(model, region, 32, 32, 4, batch_size=4)
    assert len(l["batch_model"]) == 2
    assert abs(l["model"] - np.mean(l["batch_model"])) < 1e-15
    region2 = rng.randn(1, 2 * 32, 3 * 32)
    res, le = ro.evaluate(model, [region2, region], 32, 32, 4, batch_size=4)
    # results = the last time slice's tiles only (clear_results per slice, dual_trainer.py:505)
    assert res["model"].shape == (6, 1, 32, 32)
    np.testing.assert_array_equal(res["model"], ro.evaluate(model, [region], 32, 32, 4, batch_size=4)[0]["model"])
    res, le = ro.evaluate(model, [region, region], 32, 32, 4, batch_size=4)
    assert abs(le["model"] - l["model"]) < 1e-12  # same batches twice: same mean
    # time_index / tile_index selection (dual_trainer.py:487-488, :504-527, tile_in_batch :366-372)
    r1, l1 = ro.evaluate(model, [region2, region], 32, 32, 4, batch_size=4, time_index=1)
    np.testing.assert_array_equal(r1["model"], res["model"])
    assert abs(l1["model"] - l["model"]) < 1e-12
    rt, lt = ro.evaluate(model, [region2, region], 32, 32, 4, batch_size=4, time_index=1, tile_index=5)
    assert rt["model"].shape == (2, 1, 32, 32)  # batch [4, 6) of the 6 tiles
    assert abs(lt["model"] - l["batch_model"][1]) < 1e-12
    np.testing.assert_array_equal(rt["model"], res["model"][4:6])
    rb, lb = ro.evaluate(model, [region2, region], 32, 32, 4, batch_size=4, time_index=1, tile_index=0,
                         batch_domain="time")
    assert rb["model"].shape == (4, 1, 32, 32) and abs(lb["model"] - l["batch_model"][0]) < 1e-12
    # every slice scores its matching batch; results are the last slice's
    ra, la = ro.evaluate(model, [region2, region], 32, 32, 4, batch_size=4, tile_index=5)
    _, l2 = ro.process_region(model, region2, 32, 32, 4, batch_size=4)
    assert abs(la["model"] - 0.5 * (l2["batch_model"][1] + l["batch_model"][1])) < 1e-12
    np.testing.assert_array_equal(ra["model"], res["model"][4:6])
    rn, _ = ro.evaluate(model, [region2, region], 32, 32, 4, batch_size=4, tile_index=6)  # no such tile
    assert rn == {}
    # charbonnier (dual_trainer.py:196-198)
    p, t = torch.zeros(2, 3), torch.ones(2, 3)
    assert abs(float(ro.single_product_loss(p, t, "charbonnier")) - np.sqrt(1 + 1e-6)) < 1e-7
    with pytest.raises(Exception):
        ro.single_product_loss(p, t, "l1")
