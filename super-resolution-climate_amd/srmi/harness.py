"""The training harness around the fused step: checkpoint cadence, the loss-history
CSV and the validation-checkpoint policy of the reference's ModelTrainer.

* CheckpointStore   <- CheckpointManager (sres/controller/checkpoints.py:11-67):
  ``{results}/checkpoints/{training_version}.{train|valid}.pt`` holding
  ``dict(epoch, itime, model_state_dict, optimizer_state_dict, loss)``, the
  previous file copied to ``...{tset}.backup.pt`` before every save.
* LossRecords       <- ResultsAccumulator (sres/model/manager.py:103-288): rows
  ``[tset, f"{epoch:.3f}", f"{loss:.6f}", f"{ref_loss:.6f}"]`` appended to
  ``{save_dir}/{task}_result_recs/{dataset}_{task}_{model}_losses.csv``.
* ValidationCheckpoint <- the tail of ModelTrainer.evaluate (dual_trainer.py:534-539).
* train_timeslices  <- the epoch / time-slice / tile-batch loops of
  ModelTrainer.train (dual_trainer.py:271-347) around FusedTrainer.step: batches
  of task.batch_size tiles in shuffled order (TileBatchIterator, randomize=True,
  sres/data/tiles.py:48-74), the time-slice loss = mean of the batch losses
  (accumulate_loss, tiles.py:25-28), a train checkpoint after EVERY time slice
  (:330) and a loss record per time slice, flushed every 32 (:275, :331).
  Data parallel (the trainer's DistInfo, world > 1): every rank follows rank 0's
  shuffled batch order, steps its shard of each batch (srmi.dist.shard_range; the
  short last batch too, a rank may get no tile), and only rank 0 writes the
  checkpoint and the loss records while the others wait at a barrier.
"""
from __future__ import annotations

import csv
import math
import os
import random
import shutil
import warnings
from typing import Callable, Dict, List, Optional, Sequence

import torch

TSET_VALUES = {"train": "train", "validation": "valid", "valid": "valid", "test": "test"}
LOSSREC_FLUSH_PERIOD = 32  # dual_trainer.py:275


def _tset(tset: str) -> str:
    try:
        return TSET_VALUES[tset.lower()]
    except KeyError:
        raise ValueError(f"unknown tset {tset!r}") from None


class CheckpointStore:
    """CheckpointManager's files (checkpoints.py:18-67) for a FusedTrainer."""

    def __init__(self, results_dir: str, training_version: str, legacy_version: Optional[str] = None):
        self.results_dir = results_dir
        self.training_version = training_version
        self.legacy_version = legacy_version

    @classmethod
    def from_config(cls, c=None) -> "CheckpointStore":
        """checkpoint_path's inputs (checkpoints.py:60-66): ``cfg().platform.results``
        and ``cfg().task.training_version`` (set by ConfigContext, config.py:84; a
        context missing the model, dataset or task name has none, and the reference's
        ConfigContext raises for it too)."""
        if c is None:
            from .config import cfg
            c = cfg()
        tv = c["task"].get("training_version")
        if tv is None:
            raise ValueError("no task.training_version: the ConfigContext needs model, dataset and task names "
                             "(sres/base/util/config.py:51 joins all four)")
        return cls(str(c["platform"]["results"]), str(tv), c["task"].get("legacy_training_version"))

    def path(self, tset: str, backup: bool = False) -> str:
        v = _tset(tset)
        v = "valid" if v == "test" else v  # checkpoint_path: Test -> Validation (:63)
        p = os.path.join(self.results_dir, "checkpoints", f"{self.training_version}.{v}")
        if backup:
            p += ".backup"
        os.makedirs(os.path.dirname(p), 0o777, exist_ok=True)
        return p + ".pt"

    def save(self, trainer, epoch: int, itime: int, tset: str, loss: float) -> str:
        cpath = self.path(tset)
        if os.path.isfile(cpath):
            shutil.copyfile(cpath, self.path(tset, backup=True))
        torch.save(trainer.checkpoint(epoch=epoch, itime=itime, loss=loss), cpath)
        return cpath

    def load(self, trainer, tset: str = "train", update_model: bool = False) -> Optional[Dict]:
        """load_checkpoint (:34-52): {} when there is no file, None when it cannot be
        loaded, else the train state (model/optimizer dicts popped once applied)."""
        cpath = self.path(tset)
        if not os.path.exists(cpath):
            if self.legacy_version and self.legacy_version != self.training_version:
                v = "valid" if _tset(tset) == "test" else _tset(tset)
                old = os.path.join(self.results_dir, "checkpoints", f"{self.legacy_version}.{v}.pt")
                if os.path.exists(old):
                    warnings.warn(f"no checkpoint {cpath}, but {old} exists under the pre-round-3 name "
                                  f"'{self.legacy_version}': starting from scratch; rename it to resume", stacklevel=2)
            return {}
        try:
            state = torch.load(cpath, map_location="cpu", weights_only=True)
            if update_model:
                trainer.load_checkpoint(state)
                state.pop("model_state_dict")
                state.pop("optimizer_state_dict")
        except Exception:
            return None
        return state

    def clear(self) -> None:
        for t in ("train", "valid"):
            p = self.path(t)
            if os.path.exists(p):
                os.remove(p)


class LossRecords:
    """ResultsAccumulator (manager.py:185-262): buffered records, appended on flush."""

    def __init__(self, save_dir: str, dataset: str, task: str, model: str):
        self.save_dir, self.dataset, self.task, self.model = save_dir, dataset, task, model
        self.results: List[List[str]] = []

    @classmethod
    def from_context(cls, cc, save_dir: Optional[str] = None) -> "LossRecords":
        """ResultsAccumulator(cc) (manager.py:185-191): cc.dataset / cc.task /
        cc.model, save_dir defaulting to ``cfg().platform.processed``."""
        if save_dir is None:
            from .config import cfg
            save_dir = str(cfg()["platform"]["processed"])
        return cls(save_dir, cc.dataset, cc.task, cc.model)

    def result_file_path(self) -> str:
        d = os.path.join(self.save_dir, f"{self.task}_result_recs")
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, f"{self.dataset}_{self.task}_{self.model}_losses.csv")

    @staticmethod
    def serialize(tset: str, epoch: float, loss: float, ref_loss: float) -> List[str]:
        return [_tset(tset), f"{epoch:.3f}", f"{loss:.6f}", f"{ref_loss:.6f}"]  # ResultRecord.serialize

    def record_losses(self, tset: str, epoch: float, loss: float, ref_loss: float, flush: bool = False) -> None:
        self.results.append(self.serialize(tset, epoch, loss, ref_loss))
        if flush:
            self.flush()

    def flush(self) -> None:
        if self.results:
            with open(self.result_file_path(), "a", newline="\n") as f:
                w = csv.writer(f, delimiter=",", quotechar="|", quoting=csv.QUOTE_MINIMAL)
                for r in self.results:
                    w.writerow(r)
        self.results = []

    def refresh_state(self) -> None:
        p = self.result_file_path()
        if os.path.exists(p):
            os.remove(p)

    def load_results(self) -> List[List[str]]:
        p = self.result_file_path()
        if not os.path.exists(p):
            return []
        with open(p, newline="") as f:
            return [row for row in csv.reader(f, delimiter=",", quotechar="|", quoting=csv.QUOTE_MINIMAL)]


class ValidationCheckpoint:
    """evaluate's checkpoint policy (dual_trainer.py:534-539): the validation
    checkpoint is saved when the model loss improves on the best so far (and the
    best so far is not 0); the first evaluation always counts as an improvement."""

    def __init__(self, validation_loss: float = float("inf")):
        self.validation_loss = validation_loss

    def update(self, model_loss: float, interp_loss: float, save: Callable[[float, float], None],
               update_checkpoint: bool = True) -> bool:
        saved = False
        if model_loss < self.validation_loss or self.validation_loss == 0.0:
            if update_checkpoint and self.validation_loss > 0.0:
                save(model_loss, interp_loss)
                saved = True
            self.validation_loss = model_loss
        return saved


def batch_starts(ntiles: int, batch_size: int, randomize: bool, rng: Optional[random.Random] = None) -> List[int]:
    """TileBatchIterator (tiles.py:50-56): start indices 0, bs, 2bs, ... (shuffled)."""
    starts = list(range(0, ntiles, batch_size))
    if randomize:
        (rng or random).shuffle(starts)
    return starts


def train_timeslices(trainer, timeslices: Sequence[Callable[[], torch.Tensor]], nepochs: int, batch_size: int,
                     store: Optional[CheckpointStore] = None, records: Optional[LossRecords] = None,
                     refresh_state: bool = False, rng: Optional[random.Random] = None,
                     on_epoch_end: Optional[Callable[[int, float], None]] = None) -> Dict[str, float]:
    """ModelTrainer.train (dual_trainer.py:271-347) on the fused step.

    timeslices[i]() returns time slice i as normalised HR tiles [ntiles, C, H, W]
    on the device (load_timeslice + the batch preparation, srmi.batch).  Resume
    (refresh_state False) restores the trainer and (epoch0, itime0) from the train
    checkpoint; after every time slice the train checkpoint is saved (with its
    .backup) and the loss record written; on_epoch_end(epoch, loss) stands for
    record_eval (evaluation on the validation set, TiledInference.evaluate).

    Data parallel (trainer.info.world > 1; every rank calls this with the same time
    slices): rank 0 shuffles the batch starts with `rng` -- exactly the order one
    process would use -- and broadcasts them, so the ranks step the same global
    batches; each rank steps its shard_range of every batch with
    trainer.step(tiles, shard=(t0, gb)), so the loss and gradient scale are those of
    the whole batch (srmi.trainer) and a short last batch of gb < world tiles leaves
    some ranks with none.  trainer.batch must hold ceil(batch_size / world) tiles.
    Only rank 0 clears, saves and records; a barrier follows each of its writes."""
    from .dist import DistInfo, barrier, broadcast_ints, shard_capacity, shard_range
    info = getattr(trainer, "info", None) or DistInfo()
    dev = getattr(trainer, "device", None)
    lead = info.rank == 0
    if info.enabled and trainer.batch < shard_capacity(batch_size, info):
        raise ValueError(f"trainer batch {trainer.batch} < the {shard_capacity(batch_size, info)}-tile shard of "
                         f"a {batch_size}-tile batch over {info.world} ranks")
    epoch0, itime0, epoch_loss, interp_l = 1, 0, 0.0, 0.0
    if refresh_state:
        if lead:
            if store is not None:
                store.clear()
            if records is not None:
                records.refresh_state()
        barrier(info, dev)
    elif store is not None:
        state = store.load(trainer, "train", update_model=True)
        if state is None:
            # the reference fails here too (train_state.get on None, dual_trainer.py:287-290);
            # never train from scratch over -- and then back up over -- an unreadable checkpoint
            raise RuntimeError(f"cannot resume: the train checkpoint {store.path('train')} exists but could not be "
                               "loaded into this trainer (refresh_state=True starts over)")
        epoch0 = state.get("epoch", 1)
        itime0 = state.get("itime", 0)
        epoch_loss = state.get("loss", float("inf"))
        nepochs += epoch0
    nts = len(timeslices)
    for epoch in range(epoch0, nepochs):
        for itime in range(itime0, nts):
            tiles = timeslices[itime]()
            ntiles = tiles.shape[0]
            nb = len(range(0, ntiles, batch_size))
            starts = batch_starts(ntiles, batch_size, True, rng) if lead else [0] * nb
            starts = broadcast_ints(starts, info, dev)  # rank 0's order on every rank
            losses, ilosses = [], []
            for start in starts:
                gb = min(batch_size, ntiles - start)
                if info.enabled:
                    a, e = shard_range(gb, info)
                    out = trainer.step(tiles[start + a:start + e], shard=(a, gb))
                else:
                    out = trainer.step(tiles[start:start + gb])
                losses.append(out["loss"].clone())  # (views of the trainer's loss record)
                ilosses.append(out["interp_loss"].clone())
            # accumulate_loss: mean of the batch losses (one host sync per time slice)
            epoch_loss = float(torch.cat(losses).double().mean()) if losses else math.nan
            interp_l = float(torch.cat(ilosses).double().mean()) if ilosses else math.nan
            if lead:
                if store is not None:
                    store.save(trainer, epoch, itime, "train", epoch_loss)
                if records is not None:
                    records.record_losses("train", epoch - 1 + itime / nts, epoch_loss, interp_l,
                                          flush=((itime + 1) % LOSSREC_FLUSH_PERIOD == 0))
            if store is not None:
                barrier(info, dev)  # the checkpoint is complete before any rank goes on
        if on_epoch_end is not None:
            on_epoch_end(epoch, epoch_loss)
        itime0 = 0
    if records is not None and lead:
        records.flush()
    barrier(info, dev)
    return {"prediction": epoch_loss, "interpolated": interp_l}
