"""Data parallelism over one node: one process per GPU, torch.distributed with
backend "nccl" (= RCCL over xGMI on ROCm), or "gloo" for the CPU tests.

The reference has no distributed code on its live path; this is
the MI355X-native addition, designed for exact single-process semantics:

* tiles are sharded contiguously: rank r trains on tiles [r*B, (r+1)*B) of the
  global batch (independent samples, no batch statistics anywhere in RCAN);
* the RMSE (sres/controller/stats.py:5-8) is a global-batch quantity:
  L = sqrt(S / N_global) with S = sum over ranks of the local sums of squares,
  so ONE scalar all-reduce of S happens before backward and every rank uses
  dL/dy = (y - t) / (N_global * L) -- averaging per-rank RMSEs would not be
  the single-process gradient;
* parameter gradients are then SUMMED over ranks (no 1/world factor: the
  global count already normalises), bucket by bucket in the order backward
  finalises them (one bucket per residual group, tail/upsampler first, head
  last), each bucket's all-reduce launched right behind the backward stage that
  finalises it, overlapping with the rest of backward (GradReducer).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    force: bool = False  # diagnostic: the data-parallel machinery with a single rank

    @property
    def enabled(self) -> bool:
        return self.world > 1 or self.force


def init_from_env(backend: Optional[str] = None, force: bool = False) -> DistInfo:
    """force: run the DP path (process group, reducer stream, bucketed all-reduce)
    even at world size 1 -- measures its on-GPU cost without a second GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 and not force:
        return DistInfo()
    if world <= 1:
        os.environ.setdefault("MASTER_PORT", "29511")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return DistInfo(rank, world, local, force=force and world <= 1)


def shard_range(global_batch: int, info: DistInfo, rank: Optional[int] = None) -> Tuple[int, int]:
    """Contiguous tile shard [a, b) of this rank.  A batch that does
    not divide (the short last batch of a time slice, TileBatchIterator,
    sres/data/tiles.py:55-72) is split as evenly as it goes: the first
    global_batch % world ranks take one tile more, and a rank may get none."""
    if global_batch < 0:
        raise ValueError(f"negative batch {global_batch}")
    r = info.rank if rank is None else rank
    base, rem = divmod(global_batch, info.world)
    a = r * base + min(r, rem)
    return a, a + base + (1 if r < rem else 0)


def shard_capacity(global_batch: int, info: DistInfo) -> int:
    """The largest shard of a global batch (the per-rank trainer batch it needs)."""
    return -(-global_batch // info.world)


def broadcast_ints(values: Sequence[int], info: DistInfo, device: Optional[torch.device] = None) -> List[int]:
    """rank 0's integers on every rank (len(values) must agree across ranks).  RCCL
    needs a device tensor; gloo takes either."""
    if not info.enabled or not values:
        return list(values)
    dev = device if (device is not None and dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor(list(values), dtype=torch.int64, device=dev)
    dist.broadcast(t, 0)
    return [int(x) for x in t.cpu().tolist()]


def barrier(info: DistInfo, device: Optional[torch.device] = None) -> None:
    if info.enabled:
        if dist.get_backend() == "nccl" and device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index if device.index is not None else torch.cuda.current_device()])
        else:
            dist.barrier()


def allreduce_sum_(t: torch.Tensor, info: DistInfo):
    if info.enabled:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def global_rmse_scale(local_sq_sum: torch.Tensor, count_global: float, info: DistInfo):
    """S -> (L, dL/dy scale); local_sq_sum is a 1-element tensor, reduced in place."""
    allreduce_sum_(local_sq_sum, info)
    L = torch.sqrt(local_sq_sum / count_global)
    return L, 1.0 / (count_global * L)


@dataclass
class Bucket:
    ranges: List[Tuple[int, int]]   # (offset, numel) in the flat grad buffer
    # index g of the backward group event that finalises it (None = end of backward):
    # srmi_backward records group_events[g] once residual group g's gradients are
    # final (include/srmi.h), walking g from nlayers-1 down to 0
    event_index: Optional[int]


def grad_buckets(table, arch: str, nlayers: int) -> List[Bucket]:
    """Partition the flat gradient into buckets in backward-completion order: residual
    group nlayers-1 (with the tail / upsampler / body-tail parameters, finalised
    before it) first, group 0 last but one, the head last."""
    def ranges_where(pred):
        out = []
        for name, off, n, _ in table:
            if pred(name):
                if out and out[-1][0] + out[-1][1] == off:
                    out[-1] = (out[-1][0], out[-1][1] + n)
                else:
                    out.append((off, n))
        return out

    buckets: List[Bucket] = []
    tailish = lambda nm: nm.startswith("tail.") or nm.startswith(f"body.{nlayers}.")
    if arch == "rcan":
        for g in range(nlayers - 1, -1, -1):
            rg = ranges_where(lambda nm, g=g: nm.startswith(f"body.{g}."))
            if g == nlayers - 1:
                rg = ranges_where(tailish) + rg
            buckets.append(Bucket(rg, g))
        buckets.append(Bucket(ranges_where(lambda nm: nm.startswith("head.")), None))
    else:
        buckets.append(Bucket(ranges_where(lambda nm: not nm.startswith("head.")), None))
        buckets.append(Bucket(ranges_where(lambda nm: nm.startswith("head.")), None))
    return buckets


def bucket_stage(b: Bucket, nlayers: int, nstages: int) -> int:
    """The backward stage (srmi_backward_stages) after which bucket b is final: residual
    group g is stage nlayers - g; the head bucket (and EDSR's) the last stage."""
    return nlayers - b.event_index if b.event_index is not None else nstages - 1


class GradReducer:
    """Bucketed SUM all-reduce of the flat gradient buffer, overlapped with backward.

    Two schedules (srmi.trainer.FusedTrainer):
    * staged (the default; `reduce_stage`): the trainer enqueues the engines' backward
      stage by stage and, behind the stage that finalises a bucket, the bucket's
      gradient add and all-reduce on the last engine's stream -- no stream of the
      reducer's own;
    * event-driven (`reduce`; stream=True): the whole backward is enqueued first and a
      communication stream of the reducer's own waits for each group's HIP event."""

    def __init__(self, table, arch: str, nlayers: int, info: DistInfo, device: torch.device, stream: bool = True):
        self.info = info
        self.nlayers = nlayers
        self.buckets = grad_buckets(table, arch, nlayers)
        self.n_events = max([b.event_index for b in self.buckets if b.event_index is not None], default=-1) + 1
        self.cuda = device.type == "cuda"
        self.device = device
        self.stream = torch.cuda.Stream(device=device) if self.cuda and stream else None
        self.events = self.new_events() if self.stream is not None else []

    def stage_buckets(self, nstages: int) -> List[List[Bucket]]:
        """Buckets final after each backward stage (srmi_backward_stages)."""
        out: List[List[Bucket]] = [[] for _ in range(nstages)]
        for b in self.buckets:
            out[bucket_stage(b, self.nlayers, nstages)].append(b)
        return out

    def reduce_stage(self, buckets: Sequence[Bucket], grads: torch.Tensor, extra: Sequence[torch.Tensor] = (),
                     works: Optional[list] = None):
        """Enqueue, on the CURRENT stream, the micro-batch gradient adds and the
        asynchronous all-reduce of `buckets` (the caller has made the current stream
        wait for every engine's part of them); the all-reduce handles go to `works`."""
        if not self.info.enabled:
            return
        from .engine import axpy
        for b in buckets:
            for off, n in b.ranges:
                for x in extra:
                    if self.cuda:
                        axpy(grads[off:off + n], x[off:off + n], 1.0)
                    else:
                        grads[off:off + n].add_(x[off:off + n])
                w = dist.all_reduce(grads[off:off + n], op=dist.ReduceOp.SUM, async_op=True)
                if works is not None:
                    works.append(w)
                else:
                    w.wait()

    def covered(self) -> int:
        return sum(n for b in self.buckets for _, n in b.ranges)

    def new_events(self) -> List:
        """One more set of group events (one set per micro-batch engine).

        torch.cuda.Event creates its HIP event lazily on the first torch-side record():
        until then `cuda_event` is NULL, the engine would skip recording it and
        `Stream.wait_event` on it is a no-op -- the bucket all-reduce would not wait
        for backward at all.  So each event is created here by one record on the
        reducer's stream."""
        if not self.cuda or self.stream is None:
            return []
        evs = [torch.cuda.Event() for _ in range(max(self.n_events, 0))]
        for ev in evs:
            ev.record(self.stream)
            if not ev.cuda_event:
                raise RuntimeError("group event was not created")
        return evs

    def reduce(self, grads: torch.Tensor, events_recorded: bool = True, extra: Sequence[torch.Tensor] = (),
               extra_events: Sequence[Sequence] = ()):
        """Call right after the (asynchronous) backward has been enqueued.  With
        events_recorded False (the backward did not record the group events) every
        bucket waits for the current stream.

        extra: gradients of further micro-batch engines (same layout); bucket by
        bucket they are added into `grads` on the communication stream right
        before that bucket's all-reduce, once every engine's group event for it
        (self.events, then extra_events[k]) has fired -- so with micro-batches the
        all-reduce still overlaps the rest of backward.  The caller must not add
        them itself."""
        if not self.info.enabled:
            return
        if not self.cuda:
            for b in self.buckets:
                for off, n in b.ranges:
                    for x in extra:
                        grads[off:off + n].add_(x[off:off + n])
                    dist.all_reduce(grads[off:off + n], op=dist.ReduceOp.SUM)
            return
        from .engine import axpy
        main = torch.cuda.current_stream()
        works = []
        with torch.cuda.stream(self.stream):
            for b in self.buckets:
                if b.event_index is not None and events_recorded:
                    self.stream.wait_event(self.events[b.event_index])
                    for evs in extra_events:
                        self.stream.wait_event(evs[b.event_index])
                else:
                    self.stream.wait_stream(main)
                for off, n in b.ranges:
                    for x in extra:
                        axpy(grads[off:off + n], x[off:off + n], 1.0, stream=self.stream)
                    works.append(dist.all_reduce(grads[off:off + n], op=dist.ReduceOp.SUM, async_op=True))
        for w in works:
            w.wait()
        main.wait_stream(self.stream)
