"""Fused training step on the native engine.

Restates one iteration of ModelTrainer.train (sres/controller/dual_trainer.py:310-323)
with apply_network (:557-571) for the RCAN/EDSR plugins:

    HR tile batch -> bicubic 1/s (array.py:72-76) -> network -> RMSE (stats.py:5-8)
    [-> interp-baseline RMSE metric, dual_trainer.py:315-318]
    -> backward -> Adam (lr = task.lr, weight_decay = task.weight_decay or 0)

Everything runs asynchronously on one HIP stream: the per-step losses stay on
the device (no .item() sync) until the caller asks for them.
With a DistInfo of world > 1 the batch is this rank's shard and the loss /
gradients are all-reduced as described in srmi/dist.py.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import torch

from . import checkpoint as ckpt
from .dist import DistInfo, GradReducer, allreduce_sum_
from .engine import Engine, NetSpec, adam_step, axpy, downsample, upsample


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def default_init_(flat: torch.Tensor, table, seed: int = 0) -> None:
    """PyTorch's default Conv2d init distribution, U(+-1/sqrt(fan_in)), seeded."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    host = torch.empty(flat.numel(), dtype=torch.float32)
    shapes = {nm: s for nm, _, _, s in table}
    for name, off, n, shape in table:
        ws = shape if name.endswith("weight") else shapes[name[:-4] + "weight"]
        b = 1.0 / math.sqrt(float(math.prod(ws[1:])))
        host[off:off + n].uniform_(-b, b, generator=g)
    flat.copy_(host)


class FusedTrainer:
    """One training step = dual_trainer.py:310-323 on the native engine.

    micro > 1 splits the batch into `micro` equal micro-batches, each with its own
    engine (workspace, filter packs, side stream) on its own HIP stream, launches
    sized for 1/micro of the chip (cu_budget).  RCAN/EDSR have no coupling between
    tiles except the loss scale and the gradient sum, so the step is exact: the
    micro-batches' squared-error partials are added before the RMSE is finalised
    (one global L, as with data parallelism) and their gradients are summed before
    the all-reduce / Adam.  The two streams overlap each layer's launch ramp and
    drain with the other micro-batch's work.
    """

    def __init__(self, spec: NetSpec, batch: int, lr_hw=(48, 48), lr: float = 1e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, interp_loss: bool = True,
                 info: Optional[DistInfo] = None, device: Optional[torch.device] = None, seed: int = 0,
                 params: Optional[torch.Tensor] = None, micro: Optional[int] = None):
        self.info = info or DistInfo()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.spec = spec
        self.batch = batch
        if micro is None:
            micro = 2 if (batch % 2 == 0 and batch >= 16) else 1
        if batch % micro:
            raise ValueError(f"batch {batch} not divisible into {micro} micro-batches")
        self.micro = micro
        # SRMI_DP_FLAT=1: gradients all-reduced once after backward instead of per
        # residual group on the reducer stream overlapped with backward
        self.dp_flat = int(os.environ.get("SRMI_DP_FLAT", "0"))  # 2/3: diagnostic, no grad (3: no) all-reduce
        self.mb = batch // micro
        budget = 256 // micro if micro > 1 else 0
        if micro > 1 and os.environ.get("SRMI_MICRO_BUDGET"):  # diagnostic: CUs each engine's launches aim at
            budget = int(os.environ["SRMI_MICRO_BUDGET"])
        self.engines = [Engine(spec, self.mb, lr_hw, train=True, device=self.device, cu_budget=budget)
                        for _ in range(micro)]
        self.eng = self.engines[0]
        n = self.eng.n_params
        self.params = torch.empty(n, dtype=torch.float32, device=self.device)
        if params is not None:
            self.params.copy_(params)
        else:
            default_init_(self.params, self.eng.table, seed)
        if self.info.enabled:  # identical replicas (rank 0's weights)
            torch.distributed.broadcast(self.params, 0)
        self.grads = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.mgrads = [self.grads] + [torch.zeros(n, dtype=torch.float32, device=self.device)
                                      for _ in range(micro - 1)]
        self.m = torch.zeros_like(self.grads)
        self.v = torch.zeros_like(self.grads)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.t = 0
        self.interp_loss = interp_loss
        C, h, w, s = spec.nchannels_in, lr_hw[0], lr_hw[1], spec.scale
        self.lrbuf = torch.empty((batch, C, h, w), dtype=torch.float32, device=self.device)
        self.sr = torch.empty((batch, spec.nchannels_out, h * s, w * s), dtype=torch.float32, device=self.device)
        self.up = torch.empty_like(self.sr) if interp_loss else None
        self.loss4 = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.iloss4 = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.mloss4 = [torch.zeros(4, dtype=torch.float32, device=self.device) for _ in range(micro)]
        self.miloss4 = [torch.zeros(4, dtype=torch.float32, device=self.device) for _ in range(micro)]
        self.streams = [None] + [torch.cuda.Stream(device=self.device) for _ in range(micro - 1)]
        self.reducer = GradReducer(self.eng.table, spec.arch, spec.nlayers, self.info, self.device)
        # group events of engines 1.. (engine 0 records into reducer.events)
        self.xevents = [self.reducer.new_events() for _ in range(micro - 1)]
        for e in self.engines:
            e.pack(self.params)

    def _ctx(self, k):
        st = self.streams[k]
        return torch.cuda.stream(st) if st is not None else _Null()

    def step(self, hr: torch.Tensor) -> Dict[str, torch.Tensor]:
        """hr: this rank's HR tiles [b, C, H, W] fp32 on the device (already normalised)."""
        b = hr.shape[0]
        if b != self.batch:
            raise ValueError(f"batch {b} != trainer batch {self.batch}")
        s, mb = self.spec.scale, self.mb
        main = torch.cuda.current_stream(self.device)
        count = float(hr.numel()) * self.info.world
        for st in self.streams[1:]:
            st.wait_stream(main)
        # forward + squared-error partials per micro-batch
        for k, eng in enumerate(self.engines):
            sl = slice(k * mb, (k + 1) * mb)
            with self._ctx(k):
                downsample(hr[sl], s, out=self.lrbuf[sl])
                eng.forward(self.params, self.lrbuf[sl], out=self.sr[sl])
                eng.rmse_partial(self.sr[sl], hr[sl], self.mloss4[k], count)
                if self.interp_loss:
                    up = upsample(self.lrbuf[sl], s, out=self.up[sl])
                    eng.rmse_partial(hr[sl], up, self.miloss4[k], count)
        for st in self.streams[1:]:
            main.wait_stream(st)
        self._combine(self.loss4, self.mloss4)
        if self.dp_flat != 3:
            allreduce_sum_(self.loss4[0:1], self.info)
        Engine.rmse_finalize(self.loss4)
        if self.interp_loss:
            self._combine(self.iloss4, self.miloss4)
            if self.dp_flat != 3:
                allreduce_sum_(self.iloss4[0:1], self.info)
            Engine.rmse_finalize(self.iloss4)
        for st in self.streams[1:]:
            st.wait_stream(main)
        # backward per micro-batch with the global loss scale.  Data parallel: every
        # engine records its residual-group events; the reducer adds the engines'
        # gradients bucket by bucket on its stream and all-reduces each bucket as
        # soon as all engines are past it (overlapped with the rest of backward).
        dp = self.info.enabled and self.reducer.cuda and not self.dp_flat
        evs = [self.reducer.events] + self.xevents if dp else [None] * self.micro
        for k, eng in enumerate(self.engines):
            sl = slice(k * mb, (k + 1) * mb)
            with self._ctx(k):
                eng.backward(self.params, self.lrbuf[sl], self.mgrads[k], sr=self.sr[sl], hr=hr[sl],
                             loss4=self.loss4, events=evs[k])
        for st in self.streams[1:]:
            main.wait_stream(st)
        if dp:
            self.reducer.reduce(self.grads, events_recorded=True, extra=self.mgrads[1:], extra_events=self.xevents)
        elif self.dp_flat and self.info.enabled:
            # one flat SUM all-reduce after backward (no reducer stream, no group events)
            for g in self.mgrads[1:]:
                axpy(self.grads, g, 1.0)
            if self.dp_flat == 1:
                allreduce_sum_(self.grads, self.info)
        else:
            for g in self.mgrads[1:]:
                axpy(self.grads, g, 1.0)  # exact gradient of the whole batch
            self.reducer.reduce(self.grads, events_recorded=False)
        self.t += 1
        adam_step(self.params, self.grads, self.m, self.v, self.t, self.lr, self.betas, self.eps, self.wd)
        for k, eng in enumerate(self.engines):
            if k:
                self.streams[k].wait_stream(main)
            with self._ctx(k):
                eng.pack(self.params)
        for st in self.streams[1:]:
            main.wait_stream(st)
        return {"loss": self.loss4[3:4], "interp_loss": self.iloss4[3:4]}

    @staticmethod
    def _combine(dst, parts):
        """loss4 of the whole batch from the micro-batches' partials (sum of squares, count)."""
        if len(parts) == 1:
            dst.copy_(parts[0])
            return
        dst.copy_(parts[0])
        for q in parts[1:]:
            dst[0:1].add_(q[0:1])

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Reference-format model state_dict (CPU copies)."""
        return ckpt.model_state_dict(self.params, self.eng.table)

    def checkpoint(self, epoch: int = 0, itime: int = 0, loss: float = 0.0) -> Dict:
        """What CheckpointManager.save_checkpoint writes (checkpoints.py:18-26): model
        and torch.optim.Adam state dicts in the reference's layouts."""
        return ckpt.checkpoint(epoch, itime, self.params, self.eng.table, self.m, self.v, self.t, self.lr,
                               self.betas, self.eps, self.wd, loss)

    def load_checkpoint(self, state: Dict) -> None:
        """Resume from a reference-format checkpoint dict (checkpoints.py:35-51,
        update_model=True): weights, Adam moments, step count and hyper-parameters;
        the bf16 filter packs are rebuilt."""
        ckpt.load_model_state_dict(self.params, self.eng.table, state["model_state_dict"], strict=False)
        self.t, hp = ckpt.load_adam_state_dict(self.eng.table, state["optimizer_state_dict"], self.m, self.v)
        self.lr, self.betas, self.eps, self.wd = hp["lr"], tuple(hp["betas"]), hp["eps"], hp["weight_decay"]
        if self.info.enabled:
            for t in (self.params, self.m, self.v):
                torch.distributed.broadcast(t, 0)
        for e in self.engines:
            e.pack(self.params)
