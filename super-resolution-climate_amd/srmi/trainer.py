"""Fused training step on the native engine.

Restates one iteration of ModelTrainer.train (sres/controller/dual_trainer.py:310-323)
with apply_network (:557-571) for the RCAN/EDSR plugins:

    HR tile batch -> bicubic 1/s (array.py:72-76) -> network -> loss
    [-> interp-baseline loss metric, dual_trainer.py:315-318]
    -> backward -> Adam (lr = task.lr, weight_decay = task.weight_decay or 0)

The loss is model.loss_fn (single_product_loss, dual_trainer.py:205-212): 'l2' =
RMSE (l2loss, stats.py:5-8), 'charbonnier' = mean(sqrt(d^2 + 1e-6)) (:196-198);
anything else raises, as the reference does.

Everything runs asynchronously on one HIP stream: the per-step losses stay on
the device (no .item() sync) until the caller asks for them.
With a DistInfo of world > 1 the batch is this rank's shard and the loss /
gradients are all-reduced as described in srmi/dist.py.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch

from . import checkpoint as ckpt
from ._lib import SRMI_LOSS_MEAN, SRMI_LOSS_RMSE, TILE_LOSS_SUB, call, ptr
from .config import check_fused_task, data_downsample_factor, interp_mode
from .dist import DistInfo, GradReducer, allreduce_sum_
from .engine import Engine, NetSpec, adam_step, axpy, downsample, engine_stream, interp_size, upsample

LOSS_KINDS = {"l2": SRMI_LOSS_RMSE, "charbonnier": SRMI_LOSS_MEAN}
CHARBONNIER_EPS = 1e-6  # ModelTrainer.eps, sres/controller/dual_trainer.py:122


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
                 params: Optional[torch.Tensor] = None, micro: Optional[int] = None, loss_fn: str = "l2",
                 cu_budget: Optional[int] = None, task=None, dp_reducer_stream: bool = False):
        """task: the task config section (default: the active srmi ConfigContext's,
        if any).  apply_network's target selection is followed: when
        task.target_variables names fewer channels than the input, the loss target is
        those HR channels (index_select in the input's order, dual_trainer.py:564-568)
        and the model has that many output channels.  task.data_downsample = ds > 1
        downsamples every HR batch by ds first, as apply_network does (:561-563):
        step() then takes tiles T with floor(T / ds) = lr_hw * scale.
        dp_reducer_stream (data parallel, A/B): the gradient all-reduce on a reducer
        stream of its own that waits for each residual group's event of the whole
        enqueued backward, instead of (the default) enqueuing the backward stage by stage
        with each bucket's all-reduce behind its stage on an engine stream.
        task.downsample_mode / upsample_mode select the resampling of the model input
        and of the interp baseline ('cubic' -> bicubic, 'linear' -> bilinear,
        array.py:37-41; others raise)."""
        if loss_fn not in LOSS_KINDS:  # single_product_loss, dual_trainer.py:210-211
            raise ValueError(f"Unknown single-product loss function {loss_fn}")
        if task is None:
            from . import config as _config
            task = _config._CURRENT.get("task") if _config._CURRENT is not None else None
        tindx = check_fused_task(task, spec.nchannels_in, spec.nchannels_out)
        self.ds = data_downsample_factor(task)
        self.dmode, self.umode = interp_mode(task, True), interp_mode(task, False)
        if tindx is not None and interp_loss and spec.nchannels_out != 1:
            # loss(btarget, upsample(binput)) (:315-317) needs equal or broadcastable channels
            raise ValueError(f"interp loss of a {spec.nchannels_out}-channel target against the "
                             f"{spec.nchannels_in}-channel interpolated input does not broadcast (as in the reference)")
        self.loss_fn = loss_fn
        self.loss_kind = LOSS_KINDS[loss_fn]
        self.info = info or DistInfo()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.tindx = None if tindx is None else torch.tensor(tindx, dtype=torch.long, device=self.device)
        self.spec = spec
        self.batch = batch
        if micro is None:
            micro = 2 if (batch % 2 == 0 and batch >= 16) else 1
        if batch % micro:
            raise ValueError(f"batch {batch} not divisible into {micro} micro-batches")
        self.micro = micro
        self.mb = batch // micro
        # CUs each engine's launches are sized for (0 = the whole chip)
        budget = (256 // micro if micro > 1 else 0) if cu_budget is None else int(cu_budget)
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
        self.up = (torch.empty((batch, C, h * s, w * s), dtype=torch.float32, device=self.device)
                   if interp_loss else None)
        # Charbonnier: the elementwise loss gradient is the backward's upstream gradient
        self.dy = torch.empty_like(self.sr) if self.loss_kind == SRMI_LOSS_MEAN else None
        # the selected target channels (index_select) and, for the interp metric, that
        # target broadcast over the input's channels (1-channel target, :316-317)
        self.tgt = torch.empty_like(self.sr) if self.tindx is not None else None
        self.tgt_b = (torch.empty((batch, C, h * s, w * s), dtype=torch.float32, device=self.device)
                      if self.tindx is not None and interp_loss else None)
        # apply_network's data_downsample: the HR batch downsampled by ds first
        self.hrds = (torch.empty((batch, C, h * s, w * s), dtype=torch.float32, device=self.device)
                     if self.ds > 1 else None)
        self.loss4 = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.iloss4 = torch.zeros(4, dtype=torch.float32, device=self.device)
        # the loss sums as per-tile parts (srmi_tile_loss_parts) of the GLOBAL batch, in
        # global tile order: [loss parts | interp parts] of the step's gb tiles.  The
        # step's loss -- and the gradient scale 1/(count L) -- then depends neither on the
        # micro-batch split nor, data parallel, on how the batch is sharded over ranks:
        # every rank writes its tiles' parts into a zeroed array, one SUM all-reduce
        # (x + 0 is exact) hands every rank all of them, and every rank sums them in the
        # order one process would.
        self.gcap = batch * self.info.world
        self.gparts = torch.zeros(2 * self.gcap * TILE_LOSS_SUB, dtype=torch.float32, device=self.device)
        self.streams = [None] + [engine_stream(self.device) for _ in range(micro - 1)]
        self.dp_staged = not dp_reducer_stream
        self.reducer = GradReducer(self.eng.table, spec.arch, spec.nlayers, self.info, self.device,
                                   stream=self.info.enabled and not self.dp_staged)
        # group events of engines 1.. (engine 0 records into reducer.events)
        self.xevents = [self.reducer.new_events() for _ in range(micro - 1)]
        # staged DP backward: the stages, the buckets final after each, and per engine
        # (but the last, which reduces) an event per stage
        self.nstages = self.eng.stage_count if self.info.enabled and self.dp_staged else 0
        self.stage_buckets = self.reducer.stage_buckets(self.nstages) if self.nstages else []
        self.stage_ev = ([[torch.cuda.Event() for _ in range(self.nstages)] for _ in range(micro - 1)]
                         if self.nstages and self.device.type == "cuda" else [])
        for e in self.engines:
            e.pack(self.params)

    def _ctx(self, k):
        st = self.streams[k]
        return torch.cuda.stream(st) if st is not None else _Null()

    def _loss_parts(self, pred, target, parts, t0):
        """This micro-batch's tiles' loss parts (rows t0.. of the batch-wide parts array)."""
        nt = pred.shape[0]
        te = pred[0].numel()
        call("srmi_tile_loss_parts", ptr(pred), ptr(target), nt, te, self.loss_kind, CHARBONNIER_EPS,
             ptr(parts[t0 * TILE_LOSS_SUB:]), torch.cuda.current_stream(self.device).cuda_stream)

    def _reduce_losses(self, gb, count, icount):
        """loss4 / iloss4 of the whole (global) batch from its gb tiles' parts in tile
        order, finalised (data parallel: after the all-reduce of the parts)."""
        st = torch.cuda.current_stream(self.device).cuda_stream
        n = gb * TILE_LOSS_SUB
        if self.info.enabled:
            allreduce_sum_(self.gparts[:2 * n if self.interp_loss else n], self.info)
        call("srmi_loss_from_parts", ptr(self.gparts), gb, float(count), self.loss_kind, ptr(self.loss4), st)
        if self.interp_loss:
            call("srmi_loss_from_parts", ptr(self.gparts[n:]), gb, float(icount), self.loss_kind, ptr(self.iloss4),
                 st)

    def _shard(self, b: int, shard: Optional[Tuple[int, int]]) -> Tuple[int, int]:
        """(t0, gb): this call's tiles are tiles t0 .. t0 + b - 1 of a gb-tile global
        batch.  Default: the whole batch (one process) or, data parallel, equal shards
        in rank order."""
        if shard is None:
            return (self.info.rank * b, self.info.world * b) if self.info.enabled else (0, b)
        t0, gb = int(shard[0]), int(shard[1])
        if not self.info.enabled and (t0, gb) != (0, b):
            raise ValueError(f"shard {shard} of a {b}-tile batch without data parallelism")
        if t0 < 0 or t0 + b > gb or gb < 1 or gb > self.gcap:
            raise ValueError(f"shard {shard} of {b} tiles outside a global batch of 1..{self.gcap} tiles")
        return t0, gb

    def step(self, hr: torch.Tensor, shard: Optional[Tuple[int, int]] = None) -> Dict[str, torch.Tensor]:
        """hr: this rank's HR tiles [b, C, H, W] fp32 on the device (already normalised),
        b <= the trainer's batch (a short last batch of a time slice, as the
        reference's TileBatchIterator yields, sres/data/tiles.py:55-72).

        Data parallel, shard = (t0, gb): hr holds tiles t0 .. t0 + b - 1 of the step's
        gb-tile global batch (srmi.dist.shard_range; a rank of a short last batch may
        hold none, b = 0, and still takes part in every collective and the Adam step);
        the default is equal shards in rank order."""
        b = hr.shape[0]
        if b < (0 if self.info.enabled else 1) or b > self.batch:
            raise ValueError(f"batch {b} outside {0 if self.info.enabled else 1}..{self.batch}")
        t0, gb = self._shard(b, shard)
        s = self.spec.scale
        if self.ds > 1 and b:  # apply_network: downsample(input, scale_factor=ds) first (:561-563)
            got = tuple(interp_size(n, 1.0 / self.ds) for n in hr.shape[2:])
            if got != tuple(self.hrds.shape[2:]):
                raise ValueError(f"data_downsample={self.ds}: HR tiles {tuple(hr.shape[2:])} give {got}, "
                                 f"expected {tuple(self.hrds.shape[2:])}")
            hr = downsample(hr, self.ds, out=self.hrds[:b], mode=self.dmode)
        mb = (b + self.micro - 1) // self.micro
        sls = [slice(min(b, k * mb), min(b, (k + 1) * mb)) for k in range(self.micro)]
        main = torch.cuda.current_stream(self.device)
        if self.tindx is not None and b:  # apply_network's index_select of the target channels
            tgt = torch.index_select(hr, 1, self.tindx, out=self.tgt[:b])
            if self.tgt_b is not None:
                self.tgt_b[:b].copy_(tgt.expand(-1, hr.shape[1], -1, -1))
        else:
            tgt = hr
        # element counts of the global batch: target tiles (Co x HR) and interp tiles (C x HR)
        count = float(gb) * self.sr[0].numel()
        icount = float(gb) * self.lrbuf[0].numel() * s * s
        n = gb * TILE_LOSS_SUB
        lparts, iparts = self.gparts[:n], self.gparts[n:2 * n]
        if self.info.enabled:  # the other ranks' tiles' parts stay 0 here
            self.gparts[:2 * n].zero_()
        for st in self.streams[1:]:
            st.wait_stream(main)
        # forward + loss partials per micro-batch (an empty micro-batch adds nothing)
        for k, eng in enumerate(self.engines):
            sl = sls[k]
            if sl.stop == sl.start:
                continue
            with self._ctx(k):
                downsample(hr[sl], s, out=self.lrbuf[sl], mode=self.dmode)
                eng.forward(self.params, self.lrbuf[sl], out=self.sr[sl])
                if self.dy is not None:  # Charbonnier: the elementwise upstream gradient only
                    eng.charbonnier_partial(self.sr[sl], tgt[sl], None, count, CHARBONNIER_EPS, dy=self.dy[sl])
                self._loss_parts(self.sr[sl], tgt[sl], lparts, t0 + sl.start)
                if self.interp_loss:  # self.loss(btarget, binterp), dual_trainer.py:316-317
                    up = upsample(self.lrbuf[sl], s, out=self.up[sl], mode=self.umode)
                    itgt = hr[sl] if self.tgt_b is None else self.tgt_b[sl]
                    self._loss_parts(itgt, up, iparts, t0 + sl.start)
        for st in self.streams[1:]:
            main.wait_stream(st)
        self._reduce_losses(gb, count, icount)
        for st in self.streams[1:]:
            st.wait_stream(main)
        # backward per micro-batch with the global loss scale.  Data parallel: the
        # engines' gradients are added and all-reduced bucket by bucket as soon as every
        # engine is past the bucket, overlapped with the rest of backward
        # (_backward_dp_staged, or the reducer stream waiting on the engines' residual-group events).
        dp = self.info.enabled and self.reducer.cuda
        if dp and self.dp_staged:
            self._backward_dp_staged(sls, tgt)
            return self._finish_step(main)
        evs = [self.reducer.events] + self.xevents if dp else [None] * self.micro
        for k, eng in enumerate(self.engines):
            sl = sls[k]
            with self._ctx(k):
                if sl.stop == sl.start:  # no tiles: zero gradient (and its group events)
                    self.mgrads[k].zero_()
                    if evs[k] is not None:
                        for ev in evs[k]:
                            ev.record()
                    continue
                if self.dy is not None:
                    eng.backward(self.params, self.lrbuf[sl], self.mgrads[k], dy=self.dy[sl], events=evs[k])
                else:
                    eng.backward(self.params, self.lrbuf[sl], self.mgrads[k], sr=self.sr[sl], hr=tgt[sl],
                                 loss4=self.loss4, events=evs[k])
        for st in self.streams[1:]:
            main.wait_stream(st)
        if dp:
            self.reducer.reduce(self.grads, events_recorded=True, extra=self.mgrads[1:], extra_events=self.xevents)
        else:
            for g in self.mgrads[1:]:
                axpy(self.grads, g, 1.0)  # exact gradient of the whole batch
        return self._finish_step(main)

    def _backward_dp_staged(self, sls, tgt):
        """Data-parallel backward without a reducer stream: with two micro-batch engines
        a rank runs 3 streams (the engines' and RCCL's) instead of 4.  The engines'
        backward is enqueued stage by stage (srmi_backward_stages: tail / upsamplers,
        each residual group, head); behind the stage that finalises a bucket, the LAST
        engine's stream waits for the other engines' events of that stage, adds their
        gradients into engine 0's (the exact whole-batch gradient) and launches the
        bucket's asynchronous all-reduce.  RCCL's stream waits for that point; no engine
        stream waits for RCCL until Adam."""
        red_k = self.micro - 1
        works = []
        for s in range(self.nstages):
            for k, eng in enumerate(self.engines):
                sl = sls[k]
                with self._ctx(k):
                    if sl.stop == sl.start:  # no tiles: a zero gradient
                        if s == 0:
                            self.mgrads[k].zero_()
                    elif self.dy is not None:
                        eng.backward(self.params, self.lrbuf[sl], self.mgrads[k], dy=self.dy[sl], stages=(s, s))
                    else:
                        eng.backward(self.params, self.lrbuf[sl], self.mgrads[k], sr=self.sr[sl], hr=tgt[sl],
                                     loss4=self.loss4, stages=(s, s))
                    if k != red_k:
                        self.stage_ev[k][s].record()
            if self.stage_buckets[s]:
                with self._ctx(red_k):
                    cur = torch.cuda.current_stream(self.device)
                    for k in range(self.micro):
                        if k != red_k:
                            cur.wait_event(self.stage_ev[k][s])
                    self.reducer.reduce_stage(self.stage_buckets[s], self.grads, self.mgrads[1:], works)
        for w in works:
            w.wait()  # the current (main) stream waits for the all-reduces

    def _finish_step(self, main):
        for st in self.streams[1:]:
            main.wait_stream(st)
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
        the bf16 filter packs are rebuilt.  The model dict is loaded with FModule's
        strict semantics (common.py:50-71: unexpected or missing keys raise, only a
        re-shaped 'tail' is skipped).  Both dicts are validated into host buffers
        before anything on the device changes, so a failed load leaves the trainer
        as it was."""
        host_p = ckpt.load_model_state_dict(self.params, self.eng.table, state["model_state_dict"], strict=True,
                                            apply=False)
        t, hp, mh, vh = ckpt.load_adam_state_dict(self.eng.table, state["optimizer_state_dict"], self.m, self.v,
                                                  apply=False)
        self.params.copy_(host_p)
        self.m.copy_(mh)
        self.v.copy_(vh)
        self.t = t
        self.lr, self.betas, self.eps, self.wd = hp["lr"], tuple(hp["betas"]), hp["eps"], hp["weight_decay"]
        if self.info.enabled:
            for x in (self.params, self.m, self.v):
                torch.distributed.broadcast(x, 0)
        for e in self.engines:
            e.pack(self.params)
