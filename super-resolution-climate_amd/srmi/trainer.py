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
from typing import Dict, Optional

import torch

from .dist import DistInfo, GradReducer, allreduce_sum_
from .engine import Engine, NetSpec, adam_step, downsample, upsample


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
    def __init__(self, spec: NetSpec, batch: int, lr_hw=(48, 48), lr: float = 1e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, interp_loss: bool = True,
                 info: Optional[DistInfo] = None, device: Optional[torch.device] = None, seed: int = 0,
                 params: Optional[torch.Tensor] = None):
        self.info = info or DistInfo()
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.spec = spec
        self.batch = batch
        self.eng = Engine(spec, batch, lr_hw, train=True, device=self.device)
        n = self.eng.n_params
        self.params = torch.empty(n, dtype=torch.float32, device=self.device)
        if params is not None:
            self.params.copy_(params)
        else:
            default_init_(self.params, self.eng.table, seed)
        if self.info.enabled:  # identical replicas (rank 0's weights)
            torch.distributed.broadcast(self.params, 0)
        self.grads = torch.zeros(n, dtype=torch.float32, device=self.device)
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
        self.reducer = GradReducer(self.eng.table, spec.arch, spec.nlayers, self.info, self.device)
        self.eng.pack(self.params)

    def step(self, hr: torch.Tensor) -> Dict[str, torch.Tensor]:
        """hr: this rank's HR tiles [b, C, H, W] fp32 on the device (already normalised)."""
        b = hr.shape[0]
        s = self.spec.scale
        lr_in = self.lrbuf[:b]
        sr = self.sr[:b]
        downsample(hr, s, out=lr_in)
        self.eng.forward(self.params, lr_in, out=sr)
        count = float(hr.numel()) * self.info.world
        self.eng.rmse_partial(sr, hr, self.loss4, count)
        allreduce_sum_(self.loss4[0:1], self.info)
        Engine.rmse_finalize(self.loss4)
        if self.interp_loss:
            up = upsample(lr_in, s, out=self.up[:b])
            self.eng.rmse_partial(hr, up, self.iloss4, count)
            allreduce_sum_(self.iloss4[0:1], self.info)
            Engine.rmse_finalize(self.iloss4)
        ev = self.reducer.events if self.info.enabled and self.reducer.cuda else None
        self.eng.backward(self.params, lr_in, self.grads, sr=sr, hr=hr, loss4=self.loss4, events=ev)
        self.reducer.reduce(self.grads)
        self.t += 1
        adam_step(self.params, self.grads, self.m, self.v, self.t, self.lr, self.betas, self.eps, self.wd)
        self.eng.pack(self.params)
        return {"loss": self.loss4[3:4], "interp_loss": self.iloss4[3:4]}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Reference-format model state_dict (CPU copies)."""
        out = {}
        host = self.params.detach().cpu()
        for name, off, n, shape in self.eng.table:
            out[name] = host[off:off + n].view(shape).clone()
        return out
