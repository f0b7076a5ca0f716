"""Training-batch preparation on the device.

The reference prepares every training batch on the host in xarray:

* ``norm`` with ``task.norm == 'lnorm'`` (sres/base/source/swot/raw.py:169-181):
  per tile and channel ``(x - mean) / std`` over (y, x), ddof 0, the statistics
  kept as ``attrs['mean'] / attrs['std']`` of shape [B, C, 1, 1];
* ``xyflip`` (sres/base/source/batch.py:37-49, called by ``load_batch`` :301):
  when ``task.xyflip`` is set, one ``random.randint(0, 7)`` per batch picks a
  dihedral variant (bit 0 flips x, bit 1 flips y, bit 2 swaps the axes),
  recorded as ``attrs['xyflip']``;
* ``apply_network`` then feeds ``downsample(target)`` (dual_trainer.py:557-571,
  array.py:72-76) to the model.

``prep_batch`` does the three in one HIP kernel (``srmi_batch_prep``, tiles.hip):
one HBM read of the raw tiles, one write of the HR target and of the LR input.
The flip index is drawn on the host exactly as the reference draws it.
"""
from __future__ import annotations

import random
from typing import Dict, Optional

import torch

from ._lib import call, ptr, stream_handle


def xyflip_index(enabled: bool, rng: Optional[random.Random] = None) -> int:
    """The reference's draw (batch.py:38-40): ``random.randint(0, 7)`` if
    ``task.xyflip`` else 0 (module-level ``random``, unseeded, unless ``rng``)."""
    if not enabled:
        return 0
    return (rng or random).randint(0, 7)


def prep_batch(raw: torch.Tensor, flip_index: int = 0, scale: int = 4, with_lr: bool = True,
               hr: Optional[torch.Tensor] = None, lr: Optional[torch.Tensor] = None,
               stream=None) -> Dict[str, torch.Tensor]:
    """raw [B, C, T, T] fp32 device tiles -> {'hr': xyflip(lnorm(raw)), 'lr':
    downsample(hr, scale), 'mean': [B, C, 1, 1], 'std': [B, C, 1, 1],
    'xyflip': flip_index}.  Raises SrmiError on bad shapes (T odd, T % scale,
    flip_index outside 0..7)."""
    if raw.dtype != torch.float32 or raw.dim() != 4 or not raw.is_contiguous():
        raise ValueError("prep_batch: raw must be a contiguous fp32 [B, C, T, T] tensor")
    B, C, T, T2 = raw.shape
    if T != T2:
        raise ValueError("prep_batch: tiles must be square (xyflip swaps the axes)")
    if hr is None:
        hr = torch.empty_like(raw)
    if with_lr and lr is None:
        lr = torch.empty(B, C, T // scale, T // scale, device=raw.device, dtype=torch.float32)
    mean = torch.empty(B, C, 1, 1, device=raw.device, dtype=torch.float32)
    std = torch.empty_like(mean)
    call("srmi_batch_prep", ptr(raw), B, C, T, int(flip_index), int(scale), ptr(hr),
         ptr(lr) if with_lr else None, ptr(mean), ptr(std), stream_handle(stream))
    out = {"hr": hr, "mean": mean, "std": std, "xyflip": int(flip_index)}
    if with_lr:
        out["lr"] = lr
    return out
