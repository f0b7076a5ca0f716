"""Python handle on the native srmi engine (libsrmi.so).

One Engine = one network plan (RCAN or EDSR hyper-parameters), one tile
geometry, a batch capacity and a device workspace owned by PyTorch's caching
allocator.  Parameters live in ONE flat fp32 buffer in the reference's
state_dict order, gradients in another, Adam moments in two more: the whole
optimizer step is a single fused kernel and the gradient all-reduce works on
contiguous buckets.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import ModelConfig, ParamInfo, call, ptr, stream_handle

ARCHS = {"rcan": _lib.SRMI_ARCH_RCAN, "edsr": _lib.SRMI_ARCH_EDSR}
DTYPES = {"bf16": _lib.SRMI_DTYPE_BF16, "fp32": _lib.SRMI_DTYPE_F32}


@dataclass
class NetSpec:
    """Hyper-parameters of the plugin (config/model/*.yaml keys)."""
    arch: str = "rcan"
    nchannels_in: int = 1
    nchannels_out: int = 1
    nfeatures: int = 64
    nlayers: int = 10
    nblocks: int = 20
    cbottleneck: int = 2
    scale: int = 4
    res_scale: float = 1.0
    dtype: str = "bf16"   # engine operand type: "bf16" (bf16 MFMA operands) or "fp32" (exact fp32)
    flags: int = 0        # srmi_model_config.flags (SRMI_FLAG_CA_PASS, SRMI_FLAG_DU_PASS, SRMI_FLAG_NO_RCAB_INFER: A/B and tests)

    @staticmethod
    def from_parms(arch: str, parms: Dict, dtype: str = "bf16") -> "NetSpec":
        if parms.get("kernel_size", 3) != 3:
            raise _lib.SrmiError("srmi supports kernel_size 3 only")
        # RCAN ignores batch_norm: its RCABs are built with bn=False (sres/model/rcan/
        # network.py:70); EDSR's ResBlocks take it (edsr/network.py:15), unsupported here
        if parms.get("batch_norm", False) and arch != "rcan":
            raise _lib.SrmiError("srmi's EDSR supports batch_norm: False only (the reference configs)")
        if not parms.get("bias", True):
            raise _lib.SrmiError("srmi supports bias: True only (the reference configs)")
        return NetSpec(arch=arch, nchannels_in=int(parms["nchannels_in"]), nchannels_out=int(parms["nchannels_out"]),
                       nfeatures=int(parms["nfeatures"]), nlayers=int(parms["nlayers"]),
                       nblocks=int(parms.get("nblocks", 0) or 0), cbottleneck=int(parms.get("cbottleneck", 2) or 2),
                       scale=int(parms["scale"]), res_scale=float(parms.get("res_scale", 1.0)), dtype=dtype)

    def cstruct(self, batch: int, lr_h: int, lr_w: int, cu_budget: int = 0) -> ModelConfig:
        if self.dtype not in DTYPES:
            raise _lib.SrmiError(f"unknown engine dtype {self.dtype!r} (bf16 | fp32)")
        return ModelConfig(ARCHS[self.arch], self.nchannels_in, self.nchannels_out, self.nfeatures, self.nlayers,
                           self.nblocks if self.arch == "rcan" else 0, self.cbottleneck if self.arch == "rcan" else 1,
                           self.scale, self.res_scale, batch, lr_h, lr_w, int(cu_budget), DTYPES[self.dtype],
                           int(self.flags))


def param_names(spec: NetSpec) -> List[str]:
    """state_dict keys of the reference model, in order."""
    names = ["head.0.weight", "head.0.bias"]
    if spec.arch == "rcan":
        for g in range(spec.nlayers):
            for b in range(spec.nblocks):
                pre = f"body.{g}.body.{b}.body"
                names += [f"{pre}.0.weight", f"{pre}.0.bias", f"{pre}.2.weight", f"{pre}.2.bias",
                          f"{pre}.3.conv_du.0.weight", f"{pre}.3.conv_du.0.bias",
                          f"{pre}.3.conv_du.2.weight", f"{pre}.3.conv_du.2.bias"]
            names += [f"body.{g}.body.{spec.nblocks}.weight", f"body.{g}.body.{spec.nblocks}.bias"]
    else:
        for i in range(spec.nlayers):
            names += [f"body.{i}.body.0.weight", f"body.{i}.body.0.bias", f"body.{i}.body.2.weight",
                      f"body.{i}.body.2.bias"]
    names += [f"body.{spec.nlayers}.weight", f"body.{spec.nlayers}.bias"]
    nups = int(round(math.log2(spec.scale)))
    for k in range(nups):
        names += [f"tail.0.{2 * k}.weight", f"tail.0.{2 * k}.bias"]
    names += ["tail.1.weight", "tail.1.bias"]
    return names


def param_table(spec: NetSpec) -> List[Tuple[str, int, int, Tuple[int, ...]]]:
    cfg = spec.cstruct(1, 48, 48)
    n = C.c_longlong()
    nt = C.c_int()
    call("srmi_param_count", C.byref(cfg), C.byref(n), C.byref(nt))
    arr = (ParamInfo * nt.value)()
    call("srmi_param_table", C.byref(cfg), arr, nt.value)
    names = param_names(spec)
    if len(names) != nt.value:
        raise _lib.SrmiError(f"param table mismatch {len(names)} != {nt.value}")
    return [(names[i], arr[i].offset, arr[i].numel, tuple(arr[i].shape[:arr[i].ndim])) for i in range(nt.value)]


class Engine:
    def __init__(self, spec: NetSpec, batch: int, lr_hw: Tuple[int, int], train: bool = True,
                 device: Optional[torch.device] = None, cu_budget: int = 0):
        self.spec = spec
        self.batch = int(batch)
        self.lr_h, self.lr_w = int(lr_hw[0]), int(lr_hw[1])
        self.train_mode = bool(train)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._cfg = spec.cstruct(self.batch, self.lr_h, self.lr_w, cu_budget)
        nbytes = C.c_size_t()
        call("srmi_workspace_size", C.byref(self._cfg), int(train), C.byref(nbytes))
        self.workspace = torch.empty(int(nbytes.value) + 256, dtype=torch.uint8, device=self.device)
        h = C.c_void_p()
        call("srmi_engine_create", C.byref(self._cfg), ptr(self.workspace), self.workspace.numel(), int(train),
             C.byref(h))
        self._h = h
        self.table = param_table(spec)
        self.n_params = sum(t[2] for t in self.table)
        self.hr_h, self.hr_w = self.lr_h * spec.scale, self.lr_w * spec.scale
        self.loss4 = torch.zeros(4, dtype=torch.float32, device=self.device)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                _lib.load().srmi_engine_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # ------------------------------------------------------------------ ops
    def pack(self, params: torch.Tensor, stream=None):
        call("srmi_pack_weights", self._h, ptr(params), stream_handle(stream))

    def forward(self, params: torch.Tensor, lr: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None):
        n = lr.shape[0]
        assert lr.is_contiguous() and lr.dtype == torch.float32 and lr.device == self.device
        assert tuple(lr.shape[1:]) == (self.spec.nchannels_in, self.lr_h, self.lr_w), lr.shape
        if n > self.batch:
            raise _lib.SrmiError(f"batch {n} exceeds engine capacity {self.batch}")
        if out is None:
            out = torch.empty((n, self.spec.nchannels_out, self.hr_h, self.hr_w), dtype=torch.float32,
                              device=self.device)
        call("srmi_forward", self._h, ptr(params), ptr(lr), ptr(out), n, stream_handle(stream))
        return out

    def rmse_partial(self, pred: torch.Tensor, target: torch.Tensor, loss4: torch.Tensor, count_global: float,
                     stream=None):
        call("srmi_rmse_partial", self._h, ptr(pred), ptr(target), pred.numel(), float(count_global), ptr(loss4),
             stream_handle(stream))

    def charbonnier_partial(self, pred: torch.Tensor, target: torch.Tensor, loss4: torch.Tensor,
                            count_global: float, eps: float = 1e-6, dy: Optional[torch.Tensor] = None, stream=None):
        """ModelTrainer.charbonnier (dual_trainer.py:196-198) partial sums (+ dL/dpred into dy)."""
        call("srmi_charbonnier_partial", self._h, ptr(pred), ptr(target), pred.numel(), float(count_global),
             float(eps), ptr(loss4), ptr(dy), stream_handle(stream))

    @staticmethod
    def rmse_finalize(loss4: torch.Tensor, stream=None):
        call("srmi_rmse_finalize", ptr(loss4), stream_handle(stream))

    @staticmethod
    def loss_finalize(loss4: torch.Tensor, kind: int, stream=None):
        call("srmi_loss_finalize", ptr(loss4), int(kind), stream_handle(stream))

    @staticmethod
    def loss_combine(loss4: torch.Tensor, parts: torch.Tensor, kind: int = -1, stream=None):
        """loss4 <- sum of the micro-batch records parts[k][4] (finalised as `kind` if >= 0)."""
        assert parts.is_contiguous() and parts.shape[-1] == 4
        call("srmi_loss_combine", ptr(loss4), ptr(parts), parts.numel() // 4, int(kind), stream_handle(stream))

    @property
    def stage_count(self) -> int:
        """Stages of srmi_backward_stages: 0 = tail / upsamplers / body tail, 1..nlayers =
        residual groups nlayers-1..0, nlayers + 1 = head (RCAN); EDSR: 1."""
        return call("srmi_backward_stage_count", self._h)

    def backward(self, params: torch.Tensor, lr: torch.Tensor, grads: torch.Tensor, sr=None, hr=None, loss4=None,
                 dy=None, events: Optional[Sequence] = None, stream=None, stages: Optional[Tuple[int, int]] = None):
        """The whole backward of the last forward, or (stages = (first, last)) those
        stages of it -- each stage exactly once per backward, in order."""
        evp = None
        if events is not None:
            if any(e is not None and not e.cuda_event for e in events):
                raise RuntimeError("backward: group event not created yet (record it once before passing it)")
            evp = (C.c_void_p * len(events))(*[e.cuda_event if e is not None else None for e in events])
        if stages is not None:
            call("srmi_backward_stages", self._h, ptr(params), ptr(lr), ptr(sr), ptr(hr), ptr(loss4), ptr(dy),
                 ptr(grads), evp, int(stages[0]), int(stages[1]), stream_handle(stream))
            return
        call("srmi_backward", self._h, ptr(params), ptr(lr), ptr(sr), ptr(hr), ptr(loss4), ptr(dy), ptr(grads), evp,
             stream_handle(stream))


def engine_stream(device) -> "torch.cuda.Stream":
    """The stream of a second (third, ...) micro-batch engine: a HIGH-priority stream.

    HIP maps a process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues per
    priority, and two streams on one queue run one after the other.  Which normal-
    priority queue a new stream lands on depends on what the process used before: with
    an RCCL group up, the second engine's stream shared the default stream's queue and
    the one-rank DP step lost its two-engine overlap (44.1 vs 26.2 ms/step, every
    stream-creation offset; tools/dbg_dp.py, tools/dbg_queues.py).  High-priority
    streams come from a separate pool of queues that neither the default stream
    (engine 0) nor RCCL's streams use, so the engines never share a queue."""
    lo, hi = torch.cuda.Stream.priority_range()
    return torch.cuda.Stream(device=device, priority=hi)


# ----------------------------------------------------------------- free ops
INTERP_MODES = {"bilinear": _lib.SRMI_INTERP_BILINEAR, "bicubic": _lib.SRMI_INTERP_BICUBIC}


def interp_size(n: int, scale_factor: float) -> int:
    """F.interpolate's output size floor(n * scale_factor) (ATen compute_output_size)."""
    return int(math.floor(float(n) * float(scale_factor)))


def interpolate(x: torch.Tensor, scale_factor: float, mode: str = "bicubic", out: Optional[torch.Tensor] = None,
                stream=None) -> torch.Tensor:
    """torch.nn.functional.interpolate(x, scale_factor=scale_factor, mode=mode) with
    align_corners=False (mode 'bilinear' | 'bicubic'), NCHW fp32, any factor
    (srmi_interpolate)."""
    if mode not in INTERP_MODES:
        raise _lib.SrmiError(f"interpolation mode {mode!r}: bilinear | bicubic")
    N, Cc, H, W = x.shape
    Ho, Wo = interp_size(H, scale_factor), interp_size(W, scale_factor)
    if out is None:
        out = torch.empty((N, Cc, Ho, Wo), dtype=torch.float32, device=x.device)
    if tuple(out.shape) != (N, Cc, Ho, Wo):
        raise _lib.SrmiError(f"interpolate: out {tuple(out.shape)} != {(N, Cc, Ho, Wo)}")
    r = 1.0 / float(scale_factor)  # (float)(1 / scale_factor): ctypes rounds it to fp32 as ATen does
    call("srmi_interpolate", ptr(x), N, Cc, H, W, Ho, Wo, r, r, INTERP_MODES[mode], ptr(out), stream_handle(stream))
    return out


def downsample(hr: torch.Tensor, scale, out: Optional[torch.Tensor] = None, stream=None,
               mode: str = "bicubic") -> torch.Tensor:
    """downsample (sres/base/util/array.py:72-76): F.interpolate(scale_factor=1/scale,
    mode), NCHW fp32.  Bicubic at an even integer factor dividing the tile is the
    separable half-way [-3,19,19,-3]/32 kernel (srmi_downsample); every other factor
    or mode takes the general F.interpolate kernel (srmi_interpolate)."""
    N, Cc, H, W = hr.shape
    fs = float(scale)
    if mode == "bicubic" and fs.is_integer() and int(fs) % 2 == 0 and H % int(fs) == 0 and W % int(fs) == 0:
        scale = int(fs)
        if out is None:
            out = torch.empty((N, Cc, H // scale, W // scale), dtype=torch.float32, device=hr.device)
        call("srmi_downsample", ptr(hr), N, Cc, H, W, scale, ptr(out), stream_handle(stream))
        return out
    return interpolate(hr, 1.0 / fs, mode, out=out, stream=stream)


def upsample(lr: torch.Tensor, scale: int, out: Optional[torch.Tensor] = None, stream=None,
             mode: str = "bicubic") -> torch.Tensor:
    """upsample, the interp baseline (sres/base/util/array.py:84-87):
    F.interpolate(scale_factor=scale, mode), NCHW fp32."""
    N, Cc, h, w = lr.shape
    if mode != "bicubic":
        return interpolate(lr, float(scale), mode, out=out, stream=stream)
    if out is None:
        out = torch.empty((N, Cc, h * scale, w * scale), dtype=torch.float32, device=lr.device)
    call("srmi_upsample", ptr(lr), N, Cc, h, w, scale, ptr(out), stream_handle(stream))
    return out


def axpy(y: torch.Tensor, x: torch.Tensor, a: float = 1.0, stream=None):
    """y += a * x on flat fp32 device buffers (HIP kernel)."""
    assert y.numel() == x.numel() and y.dtype == x.dtype == torch.float32
    call("srmi_axpy", ptr(y), ptr(x), float(a), y.numel(), stream_handle(stream))
    return y


def adam_step(p, g, m, v, step: int, lr: float, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, stream=None):
    call("srmi_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), int(step), float(lr), float(betas[0]),
         float(betas[1]), float(eps), float(weight_decay), stream_handle(stream))
