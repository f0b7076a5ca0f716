"""GPU-resident checker for the full-size parity tests (test infrastructure only).

The full-size headline configurations (C2: rcan-10-20-64, B=64; C5: 441 tiles of
a 4096^2 region) are too large for the CPU oracle to finish in seconds, so the
tests run the same oracle module (oracle/rcan_oracle.py, PyTorch) on the GPU in
fp32 as the checker, with MIOpen disabled (no kernel JIT on a fresh box: convs
run as unfold + rocBLAS GEMM) and no reduced-precision math.

`bf16_operand_emulation` turns an oracle model into the engine's precision model
(what the bf16 engine actually computes):
* every 3x3 conv with 64 input channels computes y = conv(bf16(x), bf16(w)) + b,
  its backward dx = conv^T(bf16(dy), bf16(w)), dw = corr(bf16(x), bf16(dy)) (the
  engine's MFMA operands and its bf16 activation / gradient maps t, u, hb, dz, du);
* in every RCAB the channel-attention product uses the stored bf16 u while the
  pooled mean is that of the fp32 conv output (training's conv2 derives it from the
  statistics of the bf16 t and conv2's bf16 filters, csrc/ca_scale.hpp -- the same
  quantity up to fp32 summation order): out = bf16(u) * s(mean(u));
* the residual stream INSIDE a residual group is the pair hi + lo (bf16 hi plus an
  8-bit remainder, common.hpp pair codec): 16 significant bits, rounded after every
  CA add (h = pair16(h + out)); the group input, the
  group-tail / body-tail outputs stay fp32;
* the gradient stream INSIDE a residual group -- the gradient w.r.t. every RCAB's
  output -- is bf16 (the group-tail dgrad and every RCAB's conv1 dgrad store it rounded,
  EPI_DG_ACC_CA16, and the CA backward reads it): rounded where it arrives at an RCAB
  output (after autograd has summed the identity and conv paths); the gradient of the
  group input and every other gradient stay fp32.
Rounding is straight-through in backward, as in the engine (the stored values are
what backward reads; the gradient of an add is the identity).  The model's drift
from the fp32 oracle is the reference's own drift under the engine's arithmetic,
from which the tests derive their gradient bounds.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn
import torch.nn.functional as F


@contextlib.contextmanager
def exact_fp32():
    """fp32 torch math with MIOpen off (no JIT) and no TF32-style shortcuts."""
    saved = (torch.backends.cudnn.enabled, torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32)
    torch.backends.cudnn.enabled = False
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    try:
        yield
    finally:
        torch.backends.cudnn.enabled, torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = saved


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype)


class _Bf16OperandConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad):
        xb, wb = _bf(x), _bf(w)
        ctx.save_for_backward(xb, wb)
        ctx.pad = pad
        return F.conv2d(xb, wb, b, padding=pad)

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        dyb = _bf(dy)
        dx = torch.nn.grad.conv2d_input(xb.shape, wb, dyb, padding=ctx.pad)
        dw = torch.nn.grad.conv2d_weight(xb, wb.shape, dyb, padding=ctx.pad)
        return dx, dw, dy.sum(dim=(0, 2, 3)), None


class _StraightBf16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _bf(x)

    @staticmethod
    def backward(ctx, g):
        return g


def pair16(h: torch.Tensor) -> torch.Tensor:
    """The pair codec (csrc/common.hpp pair_encode4 / pair_decode4) on fp32 bit
    patterns A: hi = (A + 0x8000) >> 16, lo = byte 1 of A, value bits
    ((hi << 16) | 0x80) + (sext8(lo) << 8) = A - (A & 0xFF) + 128: h to within 128 fp32
    steps of its binade, and bf16(value) == hi (round to nearest even never ties)."""
    hf = h.float()
    a = hf.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    hi = ((a + 0x8000) >> 16) & 0xFFFF
    q = (a >> 8) & 0xFF
    q = torch.where(q >= 128, q - 256, q)
    bits = (((hi << 16) | 0x80) + (q << 8)) & 0xFFFFFFFF
    bits = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
    return bits.view(torch.float32).to(h.dtype)


class _GradBf16(torch.autograd.Function):
    """Identity forward; backward rounds the (summed) incoming gradient to bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _bf(g)


class _StraightPair16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return pair16(x)

    @staticmethod
    def backward(ctx, g):
        return g


def _emul_rcab_forward(self, x):
    """RCAB (sres/model/rcan/network.py:54-64) as the bf16 engine computes it."""
    b = self.body
    u = b[2](b[1](b[0](x)))
    s = b[3].conv_du(u.mean(dim=(2, 3), keepdim=True))
    return _GradBf16.apply(_StraightPair16.apply(_StraightBf16.apply(u) * s + x))


class _EmulConv(nn.Module):
    def __init__(self, conv: nn.Conv2d):
        super().__init__()
        self.conv = conv

    def forward(self, x):
        c = self.conv
        return _Bf16OperandConv.apply(x, c.weight, c.bias, c.padding)


def bf16_operand_emulation(model: nn.Module, pair_stream: bool = True) -> nn.Module:
    """In place: wrap every 3x3 conv with 64 input channels (not the C-channel head)
    and, with pair_stream, give every RCAB the engine's CA product and in-group pair
    residual stream (module docstring)."""
    import types
    from oracle.rcan_oracle import _RCAB
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, nn.Conv2d) and child.kernel_size == (3, 3) and child.in_channels == 64:
                setattr(mod, cname, _EmulConv(child))
    if pair_stream:
        for mod in model.modules():
            if isinstance(mod, _RCAB):
                mod.forward = types.MethodType(_emul_rcab_forward, mod)
    return model


def conv_params(model: nn.Module):
    """named parameters of a (possibly emulation-wrapped) model under the reference keys."""
    return {n.replace(".conv.", "."): p for n, p in model.named_parameters()}
