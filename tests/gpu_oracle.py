"""GPU-resident checker for the full-size parity tests (test infrastructure only).

The full-size headline configurations (C2: rcan-10-20-64, B=64; C5: 441 tiles of
a 4096^2 region) are too large for the CPU oracle to finish in seconds, so the
tests run the same oracle module (oracle/rcan_oracle.py, PyTorch) on the GPU in
fp32 as the checker, with MIOpen disabled (no kernel JIT on a fresh box: convs
run as unfold + rocBLAS GEMM) and no reduced-precision math.

`bf16_operand_emulation` turns an oracle model into the reference arithmetic
with bf16-rounded conv OPERANDS (the engine's precision model, SURVEY.md §8(c):
bf16 operands, fp32 accumulation, fp32 residual stream): every 3x3 conv with 64
input channels computes y = conv(bf16(x), bf16(w)) + b, and its backward
dx = conv^T(bf16(dy), bf16(w)), dw = corr(bf16(x), bf16(dy)); everything else
stays fp32.  Its drift from the fp32 oracle is the reference's own bf16 drift,
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


class _EmulConv(nn.Module):
    def __init__(self, conv: nn.Conv2d):
        super().__init__()
        self.conv = conv

    def forward(self, x):
        c = self.conv
        return _Bf16OperandConv.apply(x, c.weight, c.bias, c.padding)


def bf16_operand_emulation(model: nn.Module) -> nn.Module:
    """In place: wrap every 3x3 conv with 64 input channels (not the C-channel head)."""
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, nn.Conv2d) and child.kernel_size == (3, 3) and child.in_channels == 64:
                setattr(mod, cname, _EmulConv(child))
    return model


def conv_params(model: nn.Module):
    """named parameters of a (possibly emulation-wrapped) model under the reference keys."""
    return {n.replace(".conv.", "."): p for n, p in model.named_parameters()}
