"""The residual-stream pair codec (csrc/common.hpp pair_encode4 / pair_decode4) as the
tests' emulation restates it (tests/gpu_oracle.py pair16): its precision contract,
checked on the CPU over random and edge-case fp32 values."""
import torch

from gpu_oracle import pair16


def _bits(x):
    return x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF


def test_pair_keeps_16_significant_bits_and_hi_is_the_rounded_value():
    g = torch.Generator().manual_seed(5)
    x = torch.cat([torch.randn(200000, generator=g) * 10.0 ** torch.randint(-6, 6, (200000,), generator=g),
                   torch.tensor([1.0, -1.0, 2.0, 0.5, 1.9999999, -1.9999999, 3.0e-30, -7.5e20])])
    y = pair16(x)
    rel = ((y.double() - x.double()).abs() / x.double().abs()).max()
    assert float(rel) <= 2.0 ** -16
    # decode = A - (A & 0xFF) + 128 in fp32 steps, across binade boundaries too
    a, b = _bits(x), _bits(y)
    assert bool(((b - a).abs() <= 128).all())
    # round-to-nearest-even of the decoded value is the stored hi (rounded half away
    # from zero): the next conv's bf16 operand is exactly the pair's hi
    hi = ((a + 0x8000) >> 16) & 0xFFFF
    assert bool(((_bits(y.to(torch.bfloat16).float()) >> 16) == hi).all())
    # and hi differs from torch's bf16 rounding of h only at exact ties
    tie = (a & 0xFFFF) == 0x8000
    rne = _bits(x.to(torch.bfloat16).float()) >> 16
    assert bool(((rne == hi) | tie).all())
