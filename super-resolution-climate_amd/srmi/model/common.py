"""SRNet: the nn.Module behind the plugin boundary.

Drop-in for the reference's FModule-based networks (sres/model/common/common.py:30-71):
same constructor contract (``get_model(**config)`` with nchannels_in /
nchannels_out / device, hyper-parameters from cfg().model), same state_dict
keys and shapes, same tolerant load_state_dict, ``forward(x[B,Cin,h,w] fp32)
-> [B,Cout,s*h,s*w] fp32`` differentiable w.r.t. ``parameters()``.

Internally every parameter is a view into ONE flat fp32 buffer, forward and
backward are single calls into the native engine (hand-written HIP kernels on
gfx950) through a torch.autograd.Function.  There is no PyTorch/CPU fallback:
on a machine without the HIP library or a GPU, forward raises.
"""
from __future__ import annotations

from typing import Any, Dict, Mapping, Optional, Tuple

import torch
import torch.nn as nn

from .. import _lib
from ..config import init_parms
from ..engine import Engine, NetSpec, param_table


class _Node(nn.Module):
    pass


class _SRNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net: "SRNet", flat: torch.Tensor, *params):
        eng = net._engine_for(x, train=True)
        out = eng.forward(flat, x)
        net._fwd_token += 1
        ctx.net = net
        ctx.token = net._fwd_token
        ctx.eng = eng
        ctx.nparams = len(params)
        ctx.save_for_backward(x, flat, out)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, flat, out = ctx.saved_tensors
        net: SRNet = ctx.net
        if ctx.token != net._fwd_token:
            raise _lib.SrmiError("srmi: backward of a stale forward (the engine keeps one forward's activations; "
                                 "call backward before the next training-mode forward)")
        grads = torch.empty(net._n_params, dtype=torch.float32, device=flat.device)
        ctx.eng.backward(flat, x, grads, dy=gout.contiguous().float())
        views = [grads[o:o + n].view(s) for (_, o, n, s) in net._table]
        return (None, None, None, *views)


class SRNet(nn.Module):
    arch = "rcan"

    def __init__(self, **kwargs):
        super().__init__()
        custom = {k: v for k, v in kwargs.items()}
        parms = init_parms(self.arch, custom)
        self.parms = parms
        self.spec = NetSpec.from_parms(self.arch, parms, dtype=str(parms.get("dtype", "bf16")))
        self._table = None
        self._n_params = 0
        self._engines: Dict[Tuple[bool, int, int], Engine] = {}
        self._fwd_token = 0
        self._packed_version: Optional[Tuple[int, int]] = None
        self._build_params(torch.device("cpu"))

    # ------------------------------------------------------------ structure
    def _build_params(self, device):
        try:
            table = param_table(self.spec)
        except _lib.SrmiError:
            table = None
        if table is None:  # library absent: shapes from the Python mirror (construction still works)
            table = _python_table(self.spec)
        self._table = table
        self._n_params = sum(t[2] for t in table)
        flat = torch.empty(self._n_params, dtype=torch.float32, device=device)
        self._init_flat(flat)
        for name, off, n, shape in table:
            parts = name.split(".")
            mod: nn.Module = self
            for p in parts[:-1]:
                if p not in mod._modules:
                    mod.add_module(p, _Node())
                mod = mod._modules[p]
            mod.register_parameter(parts[-1], nn.Parameter(flat[off:off + n].view(shape)))
        self._flat = flat
        got = [n for n, _ in self.named_parameters()]
        assert got == [t[0] for t in table], "parameter order differs from the engine table"

    def _init_flat(self, flat):
        # PyTorch default Conv2d init distribution: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias
        import math
        with torch.no_grad():
            for name, off, n, shape in self._table:
                if name.endswith("weight"):
                    fan_in = int(math.prod(shape[1:]))
                else:
                    wshape = [t[3] for t in self._table if t[0] == name[:-4] + "weight"][0]
                    fan_in = int(math.prod(wshape[1:]))
                b = 1.0 / math.sqrt(fan_in)
                flat[off:off + n].uniform_(-b, b)

    def _is_flat(self) -> bool:
        base = self._flat
        for (name, off, n, shape), p in zip(self._table, self.parameters()):
            if p.device != base.device or p.data_ptr() != base.data_ptr() + 4 * off:
                return False
        return True

    def _reflatten(self):
        params = list(self.parameters())
        dev = params[0].device
        flat = torch.empty(self._n_params, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for (name, off, n, shape), p in zip(self._table, params):
                flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + n].view(shape)
        self._flat = flat
        self._engines.clear()
        self._packed_version = None

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        if not self._is_flat():
            self._reflatten()
        return r

    # -------------------------------------------------------------- engine
    def _engine_for(self, x: torch.Tensor, train: bool) -> Engine:
        if not x.is_cuda:
            raise _lib.SrmiError("srmi forward needs a GPU tensor (no CPU fallback)")
        if not self._is_flat():
            self._reflatten()
        if self._flat.device != x.device:
            raise _lib.SrmiError(f"input on {x.device}, model on {self._flat.device}")
        B, Cin, h, w = x.shape
        key = (train, h, w)
        eng = self._engines.get(key)
        if eng is None or eng.batch < B:
            eng = Engine(self.spec, max(B, eng.batch if eng else 0), (h, w), train=train, device=x.device)
            self._engines[key] = eng
            self._packed_version = None
        ver = (self._flat._version, id(eng))
        if self._packed_version != ver or getattr(eng, "_packed_for", None) != self._flat._version:
            eng.pack(self._flat)
            eng._packed_for = self._flat._version
            self._packed_version = ver
        return eng

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous().float()
        if self.training and torch.is_grad_enabled():
            return _SRNetFunction.apply(x, self, self._flat, *self.parameters())
        eng = self._engine_for(x, train=False)
        return eng.forward(self._flat, x)

    # --------------------------------------------------- FModule semantics
    def __getattr__(self, key: str) -> Any:
        parms = self.__dict__.get("parms")
        if parms is not None and key in parms:
            return parms[key]
        return super().__getattr__(key)

    def load_state_dict(self, state_dict: Mapping[str, Any], strict: bool = True, assign: bool = False):
        """Tolerant load of sres/model/common/common.py:50-71 (mismatched 'tail' keys are skipped)."""
        own = self.state_dict()
        for name, param in state_dict.items():
            if name in own:
                if isinstance(param, nn.Parameter):
                    param = param.data
                try:
                    with torch.no_grad():
                        own[name].copy_(param)
                except Exception:
                    if name.find("tail") >= 0:
                        print("Replace pre-trained upsampler to new one...")
                    else:
                        raise RuntimeError(f"While copying the parameter named {name}, whose dimensions in the model"
                                           f" are {own[name].size()} and whose dimensions in the checkpoint are "
                                           f"{param.size()}.")
            elif strict:
                if name.find("tail") == -1:
                    raise KeyError(f'unexpected key "{name}" in state_dict')
        if strict:
            missing = set(own.keys()) - set(state_dict.keys())
            if len(missing) > 0:
                raise KeyError(f'missing keys in state_dict: "{missing}"')


def _python_table(spec: NetSpec):
    """Shapes without the native library (construction / CPU-side tests)."""
    from ..engine import param_names
    names = param_names(spec)
    F, Ci, Co = spec.nfeatures, spec.nchannels_in, spec.nchannels_out
    shapes = []
    for nm in names:
        if nm.startswith("head.0."):
            s = (F, Ci, 3, 3) if nm.endswith("weight") else (F,)
        elif nm.startswith("tail.1."):
            s = (Co, F, 3, 3) if nm.endswith("weight") else (Co,)
        elif nm.startswith("tail.0."):
            s = (4 * F, F, 3, 3) if nm.endswith("weight") else (4 * F,)
        elif ".conv_du.0." in nm:
            s = (F // spec.cbottleneck, F, 1, 1) if nm.endswith("weight") else (F // spec.cbottleneck,)
        elif ".conv_du.2." in nm:
            s = (F, F // spec.cbottleneck, 1, 1) if nm.endswith("weight") else (F,)
        else:
            s = (F, F, 3, 3) if nm.endswith("weight") else (F,)
        shapes.append(s)
    out, off = [], 0
    import math
    for nm, s in zip(names, shapes):
        n = int(math.prod(s))
        out.append((nm, off, n, s))
        off += n
    return out
