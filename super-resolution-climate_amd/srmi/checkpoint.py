"""Checkpoints in the reference's format.

CheckpointManager.save_checkpoint (sres/controller/checkpoints.py:18-26) writes
``dict(epoch, itime, model_state_dict, optimizer_state_dict, loss)`` with
``torch.save``; load_checkpoint (:35-51) restores the model and the
``torch.optim.Adam`` state.  The plugin path (srmi.model.*: an nn.Module plus a
real torch Adam) goes through that manager unchanged.  For the fused trainer,
whose parameters and Adam moments live in flat device buffers, these helpers
convert between the flat buffers and the exact torch state-dict layouts, so a
checkpoint written by either side resumes on the other:

* model_state_dict: the reference's keys/shapes (state-dict order);
* optimizer_state_dict: torch.optim.Adam's ``{"state": {i: {"step",
  "exp_avg", "exp_avg_sq"}}, "param_groups": [...]}`` with parameter index i
  in ``model.parameters()`` order (= state-dict order for these networks).
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import torch


def model_state_dict(flat: torch.Tensor, table) -> Dict[str, torch.Tensor]:
    host = flat.detach().float().cpu()
    return {name: host[off:off + n].view(shape).clone() for name, off, n, shape in table}


def load_model_state_dict(flat: torch.Tensor, table, sd: Dict[str, torch.Tensor], strict: bool = True,
                          apply: bool = True) -> torch.Tensor:
    """A reference state dict -> the flat layout, with FModule.load_state_dict's
    semantics (sres/model/common/common.py:50-71): a key whose shape differs is
    skipped if it is under 'tail' (a re-shaped upsampler) and raises otherwise;
    with strict, unexpected keys not under 'tail' and missing keys raise.  Returns
    the host buffer; apply copies it into `flat`."""
    host = flat.detach().cpu().clone()
    names = {name for name, _, _, _ in table}
    if strict:
        extra = [k for k in sd if k not in names and "tail" not in k]
        if extra:
            raise KeyError(f'unexpected key "{extra[0]}" in state_dict')
        missing = names - set(sd)
        if missing:
            raise KeyError(f'missing keys in state_dict: "{missing}"')
    for name, off, n, shape in table:
        if name not in sd:
            continue
        t = sd[name]
        if tuple(t.shape) != tuple(shape):
            if "tail" in name:
                continue
            raise RuntimeError(f"While copying the parameter named {name}, whose dimensions in the model are "
                               f"{tuple(shape)} and whose dimensions in the checkpoint are {tuple(t.shape)}.")
        host[off:off + n] = t.detach().float().reshape(-1)
    if apply:
        flat.copy_(host)
    return host


def adam_state_dict(table, m: torch.Tensor, v: torch.Tensor, step: int, lr: float, betas=(0.9, 0.999),
                    eps: float = 1e-8, weight_decay: float = 0.0) -> Dict:
    """torch.optim.Adam.state_dict() layout for the flat moments."""
    mh, vh = m.detach().float().cpu(), v.detach().float().cpu()
    state = {}
    if step > 0:
        for i, (_, off, n, shape) in enumerate(table):
            state[i] = {"step": torch.tensor(float(step)), "exp_avg": mh[off:off + n].view(shape).clone(),
                        "exp_avg_sq": vh[off:off + n].view(shape).clone()}
    group = {"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay, "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
             "decoupled_weight_decay": False, "params": list(range(len(table)))}
    return {"state": state, "param_groups": [group]}


def load_adam_state_dict(table, sd: Dict, m: torch.Tensor, v: torch.Tensor, apply: bool = True):
    """Flat moments from a torch Adam state dict.  All parameters must share one step
    count (one param group, as dual_trainer.py:126).  apply=True copies the moments
    into m, v and returns (step, param-group hyper-parameters); apply=False leaves
    them and returns (step, hyper-parameters, m_host, v_host)."""
    groups = sd["param_groups"]
    if len(groups) != 1 or len(groups[0]["params"]) != len(table):
        raise ValueError("expected one Adam param group over all model parameters")
    mh = torch.zeros(m.numel(), dtype=torch.float32)
    vh = torch.zeros(v.numel(), dtype=torch.float32)
    steps = set()
    for i, (name, off, n, shape) in enumerate(table):
        st = sd["state"].get(groups[0]["params"][i])
        if st is None:
            steps.add(0)
            continue
        steps.add(int(float(st["step"])))
        for key, dst in (("exp_avg", mh), ("exp_avg_sq", vh)):
            x = st[key]
            if x.numel() != n:
                raise ValueError(f"{name}: Adam {key} has {x.numel()} elements, expected {n}")
            dst[off:off + n] = x.float().reshape(-1)
    if len(steps) != 1:
        raise ValueError(f"parameters at different Adam steps: {sorted(steps)}")
    g = groups[0]
    hp = {k: g[k] for k in ("lr", "betas", "eps", "weight_decay")}
    if not apply:
        return steps.pop(), hp, mh, vh
    m.copy_(mh)
    v.copy_(vh)
    return steps.pop(), hp


def checkpoint(epoch: int, itime: int, flat, table, m, v, step, lr, betas, eps, wd, loss: float) -> Dict:
    """The dict CheckpointManager.save_checkpoint writes (checkpoints.py:20)."""
    return dict(epoch=epoch, itime=itime, model_state_dict=model_state_dict(flat, table),
                optimizer_state_dict=adam_state_dict(table, m, v, step, lr, betas, eps, wd), loss=loss)
