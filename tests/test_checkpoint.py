"""Checkpoint compatibility: srmi.checkpoint converts the
fused trainer's flat weights / Adam moments to and from the exact layouts of the
reference's CheckpointManager (sres/controller/checkpoints.py:18-51): the model
state dict of the reference network and torch.optim.Adam.state_dict()."""
import io

import torch

from oracle import rcan_oracle as ro
from srmi import checkpoint as ck
from srmi.engine import NetSpec
from srmi.model.common import _python_table


def _setup():
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=1, nblocks=2)
    table = _python_table(spec)
    model = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=1, nblocks=2)
    ro.init_params_numpy(model, 0)
    return table, model


def test_adam_state_dict_round_trip_with_torch_adam():
    table, model = _setup()
    assert [n for n, _, _, _ in table] == [n for n, _ in model.named_parameters()]
    opt = torch.optim.Adam(model.parameters(), lr=3e-4, weight_decay=1e-5)
    hr = torch.tensor(ro.synthetic_hr(2, 2, 48, 5))
    for _ in range(2):
        opt.zero_grad()
        ro.l2loss(model(ro.downsample(hr, 4)), hr).backward()
        opt.step()
    n = sum(t[2] for t in table)
    m, v = torch.zeros(n), torch.zeros(n)
    step, hp = ck.load_adam_state_dict(table, opt.state_dict(), m, v)
    assert step == 2 and hp["lr"] == 3e-4 and hp["weight_decay"] == 1e-5
    sd = ck.adam_state_dict(table, m, v, step, hp["lr"], hp["betas"], hp["eps"], hp["weight_decay"])
    ref = opt.state_dict()
    for i in ref["state"]:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sd["state"][i][k], ref["state"][i][k])
        assert float(sd["state"][i]["step"]) == float(ref["state"][i]["step"])
    # a fresh torch Adam accepts our dict and continues identically
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    model2 = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=1, nblocks=2)
    ck.load_model_state_dict(flat, table, ck.model_state_dict(flat, table))
    model2.load_state_dict(ck.model_state_dict(flat, table))
    opt2 = torch.optim.Adam(model2.parameters(), lr=1.0)
    opt2.load_state_dict(sd)
    for o, mm in ((opt, model), (opt2, model2)):
        o.zero_grad()
        ro.l2loss(mm(ro.downsample(hr, 4)), hr).backward()
        o.step()
    for p1, p2 in zip(model.parameters(), model2.parameters()):
        assert torch.equal(p1, p2)


def test_checkpoint_dict_is_torch_save_loadable():
    table, model = _setup()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    n = flat.numel()
    c = ck.checkpoint(3, 7, flat, table, torch.zeros(n), torch.zeros(n), 0, 1e-4, (0.9, 0.999), 1e-8, 0.0, 0.5)
    buf = io.BytesIO()
    torch.save(c, buf)
    buf.seek(0)
    back = torch.load(buf, weights_only=True)
    assert back["epoch"] == 3 and back["itime"] == 7 and back["loss"] == 0.5
    model.load_state_dict(back["model_state_dict"])  # the reference network accepts it
    assert back["optimizer_state_dict"]["state"] == {}
