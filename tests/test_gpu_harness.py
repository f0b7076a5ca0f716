"""The harness around the fused step on the GPU: model.loss_fn = 'charbonnier',
short last batches, the per-batch loss semantics of process_image / evaluate, and
the time-slice training loop with its checkpoint cadence and loss CSV
(sres/controller/dual_trainer.py:196-212, :271-347, :396-543)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import rcan_oracle as ro  # noqa: E402
from srmi._lib import call, ptr  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.trainer import FusedTrainer, default_init_  # noqa: E402


def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _small(C=2, nl=2, nb=2, seed=3):
    spec = NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=nl, nblocks=nb,
                   cbottleneck=2, scale=4)
    model = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=nl, nblocks=nb)
    ro.init_params_numpy(model, seed)
    table = param_table(spec)
    sd = dict(model.named_parameters())
    flat = torch.cat([sd[n].detach().reshape(-1).float() for n, _, _, _ in table])
    return spec, model.double(), table, flat


def test_charbonnier_step_vs_oracle():
    d = dev()
    spec, model, table, flat = _small()
    hr = ro.synthetic_hr(2, 2, 192, 31)
    tr = FusedTrainer(spec, 2, (48, 48), device=d, params=flat.to(d), loss_fn="charbonnier")
    res = tr.step(torch.tensor(hr, device=d))
    torch.cuda.synchronize()
    h = torch.tensor(hr, dtype=torch.float64)
    lr_in = ro.downsample(h, 4)
    out = model(lr_in)
    loss = ro.single_product_loss(out, h, "charbonnier")
    loss.backward()
    iloss = float(ro.single_product_loss(h, ro.upsample(lr_in, 4), "charbonnier"))
    assert abs(float(res["loss"]) - float(loss)) < 2e-3 * float(loss)
    assert abs(float(res["interp_loss"]) - iloss) < 1e-5 * iloss
    g = dict(model.named_parameters())
    grads = tr.grads.cpu()
    for name, off, n, shape in table:
        assert rel_l2(grads[off:off + n].view(shape), g[name].grad) < 8e-2, name


def test_short_batch_equals_exact_batch():
    """A short last batch (b < trainer batch, split over the micro-batch engines)
    computes the same step as a trainer of exactly that batch."""
    d = dev()
    spec, _, table, flat = _small(nl=1, nb=2)
    hr = torch.tensor(ro.synthetic_hr(5, 2, 192, 41), device=d)
    a = FusedTrainer(spec, 16, (48, 48), device=d, params=flat.to(d), micro=2)
    b = FusedTrainer(spec, 5, (48, 48), device=d, params=flat.to(d), micro=1)
    ra, rb = a.step(hr), b.step(hr)
    torch.cuda.synchronize()
    assert abs(float(ra["loss"]) - float(rb["loss"])) <= 1e-6 * float(rb["loss"])
    # different engine sizings -> different split-K chunkings of the filter gradients:
    # fp32 partial sums in another order (as in test_gpu_dp)
    assert rel_l2(a.grads, b.grads) < 2e-4
    # one tile: the second engine gets no tiles at all
    c = FusedTrainer(spec, 1, (48, 48), device=d, params=a.params.clone(), micro=1)
    r1 = a.step(hr[:1])
    rc = c.step(hr[:1])
    torch.cuda.synchronize()
    assert abs(float(r1["loss"]) - float(rc["loss"])) <= 1e-6 * float(rc["loss"])


@pytest.mark.parametrize("kind,fn", [(0, "l2"), (1, "charbonnier")])
def test_batch_losses_kernel(kind, fn):
    d = dev()
    rng = np.random.RandomState(5)
    p = torch.tensor(rng.randn(9, 2, 24, 24), dtype=torch.float32, device=d)
    t = torch.tensor(rng.randn(9, 2, 24, 24), dtype=torch.float32, device=d)
    out = torch.zeros(1 + 3, device=d)
    work = torch.zeros(9, device=d)
    call("srmi_batch_losses", ptr(p), ptr(t), 9, 2 * 24 * 24, 4, kind, 1e-6, ptr(work), ptr(out),
         torch.cuda.current_stream().cuda_stream)
    ref = ro.batch_losses(p.double().cpu(), t.double().cpu(), 4, fn)
    np.testing.assert_allclose(out[1:].cpu().numpy(), ref, rtol=1e-6)
    assert abs(float(out[0]) - np.mean(ref)) < 1e-6 * np.mean(ref)


def _flat1(seed=11):
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=1, nblocks=2, cbottleneck=2,
                   scale=4)
    model = ro.RCANOracle(nchannels_in=1, nchannels_out=1, nlayers=1, nblocks=2).double()
    ro.init_params_numpy(model, seed)
    table = param_table(spec)
    sd = dict(model.named_parameters())
    flat = torch.cat([sd[n].detach().reshape(-1).float() for n, _, _, _ in table])
    return spec, model, flat


@pytest.mark.parametrize("graph", [True, False])
def test_process_region_batch_loss_semantics(graph):
    """9 tiles scored in batches of 4 (4, 4, 1): the loss is the mean of the three
    batch RMSEs (dual_trainer.py:443-446), not the RMSE over all tiles."""
    from srmi.inference import TiledInference
    d = dev()
    spec, model, flat = _flat1()
    rng = np.random.RandomState(12)
    region = rng.randn(1, 3 * 192, 3 * 192)
    # tile row 0 smooth (random walk: the bicubic baseline does well), the rest white
    # noise: the batches' losses differ, so the mean of batch losses != all-tile loss
    region[:, :192] = np.cumsum(np.cumsum(region[:, :192], axis=1), axis=2)
    region = region.astype(np.float32)
    ti = TiledInference(spec, flat.to(d), region.shape, (192, 192), device=d, graph=graph, batch_size=4)
    images, losses = ti.process_region(torch.tensor(region, device=d))
    ref_img, ref = ro.process_region(model, region.astype(np.float64), 192, 192, 4, batch_size=4)
    b = ti.batch_losses()
    np.testing.assert_allclose(b["interpolated"].cpu().numpy(), ref["batch_interpolated"], rtol=1e-5)
    np.testing.assert_allclose(b["model"].cpu().numpy(), ref["batch_model"], rtol=2e-3)
    assert abs(float(losses["interpolated"]) - ref["interpolated"]) < 1e-5 * ref["interpolated"]
    assert abs(float(losses["model"]) - ref["model"]) < 2e-3 * ref["model"]
    rmse_all = float(np.sqrt(np.mean([x ** 2 for x in ref["batch_interpolated"]])))  # the old all-tile form
    assert abs(rmse_all - ref["interpolated"]) > 1e-3 * ref["interpolated"]


def test_evaluate_vs_oracle_and_validation_policy(tmp_path):
    from srmi.harness import CheckpointStore, ValidationCheckpoint
    from srmi.inference import TiledInference
    d = dev()
    spec, model, flat = _flat1()
    rng = np.random.RandomState(13)
    regions = [rng.randn(1, 2 * 192, 3 * 192).astype(np.float32) for _ in range(2)]
    ti = TiledInference(spec, flat.to(d), regions[0].shape, (192, 192), device=d, graph=True, batch_size=4)
    res, losses = ti.evaluate([torch.tensor(r, device=d) for r in regions])
    ref_res, ref = ro.evaluate(model, [r.astype(np.float64) for r in regions], 192, 192, 4, batch_size=4)
    # results: the last time slice's 6 tiles (clear_results per slice, dual_trainer.py:505, :545-549)
    assert res["model"].shape == (6, 1, 192, 192) and res["input"].shape == (6, 1, 48, 48)
    assert rel_l2(res["target"], ref_res["target"]) < 1e-5
    assert rel_l2(res["interpolated"], ref_res["interpolated"]) < 1e-5
    assert rel_l2(res["model"], ref_res["model"]) < 2e-2
    assert abs(losses["interpolated"] - ref["interpolated"]) < 1e-5 * ref["interpolated"]
    assert abs(losses["model"] - ref["model"]) < 2e-3 * ref["model"]
    # the validation checkpoint follows evaluate's improvement policy
    tr = FusedTrainer(spec, 4, (48, 48), device=d, params=flat.to(d), micro=1)
    store = CheckpointStore(str(tmp_path), "sres-rcan-test")
    vc = ValidationCheckpoint()
    save = lambda ml, il: store.save(tr, 1, 0, "valid", ml)  # noqa: E731
    assert vc.update(losses["model"], losses["interpolated"], save)
    assert os.path.exists(store.path("valid"))
    assert not vc.update(losses["model"] * 1.01, losses["interpolated"], save)
    # the saved validation weights reload into the inference engines
    state = torch.load(store.path("valid"), weights_only=True)
    assert abs(state["loss"] - losses["model"]) < 1e-12
    ti.set_params(tr.params)


def test_evaluate_time_and_tile_index_selection_vs_oracle():
    """evaluate(time_index=, tile_index=) (dual_trainer.py:487-488, :504-527,
    tile_in_batch :366-372) against the oracle's restatement: one time slice, one
    batch per slice (tile domain and time domain), no matching batch."""
    from srmi.inference import TiledInference
    d = dev()
    spec, model, flat = _flat1()
    rng = np.random.RandomState(19)
    regions = [rng.randn(1, 2 * 192, 3 * 192).astype(np.float32) for _ in range(3)]
    ti = TiledInference(spec, flat.to(d), regions[0].shape, (192, 192), device=d, graph=True, batch_size=4)
    dr = [torch.tensor(r, device=d) for r in regions]
    r64 = [r.astype(np.float64) for r in regions]
    for kw in (dict(time_index=1), dict(tile_index=5), dict(time_index=2, tile_index=2),
               dict(tile_index=1, batch_domain="time"), dict(time_index=0, tile_index=0, batch_domain="time")):
        res, losses = ti.evaluate(dr, **kw)
        ref_res, ref = ro.evaluate(model, r64, 192, 192, 4, batch_size=4, **kw)
        for k in ("input", "target", "model", "interpolated"):
            assert tuple(res[k].shape) == ref_res[k].shape, (kw, k)
        assert rel_l2(res["target"], ref_res["target"]) < 1e-5
        assert abs(losses["interpolated"] - ref["interpolated"]) < 1e-5 * ref["interpolated"], kw
        assert abs(losses["model"] - ref["model"]) < 2e-3 * ref["model"], kw
    res, losses = ti.evaluate(dr, tile_index=6)  # 6 tiles per slice: no batch holds tile 6
    assert res["model"].numel() == 0 and np.isnan(losses["model"])


def test_process_image_var_selection():
    """process_image's per-variable return and kwargs 'var' (dual_trainer.py:413-414,
    :437-446): with var given, the images under that name are channel 0 (ivar from
    enumerate(output_vars)), the losses are those of all channels."""
    from srmi.inference import TiledInference
    d = dev()
    spec, _, table, flat = _small(C=2, nl=1, nb=1)
    rng = np.random.RandomState(23)
    region = torch.tensor(rng.randn(2, 192, 2 * 192).astype(np.float32), device=d)
    ti = TiledInference(spec, flat.to(d), tuple(region.shape), (192, 192), device=d, graph=False, batch_size=4)
    imgs, losses = ti.process_image(region, ["SSS", "SST"])
    imgs = {v: {k: t.clone() for k, t in d_.items()} for v, d_ in imgs.items()}  # (views of the engine's buffers)
    assert sorted(imgs) == ["SSS", "SST"] and imgs["SST"]["model"].shape == (192, 384)
    full, fl = ti.process_region(region)
    assert torch.equal(imgs["SST"]["model"], full["model"][1]) and torch.equal(imgs["SSS"]["target"], full["target"][0])
    assert losses["SST"] == losses["SSS"] == {"model": float(fl["model"]), "interpolated": float(fl["interpolated"])}
    one, l1 = ti.process_image(region, ["SSS", "SST"], var="SST")
    assert list(one) == ["SST"] and torch.equal(one["SST"]["model"], full["model"][0])
    assert l1["SST"] == losses["SST"]


def test_evaluate_graph_replay_after_compacted_region():
    """[clean, one NaN tile, clean] with the graph path: the middle region takes the
    compacted (tile-dropping) path, the last one replays the graph; the results
    are the last region's full tile set (target as long as model), and the losses
    average every batch of all three regions, as the oracle computes them."""
    from srmi.inference import TiledInference
    d = dev()
    spec, model, flat = _flat1()
    rng = np.random.RandomState(17)
    regions = [rng.randn(1, 2 * 192, 3 * 192).astype(np.float32) for _ in range(3)]
    regions[1][0, 200, 5] = np.nan  # tile (1, 0) of the middle region is dropped
    ti = TiledInference(spec, flat.to(d), regions[0].shape, (192, 192), device=d, graph=True, batch_size=4)
    res, losses = ti.evaluate([torch.tensor(r, device=d) for r in regions])
    ref_res, ref = ro.evaluate(model, [r.astype(np.float64) for r in regions], 192, 192, 4, batch_size=4)
    for k in ("input", "target", "model", "interpolated"):
        assert res[k].shape[0] == 6 == ref_res[k].shape[0], k
    assert rel_l2(res["target"], ref_res["target"]) < 1e-6
    assert rel_l2(res["interpolated"], ref_res["interpolated"]) < 1e-5
    assert rel_l2(res["model"], ref_res["model"]) < 2e-2
    assert abs(losses["interpolated"] - ref["interpolated"]) < 1e-5 * ref["interpolated"]
    assert abs(losses["model"] - ref["model"]) < 2e-3 * ref["model"]


def test_train_timeslices_checkpoints_csv_and_resume(tmp_path):
    """dual_trainer.train's loop: a train checkpoint (+ .backup) after every time
    slice, loss rows [tset, epoch, loss, ref_loss], and a resumed run continuing
    from (epoch, itime) reproduces the uninterrupted one."""
    import random
    from srmi.harness import CheckpointStore, LossRecords, train_timeslices
    d = dev()
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=1, nblocks=1, cbottleneck=2,
                   scale=4)
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=2)
    slices = [torch.tensor(ro.synthetic_hr(5, 1, 192, 50 + i), device=d) for i in range(3)]
    ts = [(lambda i=i: slices[i]) for i in range(3)]
    # from scratch, nepochs=3: epochs range(1, 3) (the reference's loop bounds, :279, :296)
    a = FusedTrainer(spec, 2, (48, 48), device=d, params=flat, micro=1)
    sa = CheckpointStore(str(tmp_path / "a"), "sres-rcan-x")
    ra = LossRecords(str(tmp_path / "a"), "swot", "SST-tiles-48", "rcan")
    out_a = train_timeslices(a, ts, 3, 2, store=sa, records=ra, refresh_state=True, rng=random.Random(0))
    rows = ra.load_results()
    assert len(rows) == 6 and rows[0][0] == "train" and rows[0][1] == "0.000" and rows[1][1] == "0.333"
    assert all(len(r) == 4 and len(r[2].split(".")[1]) == 6 for r in rows)
    assert os.path.exists(sa.path("train")) and os.path.exists(sa.path("train", backup=True))
    st = torch.load(sa.path("train"), weights_only=True)
    assert st["epoch"] == 2 and st["itime"] == 2 and abs(st["loss"] - out_a["prediction"]) < 1e-12
    # one epoch (nepochs=2), then the train checkpoint restores a fresh trainer
    b = FusedTrainer(spec, 2, (48, 48), device=d, params=flat, micro=1)
    sb = CheckpointStore(str(tmp_path / "b"), "sres-rcan-x")
    rng = random.Random(0)
    train_timeslices(b, ts, 2, 2, store=sb, refresh_state=True, rng=rng)
    c = FusedTrainer(spec, 2, (48, 48), device=d, params=torch.zeros_like(flat), micro=1)
    # resume: epoch0 = 1 and itime0 = 2 from the file -> replays time slice 2 of epoch 1
    # (the reference's itime0 quirk), then epoch 2 in full
    state = sb.load(c, "train", update_model=True)
    assert state["epoch"] == 1 and state["itime"] == 2 and c.t == b.t
    torch.cuda.synchronize()
    assert torch.equal(c.params, b.params)


def test_target_channel_subset_step_vs_oracle():
    """apply_network's index_select (dual_trainer.py:564-568): a 2-variable input
    with target_variables = [SST] trains a 2-in / 1-out model against HR channel 1;
    the interp metric is loss(btarget, upsample(binput)) with the 1-channel target
    broadcast over the 2 interpolated channels, as torch evaluates it (:316-317)."""
    d = dev()
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=1, nfeatures=64, nlayers=1, nblocks=2,
                   cbottleneck=2, scale=4)
    model = ro.RCANOracle(nchannels_in=2, nchannels_out=1, nlayers=1, nblocks=2)
    ro.init_params_numpy(model, 5)
    table = param_table(spec)
    sd = dict(model.named_parameters())
    flat = torch.cat([sd[n].detach().reshape(-1).float() for n, _, _, _ in table])
    task = {"input_variables": {"SSS": "a", "SST": "b"}, "target_variables": ["SST"]}
    hr = ro.synthetic_hr(4, 2, 192, 77)
    tr = FusedTrainer(spec, 4, (48, 48), device=d, params=flat.to(d), task=task)
    res = tr.step(torch.tensor(hr, device=d))
    torch.cuda.synchronize()
    model = model.double()
    h = torch.tensor(hr, dtype=torch.float64)
    lr_in = ro.downsample(h, 4)
    tgt = h[:, 1:2]
    out = model(lr_in)
    loss = ro.l2loss(out, tgt)
    loss.backward()
    iloss = float(ro.l2loss(tgt, ro.upsample(lr_in, 4)))  # broadcast [4,1] against [4,2]
    assert abs(float(res["loss"]) - float(loss)) < 2e-3 * float(loss)
    assert abs(float(res["interp_loss"]) - iloss) < 1e-5 * iloss
    g = dict(model.named_parameters())
    grads = tr.grads.cpu()
    for name, off, n, shape in table:
        assert rel_l2(grads[off:off + n].view(shape), g[name].grad) < 8e-2, name


@pytest.mark.parametrize("task,side", [
    ({"data_downsample": 2}, 384),
    ({"data_downsample": 3, "downsample_mode": "linear", "upsample_mode": "linear"}, 576),
    ({"data_downsample": 1.5}, 289),   # floor(289 / 1.5) = 192 (F.interpolate's size)
    ({"downsample_mode": "linear", "upsample_mode": "cubic"}, 192),
    ({"downsample_mode": "cubic", "upsample_mode": "linear"}, 192),
])
def test_data_downsample_step_vs_oracle(task, side):
    """apply_network's data_downsample (dual_trainer.py:561-563) at even, odd and
    fractional factors, and task.downsample_mode / upsample_mode (torch_interp_mode,
    array.py:37-41: 'linear' -> bilinear, 'cubic' -> bicubic): the HR batch is
    downsampled by ds first and becomes both the loss target and the source of the
    model input (downsample_mode); the interp metric compares it with the upsampled
    input (upsample_mode, :316-317)."""
    from srmi.config import data_downsample_factor, interp_mode
    d = dev()
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=1, nblocks=2,
                   cbottleneck=2, scale=4)
    model = ro.RCANOracle(nchannels_in=2, nchannels_out=2, nlayers=1, nblocks=2)
    ro.init_params_numpy(model, 6)
    table = param_table(spec)
    sd = dict(model.named_parameters())
    flat = torch.cat([sd[n].detach().reshape(-1).float() for n, _, _, _ in table])
    hr = ro.synthetic_hr(4, 2, side, 78)
    tr = FusedTrainer(spec, 4, (48, 48), device=d, params=flat.to(d), task=task)
    res = tr.step(torch.tensor(hr, device=d))
    torch.cuda.synchronize()
    ds = data_downsample_factor(task)
    dm, um = interp_mode(task, True), interp_mode(task, False)
    if ds > 1:
        with pytest.raises(ValueError, match="data_downsample"):  # tiles of the wrong size
            tr.step(torch.zeros(4, 2, 192, 192, device=d))
    model = model.double()
    h = torch.tensor(hr, dtype=torch.float64)
    if ds > 1:
        h = ro.downsample(h, ds, dm)
    assert tuple(h.shape[2:]) == (192, 192)
    lr_in = ro.downsample(h, 4, dm)
    out = model(lr_in)
    loss = ro.l2loss(out, h)
    loss.backward()
    iloss = float(ro.l2loss(h, ro.upsample(lr_in, 4, um)))
    assert abs(float(res["loss"]) - float(loss)) < 2e-3 * float(loss)
    assert abs(float(res["interp_loss"]) - iloss) < 1e-5 * iloss
    g = dict(model.named_parameters())
    grads = tr.grads.cpu()
    for name, off, n, shape in table:
        assert rel_l2(grads[off:off + n].view(shape), g[name].grad) < 8e-2, name
