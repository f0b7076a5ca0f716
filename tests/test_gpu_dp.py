"""Data-parallel training step on the HIP path, world size 2, both ranks on cuda:0
with the gloo backend (the pool's boxes have one GPU; gloo all-reduces CUDA
tensors).  Exercises the real product path of srmi.trainer.FusedTrainer +
srmi.dist.GradReducer: per-group HIP events of BOTH micro-batch engines, the
per-bucket micro-batch gradient sum (srmi_axpy) on the communication stream and
the bucketed all-reduce overlapped with backward.  2 ranks x 8 tiles must equal
1 process x 16 tiles (global RMSE, summed gradients) to fp32 summation order
(2e-4 rel-L2 on the gradient)."""
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _spec():
    from srmi.engine import NetSpec
    return NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=2, nblocks=3, cbottleneck=2,
                   scale=4)


def _worker(rank, port, q, reducer_stream=False):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from oracle import rcan_oracle as ro
    from srmi.dist import init_from_env, shard_range
    from srmi.engine import param_table
    from srmi.trainer import FusedTrainer, default_init_
    info = init_from_env("gloo")
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    spec = _spec()
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=5)
    hr_all = torch.tensor(ro.synthetic_hr(16, 2, 192, 17)).to(d)
    a, b = shard_range(16, info)
    tr = FusedTrainer(spec, b - a, (48, 48), device=d, params=flat, micro=2, info=info,
                      dp_reducer_stream=reducer_stream)
    out = tr.step(hr_all[a:b].contiguous())
    torch.cuda.synchronize()
    q.put((rank, float(out["loss"]), float(out["interp_loss"]), tr.grads.cpu().numpy(), tr.params.cpu().numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("reducer_stream", [False, True])
def test_dp_world2_micro2_matches_single_process(reducer_stream):
    """Both DP schedules: the default staged one (backward enqueued stage by stage,
    each bucket's gradient add and all-reduce behind its stage on engine 1's stream)
    and the reducer stream waiting on the group events (dp_reducer_stream)."""
    import multiprocessing as mp
    from oracle import rcan_oracle as ro
    from srmi.engine import param_table
    from srmi.trainer import FusedTrainer, default_init_
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31000 + random.randint(0, 2000)
    ps = [ctx.Process(target=_worker, args=(r, port, q, reducer_stream)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=100) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    d = torch.device("cuda", 0)
    spec = _spec()
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=5)
    hr = torch.tensor(ro.synthetic_hr(16, 2, 192, 17)).to(d)
    tr = FusedTrainer(spec, 16, (48, 48), device=d, params=flat, micro=1)
    out = tr.step(hr)
    torch.cuda.synchronize()
    loss, iloss, g = float(out["loss"]), float(out["interp_loss"]), tr.grads.cpu().numpy()
    for rank, l_r, il_r, g_r, p_r in res:
        assert abs(l_r - loss) <= 1e-6 * abs(loss), (rank, l_r, loss)
        assert abs(il_r - iloss) <= 1e-6 * abs(iloss)
        # micro-batch engines of 4 tiles vs one engine of 16: different split-K chunkings
        # of the filter gradients, so fp32 partial sums add in a different order
        # (strong cancellation in weight gradients amplifies that to ~4e-5)
        assert np.linalg.norm(g_r - g) / np.linalg.norm(g) < 2e-4
    np.testing.assert_array_equal(res[0][4], res[1][4])  # replicas stay identical after Adam


def test_group_events_exist_before_backward():
    """The reducer's per-group events (and every micro-batch engine's extra set) must
    hold a real HIP event before the first backward: torch.cuda.Event creates it
    lazily, and a NULL handle would make the engine skip the record and the bucket's
    wait_event a no-op (the all-reduce would then race the backward)."""
    import sys
    sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
    from srmi.dist import DistInfo, GradReducer
    from srmi.engine import Engine, param_table
    d = torch.device("cuda", 0)
    spec = _spec()
    red = GradReducer(param_table(spec), "rcan", spec.nlayers, DistInfo(rank=0, world=2), d)
    assert red.n_events == spec.nlayers
    for evs in (red.events, red.new_events()):
        assert len(evs) == spec.nlayers and all(ev.cuda_event for ev in evs)
    with pytest.raises(RuntimeError, match="group event"):
        Engine.backward(None, None, None, None, events=[torch.cuda.Event()])


def _force_dp_rccl_worker(port, q, reducer_stream=False):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from oracle import rcan_oracle as ro
    from srmi.dist import init_from_env
    from srmi.engine import param_table
    from srmi.trainer import FusedTrainer, default_init_
    info = init_from_env("nccl", force=True)
    assert info.enabled and dist.get_backend() == "nccl"
    d = torch.device("cuda", 0)
    spec = _spec()
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table), device=d)
    default_init_(flat, table, seed=6)
    hr = torch.tensor(ro.synthetic_hr(16, 2, 192, 23)).to(d)
    dp = FusedTrainer(spec, 16, (48, 48), device=d, params=flat, micro=2, info=info,
                      dp_reducer_stream=reducer_stream)
    ref = FusedTrainer(spec, 16, (48, 48), device=d, params=flat, micro=2)
    out = []
    for _ in range(2):
        a, b = dp.step(hr), ref.step(hr)
        torch.cuda.synchronize()
        out.append((float(a["loss"]), float(b["loss"]), torch.equal(dp.grads, ref.grads),
                    float((dp.grads - ref.grads).abs().max())))
    q.put((out, torch.equal(dp.params, ref.params)))
    dist.destroy_process_group()


@pytest.mark.parametrize("reducer_stream", [False, True])
def test_force_dp_rccl_bucketed_allreduce_waits_for_backward(reducer_stream):
    """The DP path over a real RCCL communicator (backend "nccl", one rank): every
    bucket's micro-batch gradient sum and all-reduce run behind the backward stage
    that finalises it (the default: on engine 1's stream after engine 0's stage
    event) or on the reducer stream behind the engines' group events.  At one rank the
    SUM all-reduce is the identity, so the gradients must equal the non-DP step's bit
    for bit -- a bucket that did not wait for its backward group would read
    unfinished gradients and differ."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_force_dp_rccl_worker, args=(33000 + random.randint(0, 2000), q, reducer_stream))
    p.start()
    out, params_equal = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    for l_dp, l_ref, g_equal, gmax in out:
        assert l_dp == l_ref and g_equal, (l_dp, l_ref, gmax)
    assert params_equal


def _infer_worker(rank, port, q, regions, flat_np):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from srmi.dist import init_from_env
    from srmi.engine import NetSpec
    from srmi.inference import TiledInference
    info = init_from_env("gloo")
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=1, nblocks=2, cbottleneck=2,
                   scale=4)
    ti = TiledInference(spec, torch.tensor(flat_np, device=d), regions[0].shape, (192, 192), device=d,
                        batch_size=4, info=info)
    out = []
    for r in regions:
        images, losses = ti.process_region(torch.tensor(r, device=d))
        b = ti.batch_losses()
        torch.cuda.synchronize()
        out.append(({k: v.cpu().numpy() for k, v in images.items()}, float(losses["model"]),
                    float(losses["interpolated"]), b["model"].cpu().numpy(), b["interpolated"].cpu().numpy()))
    res, el = ti.evaluate([torch.tensor(r, device=d) for r in regions])
    q.put((rank, out, {k: v.cpu().numpy() for k, v in res.items()}, el))
    dist.destroy_process_group()


def test_multirank_tiled_inference_world2_bit_identical_to_one_rank():
    """SURVEY.md §8(e) for C5: the region's tiles dealt round-robin over 2 ranks
    (gloo, both on cuda:0), mosaics and per-batch losses all-gathered -- bit-identical
    to the one-rank TiledInference (graph replay, two micro-batch engines), also for
    a region with a dropped (non-finite) tile, and through evaluate()."""
    import multiprocessing as mp
    from srmi.engine import NetSpec, param_table
    from srmi.inference import TiledInference
    from srmi.trainer import default_init_
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=1, nblocks=2, cbottleneck=2,
                   scale=4)
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table))
    default_init_(flat, table, seed=8)
    rng = np.random.RandomState(29)
    regions = [rng.randn(1, 5 * 192, 7 * 192 + 50).astype(np.float32) for _ in range(2)]  # 35 tiles, ragged edge
    regions[1][0, 2 * 192 + 7, 3 * 192 + 9] = np.inf
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 37000 + random.randint(0, 2000)
    ps = [ctx.Process(target=_infer_worker, args=(r, port, q, regions, flat.numpy())) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=200) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    d = torch.device("cuda", 0)
    ti = TiledInference(spec, flat.to(d), regions[0].shape, (192, 192), device=d, batch_size=4)
    for i, r in enumerate(regions):
        images, losses = ti.process_region(torch.tensor(r, device=d))
        b = ti.batch_losses()
        torch.cuda.synchronize()
        for rank, out, _, _ in res:
            im_r, lm, li, bm, bi = out[i]
            for k, v in images.items():
                np.testing.assert_array_equal(im_r[k], v.cpu().numpy(), err_msg=f"rank {rank} region {i} {k}")
            assert lm == float(losses["model"]) and li == float(losses["interpolated"])
            np.testing.assert_array_equal(bm, b["model"].cpu().numpy())
            np.testing.assert_array_equal(bi, b["interpolated"].cpu().numpy())
    ref_res, ref_l = ti.evaluate([torch.tensor(r, device=d) for r in regions])
    for rank, _, er, el in res:
        assert el == ref_l
        for k, v in ref_res.items():
            np.testing.assert_array_equal(er[k], v.cpu().numpy())


def _harness_worker(rank, port, q, root, flat_np):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from oracle import rcan_oracle as ro
    from srmi.dist import init_from_env
    from srmi.harness import CheckpointStore, LossRecords, train_timeslices
    from srmi.trainer import FusedTrainer
    info = init_from_env("gloo")
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    slices = [torch.tensor(ro.synthetic_hr(13, 2, 192, 60 + i)).to(d) for i in range(2)]
    # ceil(4 / 2) = 2 tiles per rank, as two micro-batch engines of one tile
    tr = FusedTrainer(_spec(), 2, (48, 48), device=d, params=torch.tensor(flat_np, device=d), micro=2, info=info)
    rec = []
    step = tr.step

    def recording_step(hr, shard=None):
        p = tr.params.clone()
        out = step(hr, shard=shard)
        torch.cuda.synchronize()
        rec.append((p.cpu().numpy(), float(out["loss"]), float(out["interp_loss"]), tr.grads.cpu().numpy(),
                    hr.shape[0], shard))
        return out
    tr.step = recording_step
    out = train_timeslices(tr, [lambda i=i: slices[i] for i in range(2)], 2, 4,
                           store=CheckpointStore(root, "dp"), records=LossRecords(root, "ds", "t", "m"),
                           refresh_state=True, rng=random.Random(3))
    q.put((rank, rec, out, tr.params.cpu().numpy()))
    dist.destroy_process_group()


def test_train_timeslices_world2_matches_one_process(tmp_path):
    """C3's training loop (dual_trainer.py:301-331; TileBatchIterator tiles.py:55-72)
    on the HIP path at world 2 (gloo, both ranks on cuda:0): 2 time slices of 13 tiles
    at batch_size 4, so every slice ends with a 1-tile batch that rank 1 has no tile
    of.  Replayed step by step in one process (its params set to the ranks' params
    before each step): every loss is bit-identical (the global batch's per-tile loss
    parts, all-reduced and summed in tile order), the gradients agree to fp32 summation
    order (2e-4 rel-L2), the replicas stay identical after Adam, and rank 0 alone wrote
    one checkpoint (+ backup) and one CSV row per time slice."""
    import multiprocessing as mp
    from oracle import rcan_oracle as ro
    from srmi.engine import param_table
    from srmi.harness import LossRecords, train_timeslices
    from srmi.trainer import FusedTrainer, default_init_
    spec = _spec()
    table = param_table(spec)
    flat = torch.empty(sum(t[2] for t in table))
    default_init_(flat, table, seed=9)
    root = str(tmp_path / "dp")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 41000 + random.randint(0, 2000)
    ps = [ctx.Process(target=_harness_worker, args=(r, port, q, root, flat.numpy())) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=200) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    (_, rec0, out0, p0), (_, rec1, out1, p1) = res
    assert len(rec0) == len(rec1) == 8
    np.testing.assert_array_equal(p0, p1)
    assert out0 == out1
    assert [r[4] for r in rec1].count(0) == 2   # rank 1 had no tile of either 1-tile batch
    assert all(r0[1] == r1[1] for r0, r1 in zip(rec0, rec1))
    # one process, same rng, each step from the ranks' params
    d = torch.device("cuda", 0)
    slices = [torch.tensor(ro.synthetic_hr(13, 2, 192, 60 + i)).to(d) for i in range(2)]
    one = FusedTrainer(spec, 4, (48, 48), device=d, params=flat.to(d), micro=1)
    step, k = one.step, [0]

    def replay(hr, shard=None):
        p_dp, l_dp, il_dp, g_dp, _, _ = rec0[k[0]]
        one.params.copy_(torch.tensor(p_dp, device=d))
        for e in one.engines:
            e.pack(one.params)
        out = step(hr, shard=shard)
        torch.cuda.synchronize()
        assert float(out["loss"]) == l_dp and float(out["interp_loss"]) == il_dp, k[0]
        g = one.grads.cpu().numpy()
        assert np.linalg.norm(g_dp - g) / np.linalg.norm(g) < 2e-4, k[0]
        k[0] += 1
        return out
    one.step = replay
    train_timeslices(one, [lambda i=i: slices[i] for i in range(2)], 2, 4, rng=random.Random(3))
    assert k[0] == 8
    assert sorted(os.listdir(os.path.join(root, "checkpoints"))) == ["dp.train.backup.pt", "dp.train.pt"]
    rows = LossRecords(root, "ds", "t", "m").load_results()
    assert [r[1] for r in rows] == ["0.000", "0.500"]
