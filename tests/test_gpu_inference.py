"""Tiled-region inference on the HIP path (srmi.inference.TiledInference, the
srmi_region_to_tiles / srmi_tiles_to_region kernels) against the oracle's
restatement of process_image + assemble_images (parity pinned by restatement:
the reference's own functions need xarray, which is absent)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import rcan_oracle as ro  # noqa: E402
from srmi._lib import call, ptr  # noqa: E402
from srmi.engine import NetSpec, param_table  # noqa: E402
from srmi.inference import TiledInference  # noqa: E402


def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def rel_l2(a, b):
    a = torch.as_tensor(np.asarray(a, dtype=np.float64))
    b = torch.as_tensor(np.asarray(b, dtype=np.float64))
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


# W % 4 != 0: the scalar region_to_tiles; == 0: the register-resident one.  tx % 4 != 0:
# the scalar tiles_to_region; == 0: the float4 one
@pytest.mark.parametrize("wextra,tx", [(3, 56), (4, 56), (3, 55)])
def test_region_tiles_kernels(wextra, tx):
    d = dev()
    rng = np.random.RandomState(4)
    region = (rng.randn(2, 3 * 40 + 7, 2 * 56 + wextra) * 3 + 1).astype(np.float32)
    C, H, W = region.shape
    ty = 40
    n = (H // ty) * (W // tx)
    rg = torch.tensor(region, device=d)
    tiles = torch.empty(n, C, ty, tx, device=d)
    mean = torch.empty(n, C, device=d)
    std = torch.empty(n, C, device=d)
    bad = torch.empty(n, dtype=torch.int32, device=d)
    st = torch.cuda.current_stream().cuda_stream
    call("srmi_region_to_tiles", ptr(rg), C, H, W, ty, tx, ptr(tiles), ptr(mean), ptr(std), ptr(bad), st)
    ref_t, ref_m, ref_s, ids, grid = ro.region_to_tiles(region.astype(np.float64), ty, tx)
    assert list(ids) == list(range(n)) and int(bad.sum()) == 0
    np.testing.assert_allclose(mean.cpu().numpy(), ref_m, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(std.cpu().numpy(), ref_s, rtol=1e-5)
    np.testing.assert_allclose(tiles.cpu().numpy(), ref_t, atol=2e-5)
    out = torch.empty(C, grid[0] * ty, grid[1] * tx, device=d)
    call("srmi_tiles_to_region", ptr(tiles), ptr(mean), ptr(std), None, C, ty, tx, grid[0], grid[1], ptr(out), st)
    np.testing.assert_allclose(out.cpu().numpy(), region[:, :grid[0] * ty, :grid[1] * tx], rtol=1e-5, atol=1e-4)
    # a NaN marks its tile bad; an inverse map with -1 leaves that cell NaN
    region2 = region.copy()
    region2[1, ty + 3, 5] = np.nan
    call("srmi_region_to_tiles", ptr(torch.tensor(region2, device=d)), C, H, W, ty, tx, ptr(tiles), ptr(mean),
         ptr(std), ptr(bad), st)
    assert bad.cpu().tolist() == [0, 0, 1, 0, 0, 0]
    inv = torch.tensor([0, 1, -1, 2, 3, 4], dtype=torch.int32, device=d)
    call("srmi_tiles_to_region", ptr(tiles), None, None, ptr(inv), C, ty, tx, grid[0], grid[1], ptr(out), st)
    o = out.cpu().numpy()
    assert np.isnan(o[:, ty:2 * ty, 0:tx]).all() and np.isfinite(o[:, :ty]).all()


def _small_rcan():
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=1, nblocks=2, cbottleneck=2,
                   scale=4)
    model = ro.RCANOracle(nchannels_in=1, nchannels_out=1, nlayers=1, nblocks=2).double()
    ro.init_params_numpy(model, 11)
    table = param_table(spec)
    sd = dict(model.named_parameters())
    flat = torch.empty(sum(t[2] for t in table), dtype=torch.float32)
    for name, off, n, shape in table:
        flat[off:off + n] = sd[name].detach().float().reshape(-1)
    return spec, model, flat


@pytest.mark.parametrize("graph", [True, False])
def test_tiled_inference_matches_oracle(graph):
    d = dev()
    spec, model, flat = _small_rcan()
    rng = np.random.RandomState(7)
    # smooth-ish field so the bicubic baseline is meaningful; ragged edge cropped
    base = rng.randn(1, 2 * 192 + 17, 3 * 192 + 9)
    region = (base + np.roll(base, 1, 1) + np.roll(base, 1, 2)).astype(np.float32)
    ti = TiledInference(spec, flat.to(d), region.shape, (192, 192), device=d, graph=graph)
    images, losses = ti.process_region(torch.tensor(region, device=d))
    ref_img, ref_loss = ro.process_region(model, region.astype(np.float64), 192, 192, 4)
    for k in ("input", "target", "interpolated"):
        assert rel_l2(images[k].cpu().numpy(), ref_img[k]) < 1e-5, k
    assert rel_l2(images["model"].cpu().numpy(), ref_img["model"]) < 2e-2
    assert abs(float(losses["interpolated"]) - ref_loss["interpolated"]) < 1e-5 * ref_loss["interpolated"] + 1e-7
    assert abs(float(losses["model"]) - ref_loss["model"]) < 2e-3 * ref_loss["model"]
    # a second region through the same (captured) pipeline
    region2 = (region[:, ::-1, :].copy() * 0.5 + 2.0).astype(np.float32)
    images2, losses2 = ti.process_region(torch.tensor(region2, device=d))
    ref_img2, ref_loss2 = ro.process_region(model, region2.astype(np.float64), 192, 192, 4)
    assert rel_l2(images2["target"].cpu().numpy(), ref_img2["target"]) < 1e-5
    assert rel_l2(images2["model"].cpu().numpy(), ref_img2["model"]) < 2e-2


@pytest.mark.parametrize("graph,task,tile", [
    (True, {"data_downsample": 2}, 384),
    (False, {"data_downsample": 2}, 384),
    (True, {"data_downsample": 3, "downsample_mode": "linear", "upsample_mode": "linear"}, 576),
    (False, {"data_downsample": 1.5, "upsample_mode": "linear"}, 289),
])
def test_tiled_inference_data_downsample_vs_oracle(graph, task, tile):
    """apply_network's data_downsample in process_image (dual_trainer.py:423,
    :561-563) at even, odd and fractional factors, with task.downsample_mode /
    upsample_mode (array.py:37-41): the normalised tiles are downsampled by ds first,
    so target, model and interpolated -- and their mosaics -- are at 192² per tile."""
    from srmi.config import data_downsample_factor, interp_mode
    d = dev()
    spec, model, flat = _small_rcan()
    rng = np.random.RandomState(9)
    base = rng.randn(1, 2 * tile + 5, 2 * tile + 11)
    region = (base + np.roll(base, 1, 1) + np.roll(base, 1, 2)).astype(np.float32)
    ti = TiledInference(spec, flat.to(d), region.shape, (tile, tile), device=d, graph=graph, task=task)
    images, losses = ti.process_region(torch.tensor(region, device=d))
    ref_img, ref_loss = ro.process_region(model, region.astype(np.float64), tile, tile, 4,
                                          data_downsample=data_downsample_factor(task),
                                          dmode=interp_mode(task, True), umode=interp_mode(task, False))
    assert images["target"].shape[-1] == 2 * 192 and images["input"].shape[-1] == 2 * 48
    for k in ("input", "target", "interpolated"):
        assert rel_l2(images[k].cpu().numpy(), ref_img[k]) < 1e-5, k
    assert rel_l2(images["model"].cpu().numpy(), ref_img["model"]) < 2e-2
    assert abs(float(losses["interpolated"]) - ref_loss["interpolated"]) < 1e-5 * ref_loss["interpolated"] + 1e-7
    assert abs(float(losses["model"]) - ref_loss["model"]) < 2e-3 * ref_loss["model"]


def test_tiled_inference_drops_nonfinite_tiles():
    d = dev()
    spec, model, flat = _small_rcan()
    rng = np.random.RandomState(8)
    region = rng.randn(1, 2 * 192, 2 * 192).astype(np.float32)
    region[0, 200, 10] = np.nan  # tile (1, 0) -> id 2
    ti = TiledInference(spec, flat.to(d), region.shape, (192, 192), device=d, graph=True)
    images, losses = ti.process_region(torch.tensor(region, device=d))
    ref_img, ref_loss = ro.process_region(model, region.astype(np.float64), 192, 192, 4)
    m = images["model"].cpu().numpy()
    assert np.isnan(m[0, 192:, :192]).all() and np.isnan(ref_img["model"][0, 192:, :192]).all()
    keep = np.isfinite(ref_img["model"])
    assert rel_l2(m[keep], ref_img["model"][keep]) < 2e-2
    assert abs(float(losses["model"]) - ref_loss["model"]) < 2e-3 * ref_loss["model"]


@pytest.mark.parametrize("graph", [True, False])
def test_tiled_inference_micro_engines_bit_identical(graph):
    """The tile batch split over 2 (or 3, uneven) engines on their own streams gives
    bit-identical mosaics and losses to one engine: every output pixel and every
    CA pool partial is computed by the same arithmetic whatever the launch sizing."""
    d = dev()
    spec, model, flat = _small_rcan()
    rng = np.random.RandomState(9)
    region = rng.randn(1, 3 * 192, 3 * 192).astype(np.float32)
    region[0, 400, 500] = np.nan  # one dropped tile: the compacted path splits too
    res = {}
    for micro in (1, 2, 3):
        ti = TiledInference(spec, flat.to(d), region.shape, (192, 192), device=d, graph=graph, micro=micro)
        res[micro] = []
        for reg in (region, np.nan_to_num(region, nan=0.5)):
            images, losses = ti.process_region(torch.tensor(reg, device=d))
            torch.cuda.synchronize()
            res[micro].append(({k: v.clone() for k, v in images.items()}, float(losses["model"])))
    for micro in (2, 3):
        for (imgs, loss), (ref_imgs, ref_loss) in zip(res[micro], res[1]):
            for k in imgs:
                assert torch.equal(torch.nan_to_num(imgs[k], 7.0), torch.nan_to_num(ref_imgs[k], 7.0)), (micro, k)
            assert loss == ref_loss


@pytest.mark.parametrize("C,nl,nb,hw,N,cb", [(1, 2, 3, (48, 48), 5, 2), (2, 1, 2, (32, 48), 3, 2), (1, 1, 1, (8, 48), 2, 2),
                                           (2, 1, 3, (48, 48), 3, 8), (1, 2, 2, (32, 48), 2, 16)])
def test_fused_inference_rcab_matches_three_launches_and_oracle(C, nl, nb, hw, N, cb):
    """The inference RCAB as one launch with a workgroup per image (rcab_infer.hip:
    conv1 + sums of the bf16 t -> mean(u) from t's statistics with conv2's bf16 filter
    image and the CA MLP -> conv2 whose epilogue writes h + s u; u is never stored)
    against the three launches (SRMI_FLAG_NO_RCAB_INFER: conv1, conv2 + pool, CA pass)
    and the fp64 oracle forward.  The one launch differs from the three only in the
    summation order of mean(u) and in adding the fp32 u to h instead of bf16(u), so
    both sit within bf16 noise of the oracle and of each other.  cb: the CA bottleneck
    (CR = 64 / cb = 32, 8, 4)."""
    from srmi._lib import SRMI_FLAG_NO_RCAB_INFER
    from srmi.engine import Engine
    from srmi.trainer import default_init_
    d = dev()
    out = []
    for flags in (0, SRMI_FLAG_NO_RCAB_INFER):
        spec = NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=nl, nblocks=nb,
                       cbottleneck=cb, scale=4, flags=flags)
        table = param_table(spec)
        flat = torch.empty(sum(t[2] for t in table), device=d)
        default_init_(flat, table, seed=3)
        e = Engine(spec, N, hw, train=False, device=d)
        e.pack(flat)
        g = torch.Generator().manual_seed(11)
        lr = torch.randn(N, C, hw[0], hw[1], generator=g)
        out.append(e.forward(flat, lr.to(d)).clone().cpu().double())
    torch.cuda.synchronize()
    model = ro.RCANOracle(nchannels_in=C, nchannels_out=C, nlayers=nl, nblocks=nb, nfeatures=64,
                          cbottleneck=cb).double()
    sd = dict(model.named_parameters())
    fl = flat.cpu()
    with torch.no_grad():
        for name, off, n, shape in table:
            sd[name].copy_(fl[off:off + n].view(shape).double())
        ref = model(lr.double())
    e_one, e_three = rel_l2(out[0], ref), rel_l2(out[1], ref)
    assert e_one < 2e-2 and e_three < 2e-2, (e_one, e_three)
    assert e_one <= 1.5 * e_three + 1e-3, (e_one, e_three)
    assert rel_l2(out[0], out[1]) < 1e-2
    assert float(out[0].abs().sum()) > 0
