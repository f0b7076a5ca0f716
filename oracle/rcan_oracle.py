"""CPU oracle for the RCAN / EDSR tiled super-resolution hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline -- never as the thing measured or shipped.  The
product path (``srmi``) never imports it and fails loudly when its HIP library
is missing.

This is a plain PyTorch-CPU restatement (fp32 or fp64) of the reference's
algorithm, written independently and pinned against golden vectors generated
from the imported reference (``tests/golden/make_golden.py``):

* RCAN network ......... sres/model/rcan/network.py:7-77, blocks.py:58-76
* EDSR network ......... sres/model/edsr/network.py:9-32,
                         sres/model/common/residual.py:26-50, upsample.py:32-66
* parameter plumbing ... sres/model/common/common.py:9-48 (defaults, scale)
* default_conv ......... sres/model/common/cnn.py:8-9 (3x3, padding k//2)
* downsample/upsample .. sres/base/util/array.py:72-87 (bicubic, 'cubic')
* l2loss (RMSE) ........ sres/controller/stats.py:5-8
* train step ........... sres/controller/dual_trainer.py:310-323, :557-571
* Adam ................. torch.optim.Adam defaults used at dual_trainer.py:126
* batch preparation .... norm lnorm + xyflip (swot/raw.py:160-181,
                         sres/base/source/batch.py:33-49)
* on-disk LLC source ... load_file + mds2d + subset_roi + get_tiles
                         (swot/raw.py:133-145, :38-45, :216-233; swot/util.py:3-7)
* tiled inference ...... get_tiles + lnorm (sres/base/source/swot/raw.py:216-233,
                         :169-181), denorm + assemble_images + process_image
                         (dual_trainer.py:67-77, :482-512, :396-480); pinned by
                         restatement only (the reference wraps them in xarray,
                         which is not installed)

State-dict keys are identical to the reference model's.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# ---------------------------------------------------------------------------
# hyper-parameters (sres/model/common/common.py:9-20 defaults;
# config/model/rcan-10-20-64.yaml values)
# ---------------------------------------------------------------------------
COMMON_DEFAULTS = dict(nchannels_in=1, nchannels_out=1, nfeatures=64, kernel_size=3,
                       nlayers=16, downscale_factors=[2, 2], bias=True, batch_norm=False,
                       res_scale=1.0, ups_mode="bicubic")
RCAN_DEFAULTS = dict(cbottleneck=2, nblocks=20)


def _conv(cin: int, cout: int, k: int, bias: bool = True) -> nn.Conv2d:
    # sres/model/common/cnn.py:8-9
    return nn.Conv2d(cin, cout, k, padding=k // 2, bias=bias)


class _CA(nn.Module):
    """Channel attention: sres/model/rcan/network.py:31-47."""

    def __init__(self, nf: int, reduction: int):
        super().__init__()
        self.conv_du = nn.Sequential(nn.Conv2d(nf, nf // reduction, 1, padding=0, bias=True), nn.ReLU(),
                                     nn.Conv2d(nf // reduction, nf, 1, padding=0, bias=True), nn.Sigmoid())

    def forward(self, x):
        return x * self.conv_du(x.mean(dim=(2, 3), keepdim=True))


class _RCAB(nn.Module):
    """sres/model/rcan/network.py:50-64 (conv-ReLU-conv-CA + skip)."""

    def __init__(self, nf: int, k: int, reduction: int):
        super().__init__()
        self.body = nn.Sequential(_conv(nf, nf, k), nn.ReLU(), _conv(nf, nf, k), _CA(nf, reduction))

    def forward(self, x):
        return self.body(x) + x


class _RG(nn.Module):
    """sres/model/rcan/network.py:67-77 (nblocks RCAB + conv, skip)."""

    def __init__(self, nf: int, k: int, reduction: int, nblocks: int):
        super().__init__()
        self.body = nn.Sequential(*[_RCAB(nf, k, reduction) for _ in range(nblocks)], _conv(nf, nf, k))

    def forward(self, x):
        return self.body(x) + x


def _upsampler(scale: int, nf: int) -> nn.Sequential:
    """sres/model/rcan/blocks.py:58-76 and sres/model/common/upsample.py:32-66."""
    m: List[nn.Module] = []
    if scale & (scale - 1) == 0:
        for _ in range(int(math.log2(scale))):
            m += [_conv(nf, 4 * nf, 3), nn.PixelShuffle(2)]
    elif scale == 3:
        m += [_conv(nf, 9 * nf, 3), nn.PixelShuffle(3)]
    else:
        raise NotImplementedError(scale)
    return nn.Sequential(*m)


def resolve_parms(model: str, **kw) -> Dict:
    """init_parms (sres/model/common/common.py:22-28): defaults <- model yaml <- kwargs."""
    p = dict(COMMON_DEFAULTS)
    if model == "rcan":
        p.update(RCAN_DEFAULTS)
    p.update({k: v for k, v in kw.items() if v is not None})
    p["scale"] = int(math.prod(p["downscale_factors"]))
    return p


class RCANOracle(nn.Module):
    """RCAN (sres/model/rcan/network.py:7-27) with identical state-dict keys."""

    def __init__(self, **kw):
        super().__init__()
        p = resolve_parms("rcan", **kw)
        self.parms = p
        nf, k = p["nfeatures"], p["kernel_size"]
        self.head = nn.Sequential(_conv(p["nchannels_in"], nf, k))
        self.body = nn.Sequential(*[_RG(nf, k, p["cbottleneck"], p["nblocks"]) for _ in range(p["nlayers"])],
                                  _conv(nf, nf, k))
        self.tail = nn.Sequential(_upsampler(p["scale"], nf), _conv(nf, p["nchannels_out"], k))

    def forward(self, x):
        x = self.head(x)
        res = self.body(x) + x
        return self.tail(res)


class _ResBlock(nn.Module):
    """sres/model/common/residual.py:26-50."""

    def __init__(self, nf: int, k: int, res_scale: float):
        super().__init__()
        self.body = nn.Sequential(_conv(nf, nf, k), nn.ReLU(), _conv(nf, nf, k))
        self.res_scale = res_scale

    def forward(self, x):
        return self.body(x).mul(self.res_scale) + x


class EDSROracle(nn.Module):
    """EDSR (sres/model/edsr/network.py:9-32) with identical state-dict keys."""

    def __init__(self, **kw):
        super().__init__()
        p = resolve_parms("edsr", **kw)
        self.parms = p
        nf, k = p["nfeatures"], p["kernel_size"]
        self.head = nn.Sequential(_conv(p["nchannels_in"], nf, k))
        self.body = nn.Sequential(*[_ResBlock(nf, k, p["res_scale"]) for _ in range(p["nlayers"])],
                                  _conv(nf, nf, k))
        self.tail = nn.Sequential(_upsampler(p["scale"], nf), _conv(nf, p["nchannels_out"], k))

    def forward(self, x):
        x = self.head(x)
        res = self.body(x) + x
        return self.tail(res)


def build(model: str, **kw) -> nn.Module:
    return {"rcan": RCANOracle, "edsr": EDSROracle}[model](**kw)


# ---------------------------------------------------------------------------
# deterministic parameter init: the distribution of PyTorch's default Conv2d
# init (kaiming_uniform a=sqrt(5) -> U(-1/sqrt(fan_in), 1/sqrt(fan_in)); bias
# the same bound), drawn from numpy RandomState so it is stream-stable.
# ---------------------------------------------------------------------------
def init_params_numpy(model: nn.Module, seed: int) -> None:
    rs = np.random.RandomState(seed)
    with torch.no_grad():
        for name, mod in model.named_modules():
            if isinstance(mod, nn.Conv2d):
                fan_in = mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
                bound = 1.0 / math.sqrt(fan_in)
                w = rs.uniform(-bound, bound, size=tuple(mod.weight.shape))
                mod.weight.copy_(torch.from_numpy(w))
                if mod.bias is not None:
                    b = rs.uniform(-bound, bound, size=tuple(mod.bias.shape))
                    mod.bias.copy_(torch.from_numpy(b))


# ---------------------------------------------------------------------------
# data path pieces on the hot path
# ---------------------------------------------------------------------------
def downsample(hr: torch.Tensor, scale, mode: str = "bicubic") -> torch.Tensor:
    """array.py:72-76: F.interpolate(scale_factor=1/scale, mode=torch_interp_mode(True))
    (array.py:37-41: task.downsample_mode 'cubic' -> 'bicubic', 'linear' -> 'bilinear')."""
    return F.interpolate(hr, scale_factor=1.0 / scale, mode=mode)


def downsample_explicit(hr: np.ndarray, scale: int) -> np.ndarray:
    """Closed form of the bicubic (A=-0.75, align_corners=False) 1/scale
    resampling: src = scale*d + (scale-1)/2 is exactly half-way between two
    samples, so each output is the separable 4-tap [-3,19,19,-3]/32 filter over
    rows/cols scale*d + scale/2 - 2 .. +1 (never clamped for scale >= 4)."""
    w = np.array([-3.0, 19.0, 19.0, -3.0]) / 32.0
    B, C, H, W = hr.shape
    h, wd = H // scale, W // scale
    o = scale // 2 - 2
    ys = np.arange(h)[:, None] * scale + o + np.arange(4)[None, :]
    xs = np.arange(wd)[:, None] * scale + o + np.arange(4)[None, :]
    rows = np.einsum("bchkx,k->bchx", hr[:, :, ys, :], w)          # [B,C,h,W]
    return np.einsum("bchwk,k->bchw", rows[:, :, :, xs], w)         # [B,C,h,w]


def upsample(lr: torch.Tensor, scale: int, mode: str = "bicubic") -> torch.Tensor:
    """array.py:84-87: interp baseline, xscale with torch_interp_mode(False)
    (task.upsample_mode)."""
    return F.interpolate(lr, scale_factor=scale, mode=mode)


def l2loss(prd: torch.Tensor, tar: torch.Tensor, squared: bool = False) -> torch.Tensor:
    """stats.py:5-8 -- RMSE unless squared."""
    loss = ((prd - tar) ** 2).mean()
    return loss if squared else torch.sqrt(loss)


def lnorm(x: np.ndarray) -> np.ndarray:
    """Per-tile, per-channel normalisation to mean 0 / std 1 (ddof 0), the
    statistics of the reference's 'lnorm' tiles (sres/base/source/swot/raw.py:177-181)."""
    m = x.mean(axis=(2, 3), keepdims=True)
    s = x.std(axis=(2, 3), keepdims=True)
    return (x - m) / s


def synthetic_hr(batch: int, nchan: int, size: int, seed: int = 1234) -> np.ndarray:
    """HR tiles ~ N(0,1) from RandomState(seed), lnorm-normalised."""
    rs = np.random.RandomState(seed)
    return lnorm(rs.standard_normal((batch, nchan, size, size))).astype(np.float32)


# ---------------------------------------------------------------------------
# Adam (torch.optim.Adam defaults: betas (0.9,0.999), eps 1e-8, no amsgrad)
# ---------------------------------------------------------------------------
class AdamOracle:
    def __init__(self, params: Sequence[torch.Tensor], lr: float, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay: float = 0.0):
        self.params = list(params)
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        for p, m, v in zip(self.params, self.m, self.v):
            g = p.grad
            if g is None:
                continue
            if self.wd != 0:
                g = g + self.wd * p
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            p.addcdiv_(m, denom, value=-self.lr / bc1)

    def zero_grad(self):
        for p in self.params:
            p.grad = None


def train_step(model: nn.Module, opt: AdamOracle, hr: torch.Tensor, scale: int,
               interp_loss: bool = False, dmode: str = "bicubic",
               umode: str = "bicubic") -> Tuple[float, Optional[float], torch.Tensor]:
    """One step of dual_trainer.py:310-323 with apply_network (:557-571):
    HR (requires_grad, as array2tensor does) -> downsample -> model -> RMSE ->
    backward -> Adam.  Returns (loss, interp_loss, output).  dmode / umode: the
    F.interpolate modes of task.downsample_mode / upsample_mode."""
    opt.zero_grad()
    hr = hr.detach().clone().requires_grad_(True)          # array2tensor, array.py:70
    lr_in = downsample(hr, scale, dmode)
    out = model(lr_in)
    loss = l2loss(out, hr)
    iloss = None
    if interp_loss:
        with torch.no_grad():
            iloss = float(l2loss(hr, upsample(lr_in, scale, umode)))
    loss.backward()
    opt.step()
    return float(loss), iloss, out.detach()


# --------------------------------------------------------------------------
# Tiled-region inference data path.  The reference's own
# functions wrap numpy in xarray (not installed here), so these restate them:
# parity for this row is pinned by restatement, not by golden vectors.

def region_to_tiles(region: np.ndarray, ty: int, tx: int):
    """get_tiles (sres/base/source/swot/raw.py:216-233) for C == 1 plus the 'lnorm'
    branch of norm() (raw.py:169-181).  region [C, H, W] -> (tiles [n, C, ty, tx]
    normalised, mean [n, C], std [n, C], tile_ids [n]); tiles whose mean is not
    finite are dropped, as the reference's mask does."""
    C, H, W = region.shape
    gy, gx = H // ty, W // tx
    reg = region[:, :gy * ty, :gx * tx]
    t = reg.reshape(C, gy, ty, gx, tx).swapaxes(2, 3).reshape(C, gy * gx, ty, tx).swapaxes(0, 1)
    keep = np.isfinite(t.mean(axis=(1, 2, 3)))
    ids = np.nonzero(keep)[0]
    t = t[keep]
    mean = t.mean(axis=(2, 3))
    std = t.std(axis=(2, 3))  # xarray .std(): ddof 0
    tiles = (t - mean[:, :, None, None]) / std[:, :, None, None]
    return tiles, mean, std, ids, (gy, gx)


def assemble(tiles: np.ndarray, mean: Optional[np.ndarray], std: Optional[np.ndarray], ids: np.ndarray,
             grid: Tuple[int, int]) -> np.ndarray:
    """denorm (dual_trainer.py:67-77) + assemble_images (dual_trainer.py:482-512):
    tile id -> cell (id // gx, id % gx), missing cells NaN.  -> [C, gy*ty, gx*tx]"""
    n, C, ty, tx = tiles.shape
    gy, gx = grid
    x = tiles if mean is None else tiles * std[:, :, None, None] + mean[:, :, None, None]
    out = np.full((C, gy * ty, gx * tx), np.nan, dtype=x.dtype)
    for i, tid in enumerate(ids):
        y0, x0 = (tid // gx) * ty, (tid % gx) * tx
        out[:, y0:y0 + ty, x0:x0 + tx] = x[i]
    return out


def charbonnier(prd: torch.Tensor, tar: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    """ModelTrainer.charbonnier (dual_trainer.py:196-198), eps = self.eps (:122)."""
    return torch.mean(torch.sqrt((prd - tar) ** 2 + eps))


def single_product_loss(prd: torch.Tensor, tar: torch.Tensor, loss_fn: str = "l2") -> torch.Tensor:
    """dual_trainer.py:205-212."""
    if loss_fn == "l2":
        return l2loss(prd, tar)
    if loss_fn == "charbonnier":
        return charbonnier(prd, tar)
    raise Exception("Unknown single-product loss function {}".format(loss_fn))


def batch_losses(prd: torch.Tensor, tar: torch.Tensor, batch_size: int, loss_fn: str = "l2") -> List[float]:
    """The per-batch losses of process_image / evaluate (dual_trainer.py:417-430):
    TileBatchIterator batches [0, bs), [bs, 2bs), ... (the last one short)."""
    return [float(single_product_loss(prd[a:a + batch_size], tar[a:a + batch_size], loss_fn))
            for a in range(0, prd.shape[0], batch_size)]


def process_region(model, region: np.ndarray, ty: int, tx: int, scale: int, batch_size: Optional[int] = None,
                   loss_fn: str = "l2", data_downsample=1, dmode: str = "bicubic", umode: str = "bicubic"):
    """process_image (dual_trainer.py:396-480) on one region: tiles scored in batches
    of batch_size (None: one batch of all tiles); loss = mean of the batch losses
    (:443-446).  Returns (images dict, losses dict) with the reference's image types.
    data_downsample > 1: apply_network first downsamples the (normalised) tiles by it
    (:561-563), so target, model and interpolated are at 1/ds of the tile size.
    dmode / umode: the F.interpolate modes of task.downsample_mode / upsample_mode."""
    tiles, mean, std, ids, grid = region_to_tiles(region, ty, tx)
    dt = torch.float64 if tiles.dtype == np.float64 else torch.float32
    target = torch.tensor(tiles, dtype=dt)
    if data_downsample > 1:
        target = downsample(target, data_downsample, dmode)
        tiles = target.numpy()
    lr = downsample(target, scale, dmode)
    with torch.no_grad():
        sr = model(lr)
    interp = upsample(lr, scale, umode)
    bs = batch_size or target.shape[0]
    bm = batch_losses(sr, target, bs, loss_fn)
    bi = batch_losses(interp, target, bs, loss_fn)
    losses = {"model": float(np.array(bm).mean()), "interpolated": float(np.array(bi).mean()),
              "batch_model": bm, "batch_interpolated": bi}
    images = {"input": assemble(lr.numpy(), mean, std, ids, grid), "target": assemble(tiles, mean, std, ids, grid),
              "interpolated": assemble(interp.numpy(), mean, std, ids, grid),
              "model": assemble(sr.numpy(), mean, std, ids, grid)}
    return images, losses


def evaluate(model, regions: Sequence[np.ndarray], ty: int, tx: int, scale: int, batch_size: int,
             loss_fn: str = "l2", time_index: int = -1, tile_index: int = -1, batch_domain: str = "tiles"):
    """ModelTrainer.evaluate (dual_trainer.py:482-543) over the time slices of a
    tset (no flips): losses = mean over all scored batches of all scored regions
    (:532, :541); results = the normalised tiles of the LAST scored region only:
    clear_results at the start of every time slice (:505, :545-549), then that
    slice's scored batches concatenated along the tile axis (merge_results_tiles,
    :38-42, :551-555).  time_index >= 0: only slice itime == time_index, then stop
    (:508-509, :527); tile_index >= 0: only the batch tile_in_batch accepts
    (:366-372: 'tiles' -- its range [start, end) holds tile_index; 'time' -- its
    ordinal equals it), then the next slice (:525)."""
    bm, bi, results = [], [], {}
    for itime, region in enumerate(regions):
        if not (time_index < 0 or itime == time_index):
            continue
        results = {}  # clear_results
        tiles, _, _, _, _ = region_to_tiles(region, ty, tx)
        dt = torch.float64 if tiles.dtype == np.float64 else torch.float32
        target = torch.tensor(tiles, dtype=dt)
        for ib, a in enumerate(range(0, target.shape[0], batch_size)):
            end = min(a + batch_size, target.shape[0])
            if tile_index >= 0:
                ok = (a <= tile_index < end) if batch_domain == "tiles" else (ib == tile_index)
                if not ok:
                    continue
            tb = target[a:end]
            lr = downsample(tb, scale)
            with torch.no_grad():
                sr = model(lr)
            interp = upsample(lr, scale)
            bm.append(float(single_product_loss(sr, tb, loss_fn)))
            bi.append(float(single_product_loss(interp, tb, loss_fn)))
            for k, v in (("input", lr), ("target", tb), ("model", sr), ("interpolated", interp)):
                results[k] = v.numpy() if k not in results else np.concatenate([results[k], v.numpy()])
            if tile_index >= 0:
                break
        if time_index >= 0:
            break
    return results, {"model": float(np.array(bm).mean()), "interpolated": float(np.array(bi).mean())}


# --------------------------------------------------------------------------
# Training batch preparation: 'lnorm' of select_batch ->
# norm (sres/base/source/swot/raw.py:160-181), then xyflip
# (sres/base/source/batch.py:33-49, applied by load_batch :301), then the
# apply_network input downsample (array.py:72-76).  xyflip is pinned by golden
# vectors from the imported reference (tests/golden/make_golden_batch.py);
# lnorm by restatement (xarray's mean/std over (x, y): skipna, ddof 0).

def xyflip(x: np.ndarray, flip_index: int) -> np.ndarray:
    """batch.py:37-49 for a given flip_index (the reference draws it with
    random.randint(0, 7) when task.xyflip is set, else 0): bit 0 flips x
    (axis -1), bit 1 flips y (axis -2), bit 2 swaps the two axes
    (flip_xarray_axis, batch.py:33-35), in that order."""
    if flip_index % 2 == 1:
        x = np.flip(x, axis=-1)
    if (flip_index // 2) % 2 == 1:
        x = np.flip(x, axis=-2)
    if flip_index // 4 == 1:
        x = np.swapaxes(x, -1, -2)
    return np.ascontiguousarray(x)


def prep_batch(raw: np.ndarray, flip_index: int, scale: int):
    """raw tiles [B, C, T, T] -> (hr = xyflip(lnorm(raw)), lr = downsample(hr),
    mean [B, C], std [B, C]) -- the tensors the reference's train loop hands to
    apply_network (dual_trainer.py:557-571), plus norm()'s ncstats attrs."""
    mean = raw.mean(axis=(2, 3))
    std = raw.std(axis=(2, 3))
    hr = xyflip((raw - mean[:, :, None, None]) / std[:, :, None, None], flip_index)
    return hr, downsample_explicit(hr, scale), mean, std


# --------------------------------------------------------------------------
# On-disk source -> tiles, pinned by digests of the
# reference's own load_file / get_tiles outputs (tests/golden/make_golden_llc.py).

def mds2d(d: np.ndarray, nx: int = 4320):
    """util.py:3-7 rearrange (mds2d with one array): LLC faces 1-6 -> east
    [3nx, 2nx], faces 8-13 -> west [2nx, 3nx] (face 7, the Arctic, unused)."""
    east = np.concatenate([d[:nx * nx * 3].reshape(3 * nx, nx), d[nx * nx * 3:nx * nx * 6].reshape(3 * nx, nx)], axis=1)
    west = d[nx * nx * 7:].reshape(nx * 2, nx * 3)
    return east, west


def llc_load_file(template: np.ndarray, wet_values: np.ndarray, roi: Optional[Dict] = None,
                  nx: int = 4320) -> np.ndarray:
    """SWOTRawDataLoader.load_file (sres/base/source/swot/raw.py:133-145) on
    already-decoded arrays: wet cells (template != 0) take the file's values in
    order, land is NaN; east | west.T[::-1] assembled to [1, 3nx, 4nx]; then
    subset_roi (raw.py:38-45)."""
    full = template.astype(np.float32).copy()
    mask = full != 0
    if int(mask.sum()) != len(wet_values):
        raise ValueError(f"{len(wet_values)} values for {int(mask.sum())} wet cells")
    full[mask] = wet_values
    full[~mask] = np.nan
    east, west = mds2d(full, nx)
    res = np.concatenate([east, west.T[::-1, :]], axis=1)[None]
    if roi:
        x0, xs = roi.get("x0", 0), roi.get("xs", res.shape[-1])
        y0, ys = roi.get("y0", 0), roi.get("ys", res.shape[-2])
        res = res[..., y0:y0 + ys, x0:x0 + xs]
    return res


def get_tiles(var_data: Sequence[np.ndarray], ty: int, tx: int):
    """SWOTRawDataLoader.get_tiles (raw.py:216-233) with the default TileGrid
    (origin 0, tile_grid -1 -> floor grid, sres/data/tiles.py:112-135): tiles
    flattened channel-major, tiles whose mean is not finite dropped, the rest
    reshaped to [n // C, C, ty, tx] -- with C > 1 this packs consecutive kept
    tiles of the SAME variable into the channel axis (the reference's quirk,
    reproduced).  -> (tiles, tile_ids (first n // C kept flat ids), (gy, gx))."""
    raw = np.concatenate(var_data, axis=0)
    C, H, W = raw.shape
    gy, gx = H // ty, W // tx
    region = raw[..., :gy * ty, :gx * tx]
    t = region.reshape(C, gy, ty, gx, tx).swapaxes(2, 3).reshape(C * gy * gx, ty, tx)
    msk = np.isfinite(t.mean(axis=-1).mean(axis=-1))
    kept = t[msk]
    ids = np.flatnonzero(msk)
    res = kept.reshape(kept.shape[0] // C, C, ty, tx)
    return res, ids[:res.shape[0]], (gy, gx)
