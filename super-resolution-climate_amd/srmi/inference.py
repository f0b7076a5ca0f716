"""Tiled-region inference: drop-in for ModelTrainer.process_image + assemble_images
and ModelTrainer.evaluate.

Reference (sres/controller/dual_trainer.py:396-543, sres/base/source/swot/raw.py:169-233):
a region [C, H, W] is cut floor-wise into a gy x gx grid of HR tiles (tile id =
y * gx + x), tiles holding a non-finite value are dropped, every tile/channel is
'lnorm'-normalised (mean/std over the tile, ddof 0), the LR input is the bicubic
1/s of the tile (apply_network, :557-571), the model output and the bicubic
interpolation baseline (upsample) are scored against the tile in batches of
task.batch_size tiles (TileBatchIterator, sres/data/tiles.py:48-74) with
model.loss_fn ('l2' = RMSE, 'charbonnier'), the reported loss being the mean of
the batch losses (:443-446), and each image type (input, target, interpolated,
model) is de-normalised and mosaicked back into the grid (NaN where a tile was
dropped).

Every step runs in srmi's HIP kernels (region_to_tiles, downsample, the RCAN/EDSR
inference engine, upsample, RMSE, tiles_to_region) on one stream; the whole
per-region sequence is captured once in a HIP graph (torch.cuda.CUDAGraph drives
hipGraph capture of the ctypes launches on the capture stream) and replayed per
region, so a region costs one graph launch.

Difference from the reference, by design: for C > 1 channel c of tile t is region
channel c at tile t (the reference's channel-major flattening packs neighbouring
tiles of one variable into the channel axis, SURVEY.md §8f row 3 -- identical for
the 1-variable C5 case).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ._lib import SRMI_LOSS_MEAN, SRMI_LOSS_RMSE, call, ptr, stream_handle
from .engine import Engine, NetSpec, downsample, upsample

LOSS_KINDS = {"l2": SRMI_LOSS_RMSE, "charbonnier": SRMI_LOSS_MEAN}
CHARBONNIER_EPS = 1e-6  # dual_trainer.py:122


class TiledInference:
    def __init__(self, spec: NetSpec, params: torch.Tensor, region_chw: Tuple[int, int, int],
                 tile_hr: Tuple[int, int] = (192, 192), device: Optional[torch.device] = None, graph: bool = True,
                 micro: Optional[int] = None, batch_size: int = 36, loss_fn: str = "l2"):
        """batch_size: task.batch_size (the tiles scored per batch; 36 in every
        reference task yaml); loss_fn: model.loss_fn."""
        if loss_fn not in LOSS_KINDS:
            raise ValueError(f"Unknown single-product loss function {loss_fn}")
        self.loss_kind = LOSS_KINDS[loss_fn]
        self.batch_size = int(batch_size)
        self.spec = spec
        self.device = device or params.device
        C, H, W = region_chw
        if C != spec.nchannels_in or spec.nchannels_in != spec.nchannels_out:
            raise ValueError("region channels must equal the model's input/output channels")
        ty, tx = tile_hr
        s = spec.scale
        if ty % s or tx % s:
            raise ValueError(f"tile {tile_hr} not divisible by the model scale {s}")
        self.C, self.H, self.W, self.ty, self.tx, self.s = C, H, W, ty, tx, s
        self.gy, self.gx = H // ty, W // tx
        n = self.gy * self.gx
        if n < 1:
            raise ValueError("region smaller than one tile")
        self.n = n
        self.params = params
        d = self.device
        f32 = dict(dtype=torch.float32, device=d)
        self.region = torch.empty((C, H, W), **f32)
        self.tiles = torch.empty((n, C, ty, tx), **f32)
        self.mean = torch.empty((n, C), **f32)
        self.std = torch.empty((n, C), **f32)
        self.bad = torch.zeros(n, dtype=torch.int32, device=d)
        self.lr = torch.empty((n, C, ty // s, tx // s), **f32)
        self.sr = torch.empty((n, C, ty, tx), **f32)
        self.interp = torch.empty((n, C, ty, tx), **f32)
        nb = (n + self.batch_size - 1) // self.batch_size
        self.loss_m = torch.zeros(1 + nb, **f32)   # [mean of batch losses, batch losses...]
        self.loss_i = torch.zeros(1 + nb, **f32)
        self.loss_work = torch.zeros(n, **f32)
        self.n_kept = n
        hr_shape = (C, self.gy * ty, self.gx * tx)
        self.images = {
            "input": torch.empty((C, self.gy * ty // s, self.gx * tx // s), **f32),
            "target": torch.empty(hr_shape, **f32),
            "interpolated": torch.empty(hr_shape, **f32),
            "model": torch.empty(hr_shape, **f32),
        }
        # the tile batch is split over `micro` engines on their own streams, each
        # sized for 1/micro of the chip (as srmi.trainer.FusedTrainer does): each
        # engine's launch ramps and tails overlap the other's work
        if micro is None:
            micro = 2 if n >= 32 else 1
        self.micro = max(1, min(int(micro), n))
        per = (n + self.micro - 1) // self.micro
        self.split = [min(per, n - k * per) for k in range(self.micro)]
        budget = 256 // self.micro if self.micro > 1 else 0
        self.engs = [Engine(spec, m, (ty // s, tx // s), train=False, device=d, cu_budget=budget)
                     for m in self.split]
        self.eng = self.engs[0]
        for e in self.engs:
            e.pack(params)
        self.streams = [None] + [torch.cuda.Stream(device=d) for _ in range(self.micro - 1)]
        # fork / join events, created once (also valid inside a graph capture)
        self.ev_fork = torch.cuda.Event()
        self.ev_join = [torch.cuda.Event() for _ in range(self.micro - 1)]
        self._graph = None
        self._use_graph = graph and self.device.type == "cuda"

    # ---------------------------------------------------------------- pieces
    def _tile(self):
        st = stream_handle()
        call("srmi_region_to_tiles", ptr(self.region), self.C, self.H, self.W, self.ty, self.tx, ptr(self.tiles),
             ptr(self.mean), ptr(self.std), ptr(self.bad), st)

    def _model_and_mosaic(self, tiles, lr, sr, interp, mean, std, inv, nt):
        st = stream_handle()
        downsample(tiles, self.s, out=lr)
        main = torch.cuda.current_stream(self.device)
        self.ev_fork.record(main)
        for sk in self.streams[1:]:
            sk.wait_event(self.ev_fork)
        a = 0
        for k, e in enumerate(self.engs):
            b = min(nt, a + self.split[k])
            if b > a:
                if self.streams[k] is None:
                    e.forward(self.params, lr[a:b], out=sr[a:b])
                else:
                    with torch.cuda.stream(self.streams[k]):
                        e.forward(self.params, lr[a:b], out=sr[a:b])
            a = b
        for sk, ev in zip(self.streams[1:], self.ev_join):
            ev.record(sk)
            main.wait_event(ev)
        upsample(lr, self.s, out=interp)
        te = self.C * self.ty * self.tx
        for pred, lo in ((sr, self.loss_m), (interp, self.loss_i)):
            call("srmi_batch_losses", ptr(pred), ptr(tiles), nt, te, self.batch_size, self.loss_kind,
                 CHARBONNIER_EPS, ptr(self.loss_work), ptr(lo), st)
        C, gy, gx, s = self.C, self.gy, self.gx, self.s
        for name, src, ty, tx in (("input", lr, self.ty // s, self.tx // s), ("target", tiles, self.ty, self.tx),
                                  ("interpolated", interp, self.ty, self.tx), ("model", sr, self.ty, self.tx)):
            call("srmi_tiles_to_region", ptr(src), ptr(mean), ptr(std), ptr(inv), C, ty, tx, gy, gx,
                 ptr(self.images[name]), st)

    def _all_tiles(self):
        self._kept_tiles = self.tiles
        self._model_and_mosaic(self.tiles, self.lr, self.sr, self.interp, self.mean, self.std, None, self.n)

    # ------------------------------------------------------------------- API
    def process_region(self, region: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], Dict[str, torch.Tensor]]:
        """process_image (dual_trainer.py:396-447) on one region.  region [C, H, W]
        fp32 (device) -> (images, losses); images are device tensors (input
        [C, gy*ty/s, gx*tx/s], target/interpolated/model [C, gy*ty, gx*tx]), losses
        {'model', 'interpolated'} 1-element device tensors = the mean of the batch
        losses; batch_losses() gives the per-batch values."""
        if tuple(region.shape) != (self.C, self.H, self.W):
            raise ValueError(f"region shape {tuple(region.shape)} != {(self.C, self.H, self.W)}")
        self.region.copy_(region)
        self._tile()
        self.n_kept = self.n
        # every path below scores self.tiles except the compacted one, which resets
        # this to its compacted copy (a graph replay after a compacted region must
        # not leave the previous region's tiles here)
        self._kept_tiles = self.tiles
        if bool(self.bad.any()):  # rare: drop non-finite tiles (reference get_tiles mask)
            self._run_compacted()
        elif self._use_graph:
            if self._graph is None:
                self._capture()
            self._graph.replay()
        else:
            self._all_tiles()
        return self.images, {"model": self.loss_m[0:1], "interpolated": self.loss_i[0:1]}

    def batch_losses(self) -> Dict[str, torch.Tensor]:
        """The per-batch losses of the last region (batch_model_losses /
        batch_interp_losses of process_image, dual_trainer.py:428-430)."""
        nb = (self.n_kept + self.batch_size - 1) // self.batch_size
        return {"model": self.loss_m[1:1 + nb], "interpolated": self.loss_i[1:1 + nb]}

    def set_params(self, params: torch.Tensor) -> None:
        """Load new weights (e.g. the validation checkpoint, dual_trainer.py:402/491):
        copied into the parameter buffer the engines (and the captured graph) read,
        filter packs rebuilt."""
        self.params.copy_(params)
        for e in self.engs:
            e.pack(self.params)

    def evaluate(self, regions: Sequence[torch.Tensor]) -> Tuple[Dict[str, torch.Tensor], Dict[str, float]]:
        """ModelTrainer.evaluate (dual_trainer.py:482-543) over the time slices of a
        tset: every region is tiled, normalised and scored batch by batch; the loss
        is the mean over ALL batches of all regions (:532, :541), while the results
        are those of the LAST evaluated region only -- the reference clears them at
        the start of every time slice (clear_results, :505, :545-549) and then
        concatenates that slice's batches (merge_results / merge_results_tiles,
        :551-555, :38-42): input [n, C, ty/s, tx/s], target / model / interpolated
        [n, C, ty, tx] (device tensors, normalised tiles).  The
        validation-checkpoint policy applied to the returned loss is
        ValidationCheckpoint.update (srmi.harness)."""
        bm: List[torch.Tensor] = []
        bi: List[torch.Tensor] = []
        results: Dict[str, torch.Tensor] = {k: torch.empty(0, device=self.device)
                                            for k in ("input", "target", "model", "interpolated")}
        for region in regions:
            self.process_region(region)
            nt = self.n_kept
            b = self.batch_losses()
            bm.append(b["model"].clone())
            bi.append(b["interpolated"].clone())
            # clear_results(tset) per time slice, then this slice's tiles
            results = {"input": self.lr[:nt].clone(), "target": self._kept_tiles[:nt].clone(),
                       "model": self.sr[:nt].clone(), "interpolated": self.interp[:nt].clone()}
        m = torch.cat(bm).double().cpu() if bm else torch.empty(0, dtype=torch.float64)
        i = torch.cat(bi).double().cpu() if bi else torch.empty(0, dtype=torch.float64)
        losses = {"model": float(m.mean()) if m.numel() else float("nan"),
                  "interpolated": float(i.mean()) if i.numel() else float("nan")}
        return results, losses

    def replay(self):
        """Re-run the captured per-region graph on the current region buffer (bench)."""
        if self._graph is None:
            self._capture()
        self._graph.replay()

    def _capture(self):
        self._all_tiles()  # warm-up outside capture (uploads engine tables)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._tile()
                self._all_tiles()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._graph = g

    def _run_compacted(self):
        keep = torch.nonzero(self.bad == 0).flatten()
        nt = int(keep.numel())
        self.n_kept = nt
        inv = torch.full((self.n,), -1, dtype=torch.int32, device=self.device)
        if nt == 0:
            for img in self.images.values():
                img.fill_(float("nan"))
            self.loss_m.fill_(float("nan"))
            self.loss_i.fill_(float("nan"))
            return
        inv[keep] = torch.arange(nt, dtype=torch.int32, device=self.device)
        tiles = self.tiles.index_select(0, keep).contiguous()
        self._kept_tiles = tiles
        mean = self.mean.index_select(0, keep).contiguous()
        std = self.std.index_select(0, keep).contiguous()
        self._model_and_mosaic(tiles, self.lr[:nt], self.sr[:nt], self.interp[:nt], mean, std, inv, nt)
