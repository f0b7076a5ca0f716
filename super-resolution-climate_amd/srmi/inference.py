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
from .dist import DistInfo
from .engine import Engine, NetSpec, downsample, engine_stream, interp_size, upsample

LOSS_KINDS = {"l2": SRMI_LOSS_RMSE, "charbonnier": SRMI_LOSS_MEAN}
CHARBONNIER_EPS = 1e-6  # dual_trainer.py:122


def gather_round_robin(x: torch.Tensor, n: int, world: int) -> torch.Tensor:
    """All-gather of this rank's rows of a round-robin split into grid order: rank r
    holds rows for grid tiles r, r + W, r + 2W, ... (x [n_r, ...]); every rank gets
    the [n, ...] tensor with tile i at row i.  Ranks pad to a common slot of
    ceil(n / W) rows; RCCL gathers device tensors directly, gloo (the CPU and
    one-GPU tests) through host memory."""
    import torch.distributed as dist
    npd = (n + world - 1) // world
    slot = torch.zeros((npd,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    slot[:x.shape[0]] = x
    if dist.get_backend() == "nccl":
        out = torch.empty((world * npd,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, slot)
    else:
        parts = [torch.empty_like(slot, device="cpu") for _ in range(world)]
        dist.all_gather(parts, slot.cpu())
        out = torch.cat(parts).to(x.device)
    order = torch.arange(n, device=x.device)  # tile i = rank i % W, row i // W
    return out.index_select(0, (order % world) * npd + order // world)


class TiledInference:
    def __init__(self, spec: NetSpec, params: torch.Tensor, region_chw: Tuple[int, int, int],
                 tile_hr: Tuple[int, int] = (192, 192), device: Optional[torch.device] = None, graph: bool = True,
                 micro: Optional[int] = None, batch_size: int = 36, loss_fn: str = "l2",
                 info: Optional[DistInfo] = None, task=None):
        """batch_size: task.batch_size (the tiles scored per batch; 36 in every
        reference task yaml); loss_fn: model.loss_fn.

        info (world > 1): multi-rank inference: the region's tile
        grid is dealt round-robin over the ranks (rank r runs grid tiles r, r + W,
        ...), each rank forms its tiles' per-tile loss sums, and the tiles and sums
        are all-gathered, so every rank -- rank 0 being the one that writes results --
        holds the full mosaics and the per-batch losses, bit-identical to one rank:
        the forward is batch-invariant (every tile is computed alone, whatever engine
        batch it rides in) and the batch losses are formed from the gathered per-tile
        sums in the one-rank order (srmi_batch_loss_means).  No graph in this mode."""
        if loss_fn not in LOSS_KINDS:
            raise ValueError(f"Unknown single-product loss function {loss_fn}")
        if task is None:  # the active srmi ConfigContext's task section, if any
            from . import config as _config
            task = _config._CURRENT.get("task") if _config._CURRENT is not None else None
        from .config import data_downsample_factor, interp_mode
        # apply_network's pre-downsampling (:561-563): the normalised tiles are scored
        # at 1/ds of the tile size (target, model, interpolated and their mosaics)
        self.ds = data_downsample_factor(task)
        # task.downsample_mode / upsample_mode (torch_interp_mode, array.py:37-41)
        self.dmode, self.umode = interp_mode(task, True), interp_mode(task, False)
        self.loss_kind = LOSS_KINDS[loss_fn]
        self.batch_size = int(batch_size)
        self.spec = spec
        self.device = device or params.device
        C, H, W = region_chw
        if C != spec.nchannels_in or spec.nchannels_in != spec.nchannels_out:
            raise ValueError("region channels must equal the model's input/output channels")
        ty0, tx0 = tile_hr
        s = spec.scale
        # the scored tile: floor(tile / ds) (F.interpolate's size; the region's tile at ds = 1)
        ty, tx = (interp_size(ty0, 1.0 / self.ds), interp_size(tx0, 1.0 / self.ds)) if self.ds > 1 else (ty0, tx0)
        if ty % s or tx % s or ty < s or tx < s:
            raise ValueError(f"tile {tile_hr} / data_downsample {self.ds} = {(ty, tx)} not divisible by the model "
                             f"scale {s}")
        self.C, self.H, self.W, self.ty, self.tx, self.s = C, H, W, ty, tx, s
        self.ty0, self.tx0 = ty0, tx0
        self.gy, self.gx = H // ty0, W // tx0
        n = self.gy * self.gx
        if n < 1:
            raise ValueError("region smaller than one tile")
        self.n = n
        self.info = info or DistInfo()
        # this rank's grid tiles (all of them at one rank)
        W_, r_ = (self.info.world, self.info.rank) if self.info.enabled else (1, 0)
        self.rr_world = W_
        self.n_local = len(range(r_, n, W_))
        self.n_pad = (n + W_ - 1) // W_  # per-rank gather slot
        self.params = params
        d = self.device
        f32 = dict(dtype=torch.float32, device=d)
        self.region = torch.empty((C, H, W), **f32)
        self.tiles = torch.empty((n, C, ty, tx), **f32)
        self.tiles0 = torch.empty((n, C, ty0, tx0), **f32) if self.ds > 1 else self.tiles
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
        nl = self.n_local
        if micro is None:
            # multi-rank mode runs its engines one after another on one stream
            # (_process_region_ranks), so one whole-chip engine there
            micro = 2 if nl >= 32 and not self.info.enabled else 1
        self.micro = max(1, min(int(micro), max(nl, 1)))
        per = (max(nl, 1) + self.micro - 1) // self.micro
        self.split = [max(1, min(per, nl - k * per)) for k in range(self.micro)]
        if self.info.enabled:
            graph = False
            self.idx_local = torch.arange(r_, n, W_, device=d)
            sub = (max(nl, 1), C)
            self.sub_tiles = torch.empty(sub + (ty, tx), **f32)
            self.sub_lr = torch.empty(sub + (ty // s, tx // s), **f32)
            self.sub_sr = torch.empty(sub + (ty, tx), **f32)
            self.sub_interp = torch.empty(sub + (ty, tx), **f32)
            self.sub_out = torch.zeros(1 + max(nl, 1), **f32)
            self.sums = {"model": torch.zeros(n, **f32), "interpolated": torch.zeros(n, **f32)}
        budget = 256 // self.micro if self.micro > 1 else 0
        self.engs = [Engine(spec, m, (ty // s, tx // s), train=False, device=d, cu_budget=budget)
                     for m in self.split]
        self.eng = self.engs[0]
        for e in self.engs:
            e.pack(params)
        self.streams = [None] + [engine_stream(d) for _ in range(self.micro - 1)]
        # fork / join events, created once (also valid inside a graph capture)
        self.ev_fork = torch.cuda.Event()
        self.ev_join = [torch.cuda.Event() for _ in range(self.micro - 1)]
        self._graph = None
        self._use_graph = graph and self.device.type == "cuda"

    # ---------------------------------------------------------------- pieces
    def _tile(self):
        st = stream_handle()
        call("srmi_region_to_tiles", ptr(self.region), self.C, self.H, self.W, self.ty0, self.tx0, ptr(self.tiles0),
             ptr(self.mean), ptr(self.std), ptr(self.bad), st)
        if self.ds > 1:  # apply_network: downsample(input, scale_factor=ds) of the normalised tiles
            downsample(self.tiles0, self.ds, out=self.tiles, mode=self.dmode)

    def _model_and_mosaic(self, tiles, lr, sr, interp, mean, std, inv, nt):
        st = stream_handle()
        downsample(tiles, self.s, out=lr, mode=self.dmode)
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
        upsample(lr, self.s, out=interp, mode=self.umode)
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
        if self.info.enabled:
            self._process_region_ranks()
            return self.images, {"model": self.loss_m[0:1], "interpolated": self.loss_i[0:1]}
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

    def process_image(self, region: torch.Tensor, varnames: Sequence[str], var: Optional[str] = None
                      ) -> Tuple[Dict[str, Dict[str, torch.Tensor]], Dict[str, Dict[str, float]]]:
        """process_image (dual_trainer.py:396-447) with the reference's per-variable
        return: ({vname: {image type: [y, x]}}, {vname: {'model', 'interpolated'}}).
        ``var`` selects the output variables as ``kwargs.get('var')`` does
        (:413-414): output_vars = [var] if given, else varnames.  The image of the
        i-th OUTPUT variable is channel i of the batch (assemble_images(batches,
        ivar, ...) with ivar from enumerate(output_vars), :437-438) -- so with var
        given, channel 0 is returned under that name whatever its position, exactly
        as the reference does.  The losses are over all channels, the same for every
        variable (:443-446).  The images are views of the mosaic buffers, valid until
        the next region is processed (as process_region's)."""
        images, losses = self.process_region(region)
        lm, li = float(losses["model"]), float(losses["interpolated"])
        output_vars = [var] if var is not None else list(varnames)
        out_im: Dict[str, Dict[str, torch.Tensor]] = {}
        out_l: Dict[str, Dict[str, float]] = {}
        for ivar, v in enumerate(output_vars):
            out_im[v] = {k: img[ivar] for k, img in images.items()}
            out_l[v] = {"model": lm, "interpolated": li}
        return out_im, out_l

    def evaluate(self, regions: Sequence[torch.Tensor], time_index: int = -1, tile_index: int = -1,
                 batch_domain: str = "tiles") -> Tuple[Dict[str, torch.Tensor], Dict[str, float]]:
        """ModelTrainer.evaluate (dual_trainer.py:482-543) over the time slices of a
        tset: every region is tiled, normalised and scored batch by batch; the loss
        is the mean over ALL scored batches of all scored regions (:532, :541), while
        the results are those of the LAST evaluated region only -- the reference
        clears them at the start of every time slice (clear_results, :505, :545-549)
        and then concatenates that slice's batches (merge_results / merge_results_tiles,
        :551-555, :38-42): input [n, C, ty/s, tx/s], target / model / interpolated
        [n, C, ty, tx] (device tensors, normalised tiles).

        Selection (:487-488, :504, :508-527):
        * ``time_index`` >= 0 scores only ``regions[time_index]`` (itime == time_index);
        * ``tile_index`` >= 0 scores only the batch that tile_in_batch accepts (:366-372)
          and stops there: batch_domain 'tiles' (the SWOT datasets) -- the batch whose
          tile range [start, end) holds tile_index; 'time' -- the batch whose ordinal
          is tile_index.  No matching batch: nothing is scored in that region (its
          results stay cleared).
        The validation-checkpoint policy applied to the returned loss is
        ValidationCheckpoint.update (srmi.harness)."""
        if batch_domain not in ("tiles", "time"):
            raise ValueError(f"unknown batch domain {batch_domain!r}")
        bm: List[torch.Tensor] = []
        bi: List[torch.Tensor] = []
        empty = {k: torch.empty(0, device=self.device) for k in ("input", "target", "model", "interpolated")}
        results: Dict[str, torch.Tensor] = dict(empty)
        for itime, region in enumerate(regions):
            if time_index >= 0 and itime != time_index:
                continue
            self.process_region(region)
            nt = self.n_kept
            b = self.batch_losses()
            results = dict(empty)  # clear_results(tset) at the start of the time slice
            if tile_index < 0:
                a0, a1, sel = 0, nt, slice(None)
            else:
                bs = self.batch_size
                ib = tile_index // bs if batch_domain == "tiles" else tile_index
                a0, a1 = ib * bs, min(nt, (ib + 1) * bs)
                sel = slice(ib, ib + 1)
                if a0 >= nt or (batch_domain == "tiles" and tile_index >= nt):  # no batch of this slice holds it
                    if time_index >= 0:
                        break
                    continue
            bm.append(b["model"][sel].clone())
            bi.append(b["interpolated"][sel].clone())
            results = {"input": self.lr[a0:a1].clone(), "target": self._kept_tiles[a0:a1].clone(),
                       "model": self.sr[a0:a1].clone(), "interpolated": self.interp[a0:a1].clone()}
            if time_index >= 0:
                break
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

    # ------------------------------------------------------------ multi-rank
    def _gather(self, x: torch.Tensor) -> torch.Tensor:
        return gather_round_robin(x[:self.n_local], self.n, self.rr_world)

    def _process_region_ranks(self):
        nl = self.n_local
        if nl > 0:
            torch.index_select(self.tiles, 0, self.idx_local, out=self.sub_tiles[:nl])
            downsample(self.sub_tiles[:nl], self.s, out=self.sub_lr[:nl], mode=self.dmode)
            a = 0
            for e, m in zip(self.engs, self.split):
                b = min(nl, a + m)
                if b > a:
                    e.forward(self.params, self.sub_lr[a:b], out=self.sub_sr[a:b])
                a = b
            upsample(self.sub_lr[:nl], self.s, out=self.sub_interp[:nl], mode=self.umode)
        st = stream_handle()
        te = self.C * self.ty * self.tx
        sums = {}
        for name, pred in (("model", self.sub_sr), ("interpolated", self.sub_interp)):
            work = torch.zeros(max(nl, 1), dtype=torch.float32, device=self.device)
            if nl > 0:  # per-tile sums: srmi_batch_losses' first pass into `work`; its mean pass sees
                # ONE batch of all nl tiles (the pass holds at most 1024 batches, so batches of one
                # tile would cap a rank at 1024 tiles)
                call("srmi_batch_losses", ptr(pred), ptr(self.sub_tiles), nl, te, nl, self.loss_kind, CHARBONNIER_EPS,
                     ptr(work), ptr(self.sub_out), st)
            sums[name] = self._gather(work[:, None])[:, 0]
        lr = self._gather(self.sub_lr)
        sr = self._gather(self.sub_sr)
        interp = self._gather(self.sub_interp)
        keep = torch.nonzero(self.bad == 0).flatten()
        nt = int(keep.numel())
        self.n_kept = nt
        if nt == 0:
            for img in self.images.values():
                img.fill_(float("nan"))
            self.loss_m.fill_(float("nan"))
            self.loss_i.fill_(float("nan"))
            self._kept_tiles = self.tiles[:0]
            return
        inv = None
        mean, std, tiles = self.mean, self.std, self.tiles
        if nt < self.n:
            inv = torch.full((self.n,), -1, dtype=torch.int32, device=self.device)
            inv[keep] = torch.arange(nt, dtype=torch.int32, device=self.device)
            tiles = tiles.index_select(0, keep).contiguous()
            mean = mean.index_select(0, keep).contiguous()
            std = std.index_select(0, keep).contiguous()
            lr, sr, interp = (x.index_select(0, keep).contiguous() for x in (lr, sr, interp))
            sums = {k: v.index_select(0, keep).contiguous() for k, v in sums.items()}
        self._kept_tiles = tiles
        self.lr[:nt].copy_(lr)
        self.sr[:nt].copy_(sr)
        self.interp[:nt].copy_(interp)
        for name, lo in (("model", self.loss_m), ("interpolated", self.loss_i)):
            call("srmi_batch_loss_means", ptr(sums[name]), nt, te, self.batch_size, self.loss_kind, ptr(lo), st)
        C, gy, gx, s = self.C, self.gy, self.gx, self.s
        for name, src, ty, tx in (("input", self.lr, self.ty // s, self.tx // s), ("target", tiles, self.ty, self.tx),
                                  ("interpolated", self.interp, self.ty, self.tx), ("model", self.sr, self.ty, self.tx)):
            call("srmi_tiles_to_region", ptr(src), ptr(mean), ptr(std), ptr(inv), C, ty, tx, gy, gx,
                 ptr(self.images[name]), st)

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
