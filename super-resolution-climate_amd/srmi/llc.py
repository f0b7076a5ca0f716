"""On-disk LLC4320 source -> tiles on the device.

Mirrors the reference's SWOTRawDataLoader (sres/base/source/swot/raw.py):

* ``load_file`` (:133-145): read the '>f4' mask template and a '>f4' wet-value
  file, put the values into the wet cells (land = NaN), split the LLC faces
  (``mds2d``, swot/util.py:3-7), assemble ``east | west.T[::-1]`` and cut the
  ROI (``subset_roi``, :38-45) -> [1, ys, xs];
* ``load_region_data`` (:155-158): the variables stacked -> [C, ys, xs];
* ``get_tiles`` (:216-233): floor tiling, removal of tiles whose mean is not
  finite, and -- reproduced on purpose, as the reference does it -- the
  channel-major flattening that packs consecutive kept tiles of the same
  variable into the channel axis when C > 1.

The host only reads raw file bytes (no decoding); the byte swap, mask
expansion, face rearrangement and ROI cut are HIP kernels (tiles.hip).  The
template -> ROI index map is built once per template on the device (mask scan),
after which each file is one gather.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import call, ptr, stream_handle


def _read_words(path: str) -> np.ndarray:
    """Raw file bytes as uint32 words (the '>f4' values still big-endian)."""
    b = np.fromfile(path, dtype=np.uint8)
    if b.size % 4:
        raise ValueError(f"{path}: size {b.size} is not a multiple of 4 bytes")
    return b.view(np.uint32)


class LLCSource:
    """template_path: the '>f4' hFacC template (13 * nx^2 cells); roi: the
    dataset's roi dict (y0, ys, x0, xs; missing keys = the full extent) or None."""

    def __init__(self, template_path: str, roi: Optional[Dict] = None, nx: int = 4320,
                 device: Optional[torch.device] = None):
        self.nx = nx
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        H, W = 3 * nx, 4 * nx
        roi = roi or {}
        self.x0, self.xs = int(roi.get("x0", 0)), int(roi.get("xs", W))
        self.y0, self.ys = int(roi.get("y0", 0)), int(roi.get("ys", H))
        self.y0, self.x0 = min(self.y0, H), min(self.x0, W)      # numpy slicing semantics
        self.ys, self.xs = min(self.ys, H - self.y0), min(self.xs, W - self.x0)
        words = _read_words(template_path)
        n = words.size
        if n != 13 * nx * nx:
            raise ValueError(f"template has {n} cells, LLC{nx} needs {13 * nx * nx}")
        tmpl = torch.from_numpy(words.view(np.int32)).to(self.device)
        ws = C.c_size_t(0)
        call("srmi_llc_index_map_workspace", n, C.byref(ws))
        work = torch.empty(ws.value, dtype=torch.uint8, device=self.device)
        self.idx = torch.empty(self.ys * self.xs, dtype=torch.int32, device=self.device)
        nwet = torch.zeros(1, dtype=torch.int64, device=self.device)
        call("srmi_llc_index_map", ptr(tmpl), n, nx, self.y0, self.ys, self.x0, self.xs, ptr(self.idx), ptr(nwet),
             ptr(work), ws.value, stream_handle())
        self.n_wet = int(nwet.item())
        del work, tmpl

    def load_file(self, data_path: str, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One variable, one time index -> [1, ys, xs] fp32 on the device."""
        words = _read_words(data_path)
        if words.size != self.n_wet:
            # numpy's boolean-mask assignment in the reference raises here too
            raise ValueError(f"{data_path}: {words.size} values for {self.n_wet} wet cells")
        data = torch.from_numpy(words.view(np.int32)).to(self.device)
        if out is None:
            out = torch.empty(1, self.ys, self.xs, dtype=torch.float32, device=self.device)
        call("srmi_llc_gather", ptr(data), words.size, ptr(self.idx), self.ys * self.xs, ptr(out), stream_handle())
        return out

    def load_region_data(self, data_paths: Sequence[str]) -> torch.Tensor:
        """The variables stacked on the channel axis -> [C, ys, xs]."""
        out = torch.empty(len(data_paths), self.ys, self.xs, dtype=torch.float32, device=self.device)
        for c, pth in enumerate(data_paths):
            self.load_file(pth, out=out[c:c + 1])
        return out


def get_tiles(region: torch.Tensor, ty: int, tx: int) -> Tuple[torch.Tensor, np.ndarray, Tuple[int, int]]:
    """get_tiles (raw.py:216-233) on a device region [C, H, W] -> (tiles [n//C, C,
    ty, tx], tile ids (the first n//C kept ids of the channel-major flattening, as
    the reference's coords), (gy, gx)).  One host sync for the keep mask (the
    reference does this once per time slice)."""
    if region.dtype != torch.float32 or region.dim() != 3 or not region.is_contiguous():
        raise ValueError("get_tiles: region must be a contiguous fp32 [C, H, W] device tensor")
    Cn, H, W = region.shape
    gy, gx = H // ty, W // tx
    bad = torch.empty(Cn * gy * gx, dtype=torch.int32, device=region.device)
    call("srmi_tiles_nonfinite", ptr(region), Cn, H, W, ty, tx, ptr(bad), stream_handle())
    keep = np.flatnonzero(bad.cpu().numpy() == 0)
    n = keep.size // Cn
    src = torch.from_numpy(keep[:n * Cn].astype(np.int32)).to(region.device)
    tiles = torch.empty(n, Cn, ty, tx, dtype=torch.float32, device=region.device)
    call("srmi_tiles_gather", ptr(region), Cn, H, W, ty, tx, ptr(src), n * Cn, ptr(tiles), stream_handle())
    return tiles, keep[:n], (gy, gx)
