"""Synthetic LLC4320 inputs for the on-disk source row.

The reference reads a big-endian float32 mask template (meta/hFacC_k0.data,
13 * nx^2 values, 0 = land) and one big-endian float32 file per variable and time
holding only the wet values in template order (sres/base/source/swot/raw.py:133-145).
These helpers build such inputs from an integer hash of the linear LLC index
(no RNG stream, so any chunk can be regenerated independently): ~23 % scattered
land outside the test ROI, ocean inside it except two land blocks, so that the
tiler drops some tiles and keeps others.
"""
import numpy as np

NX = 4320  # the reference's mds2d default (util.py:9): inputs must be full LLC4320 size
ROI = dict(y0=9500, ys=384, x0=8256, xs=768)  # spans the east/west seam at x = 2 * NX


def _hash(i):
    h = (i.astype(np.uint64) * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)
    return h ^ (h >> np.uint64(15))


def llc_index(Y, X, nx=NX):
    """Linear LLC index of pixel (Y, X) of the assembled [3nx, 4nx] east|west image
    (np.c_[east, west.T[::-1, :]] of mds2d, util.py:3-7)."""
    Y = np.asarray(Y, dtype=np.int64)
    X = np.asarray(X, dtype=np.int64)
    east0 = Y * nx + X
    east1 = 3 * nx * nx + Y * nx + (X - nx)
    Xw = X - 2 * nx
    west = 7 * nx * nx + Xw * 3 * nx + (3 * nx - 1 - Y)
    return np.where(X < nx, east0, np.where(X < 2 * nx, east1, west))


def template(nx=NX, roi=ROI):
    """template float32 [13 nx^2]: 1 wet / 0 land (native order; written '>f4')."""
    n = 13 * nx * nx
    tmpl = np.empty(n, dtype=np.float32)
    step = 1 << 24
    for a in range(0, n, step):
        i = np.arange(a, min(n, a + step), dtype=np.uint64)
        tmpl[a:a + len(i)] = ((_hash(i) >> np.uint64(24)) >= np.uint64(60)).astype(np.float32)  # ~23 % land
    # the ROI is ocean except two land blocks: one in tile (0, 0) (east face) and
    # one in tile (1, 2) (west face, past the seam), so get_tiles drops 2 of 8 tiles
    ys, xs = np.meshgrid(np.arange(roi["y0"], roi["y0"] + roi["ys"]), np.arange(roi["x0"], roi["x0"] + roi["xs"]),
                         indexing="ij")
    tmpl[llc_index(ys.ravel(), xs.ravel(), nx)] = 1.0
    for (ya, yb, xa, xb) in ((20, 60, 30, 90), (250, 262, 400, 470)):
        ys, xs = np.meshgrid(np.arange(roi["y0"] + ya, roi["y0"] + yb), np.arange(roi["x0"] + xa, roi["x0"] + xb),
                             indexing="ij")
        tmpl[llc_index(ys.ravel(), xs.ravel(), nx)] = 0.0
    return tmpl


def wet_values(tmpl, var: int):
    """The wet values of variable `var` in template order (float32, native order)."""
    wet = np.flatnonzero(tmpl)
    vals = np.empty(len(wet), dtype=np.float32)
    step = 1 << 24
    for a in range(0, len(wet), step):
        i = wet[a:a + step].astype(np.uint64)
        h = _hash(i + np.uint64(977 * (var + 1)))
        vals[a:a + len(i)] = (280.0 + 10.0 * np.sin(i.astype(np.float64) * 1e-5 + var)
                              + (h & np.uint64(0xFFFF)).astype(np.float64) / 65536.0).astype(np.float32)
    return vals


def write_files(root, nvars=2, nx=NX):
    """Write meta/tmpl.data and raw/var{k}.data ('>f4') under root; -> (template
    name, [data names])."""
    import os
    os.makedirs(os.path.join(root, "meta"), exist_ok=True)
    os.makedirs(os.path.join(root, "raw"), exist_ok=True)
    tmpl = template(nx)
    tmpl.astype(">f4").tofile(os.path.join(root, "meta", "tmpl.data"))
    names = []
    for k in range(nvars):
        wet_values(tmpl, k).astype(">f4").tofile(os.path.join(root, "raw", f"var{k}.data"))
        names.append(f"raw/var{k}.data")
    return "meta/tmpl.data", names
