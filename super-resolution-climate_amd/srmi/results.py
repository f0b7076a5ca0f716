"""Inference result files: drop-in for sres/data/inference.py.

Reference (sres/data/inference.py:10-50, called from WorkflowController.inference,
sres/controller/workflow.py:53-75):

* ``results_path``: ``{platform.results}/inference/{dataset}/{task}/{var}-{t}.{tiles|image}[_ds-{f:.2f}].nc``
  (``_ds-`` only when ``task.data_downsample`` != 1).
* ``save_inference_results``: one Dataset per variable and time step with the data
  variables ``input`` (dims renamed y -> ys, x -> xs), ``target``, ``interpolated``
  and ``model``, and the global attributes ``loss_keys`` / ``loss_values``.
* The arrays come in two structures:
  - Image (process_image -> assemble_images, dual_trainer.py:449-480): ``[y, x]``
    mosaics, coordinates ``arange(0, 100, 100 / n)`` on both axes;
  - Tiles (evaluate -> to_xa, dual_trainer.py:148-155): ``[tiles, channels, y, x]``
    float32 with integer coordinates, then ``squeeze()`` for one variable (the
    ``channels`` coordinate stays as a scalar) or ``sel(channels=v, drop=True)``
    for several (workflow.py:61-67).

xarray and netCDF4 are not installed here, so the file is written with
``scipy.io.netcdf_file`` -- the engine xarray itself falls back to without
netCDF4 -- as NETCDF3_64BIT: int64 coordinates are stored as int32 (xarray's
netCDF-3 coercion), float variables carry ``_FillValue = NaN`` (xarray's
default encoding), a scalar string coordinate is a char variable over a
``string{N}`` dimension.  netCDF-3 has no string-array attributes, so
``loss_keys`` is stored as ONE char attribute, the keys joined by ``,``;
``load_inference_results`` splits it back (the reference's loader zips the
attribute as a list and would need that split).  Parity of the byte layout
against xarray's own writer is unpinned (no xarray here); the round trip through
scipy is tested.
"""
from __future__ import annotations

import glob
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

STRUCTURES = ("tiles", "image")  # ResultStructure values (sres/controller/config.py:3-5)


@dataclass
class Var:
    """A labelled array (the subset of xarray.DataArray the result files need)."""
    dims: Tuple[str, ...]
    values: np.ndarray
    coords: Dict[str, np.ndarray] = field(default_factory=dict)  # dimension coordinates
    scalar_coords: Dict[str, object] = field(default_factory=dict)  # e.g. channels='SST'


def results_path(results_root: str, dataset: str, task: str, varname: str, timestep, structure: str,
                 data_downsample: float = 1.0, remove: bool = False) -> str:
    """results_path (inference.py:10-18)."""
    if structure not in STRUCTURES:
        raise ValueError(f"unknown result structure {structure!r}")
    f = float(data_downsample)
    dss = "" if f == 1.0 else f"_ds-{f:.2f}"
    p = f"{results_root}/inference/{dataset}/{task}/{varname}-{timestep}.{structure}{dss}.nc"
    os.makedirs(os.path.dirname(p), exist_ok=True)
    if remove and os.path.exists(p):
        os.remove(p)
    return p


def time_indices(results_root: str, dataset: str, task: str, varname: str, structure: str,
                 data_downsample: float = 1.0) -> List[int]:
    """time_indices (inference.py:20-22): the time steps that have a result file."""
    pat = results_path(results_root, dataset, task, varname, "*", structure, data_downsample)
    return [int(Path(fn).stem.split(".")[0].split("-")[1]) for fn in glob.glob(pat)]


def _np(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def image_results(images: Dict[str, object], varnames: Sequence[str]) -> Dict[str, Dict[str, Var]]:
    """Per-variable Image results from srmi.inference.TiledInference.process_region
    images ([C, H, W] per type): assemble_images' [y, x] arrays with coordinates
    arange(0, 100, 100 / n) (dual_trainer.py:475-478)."""
    out: Dict[str, Dict[str, Var]] = {}
    for iv, v in enumerate(varnames):
        d = {}
        for k, img in images.items():
            a = _np(img)[iv].astype(np.float64)  # np.block of float64 NaN-filled cells
            co = {cn: np.arange(0.0, 100.0, 100.0 / a.shape[ic]) for ic, cn in enumerate(("y", "x"))}
            d[k] = Var(("y", "x"), a, co)
        out[v] = d
    return out


def tiles_results(results: Dict[str, object], varnames: Sequence[str]) -> Dict[str, Dict[str, Var]]:
    """Per-variable Tiles results from TiledInference.evaluate's [n, C, h, w] arrays:
    to_xa (dual_trainer.py:148-155, float32, coords tiles / channels / y / x),
    then squeeze() for one variable or sel(channels=v, drop=True) (workflow.py:61-67)."""
    out: Dict[str, Dict[str, Var]] = {v: {} for v in varnames}
    for k, arr in results.items():
        a = _np(arr).astype(np.float32)
        n, C, h, w = a.shape
        if C != len(varnames):
            raise ValueError(f"{k}: {C} channels for {len(varnames)} variables")
        coords = {"tiles": np.arange(n), "y": np.arange(h), "x": np.arange(w)}
        for iv, v in enumerate(varnames):
            if len(varnames) == 1:  # squeeze(): every size-1 dim becomes a scalar coordinate
                dims = [d for d, s in zip(("tiles", "channels", "y", "x"), a.shape) if s != 1]
                sc = {"channels": v}
                if n == 1:
                    sc["tiles"] = 0
                co = {d: coords[d] for d in dims}
                out[v][k] = Var(tuple(dims), a.reshape([s for s in a.shape if s != 1]), co, sc)
            else:
                out[v][k] = Var(("tiles", "y", "x"), a[:, iv], dict(coords))
    return out


def _nc3(a: np.ndarray) -> np.ndarray:
    """xarray's netCDF-3 dtype coercion (int64 -> int32, bool -> int8)."""
    if a.dtype == np.int64 or a.dtype == np.uint64:
        return a.astype(np.int32)
    if a.dtype == np.bool_:
        return a.astype(np.int8)
    return a


def save_inference_results(path: str, var_results: Dict[str, Var], losses: Dict[str, float]) -> str:
    """save_inference_results (inference.py:24-31) for ONE variable: ``input``'s
    y / x renamed ys / xs, Dataset(data_vars, attrs(loss_keys, loss_values))."""
    from scipy.io import netcdf_file
    vr = dict(var_results)
    if "input" in vr:
        iv = vr["input"]
        ren = {"y": "ys", "x": "xs"}
        vr["input"] = Var(tuple(ren.get(d, d) for d in iv.dims), iv.values,
                          {ren.get(d, d): c for d, c in iv.coords.items()}, dict(iv.scalar_coords))
    dims: Dict[str, int] = {}
    coords: Dict[str, np.ndarray] = {}
    scalars: Dict[str, object] = {}
    for name, v in vr.items():
        if v.values.ndim != len(v.dims):
            raise ValueError(f"{name}: {v.values.ndim}-d values for dims {v.dims}")
        for d, s in zip(v.dims, v.values.shape):
            if dims.setdefault(d, s) != s:
                raise ValueError(f"dimension {d}: size {s} != {dims[d]}")
        coords.update(v.coords)
        scalars.update(v.scalar_coords)
    if os.path.exists(path):
        os.remove(path)
    with netcdf_file(path, "w", version=2) as f:
        f.loss_keys = ",".join(str(k) for k in losses.keys())
        f.loss_values = np.asarray([float(x) for x in losses.values()], dtype=np.float64)
        for d, s in dims.items():
            f.createDimension(d, s)
        for d, c in coords.items():  # dimension coordinates
            c = _nc3(np.asarray(c))
            cv = f.createVariable(d, c.dtype, (d,))
            cv[:] = c
            if c.dtype.kind == "f":
                cv._FillValue = np.array([np.nan], dtype=c.dtype)
        for sname, sval in scalars.items():  # scalar coordinates
            if isinstance(sval, str):
                b = np.frombuffer(sval.encode("utf-8"), dtype="S1")
                sd = f"string{len(b)}"
                if sd not in dims:
                    f.createDimension(sd, len(b))
                    dims[sd] = len(b)
                sv = f.createVariable(sname, "c", (sd,))
                sv[:] = b
            else:
                a = _nc3(np.asarray(sval))
                sv = f.createVariable(sname, a.dtype, ())
                sv.assignValue(a)
        for name, v in vr.items():
            a = _nc3(np.ascontiguousarray(v.values))
            dv = f.createVariable(name, a.dtype, v.dims)
            if a.dtype.kind == "f":
                dv._FillValue = np.array([np.nan], dtype=a.dtype)
            if v.scalar_coords:
                dv.coordinates = " ".join(v.scalar_coords.keys())
            dv[:] = a
    return path


def load_inference_results(path: str) -> Tuple[Dict[str, Var], Dict[str, float]]:
    """load_inference_results (inference.py:40-50): the data variables (``input``
    renamed back to y / x) and the losses dict."""
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as f:
        keys = f.loss_keys.decode() if isinstance(f.loss_keys, bytes) else str(f.loss_keys)
        vals = np.atleast_1d(f.loss_values).tolist()
        losses = dict(zip(keys.split(",") if keys else [], vals))
        names = [n for n in ("input", "target", "interpolated", "model") if n in f.variables]
        out: Dict[str, Var] = {}
        for n in names:
            v = f.variables[n]
            dims = tuple(v.dimensions)
            co = {d: np.array(f.variables[d][:]) for d in dims if d in f.variables}
            sc: Dict[str, object] = {}
            for s in getattr(v, "coordinates", b"").decode().split() if hasattr(v, "coordinates") else []:
                sv = f.variables[s]
                sc[s] = b"".join(sv[:].tolist()).decode() if sv.typecode() == "c" else sv.getValue()
            vals_ = np.array(v[:])
            if n == "input":
                ren = {"ys": "y", "xs": "x"}
                dims = tuple(ren.get(d, d) for d in dims)
                co = {ren.get(d, d): c for d, c in co.items()}
            out[n] = Var(dims, vals_, co, sc)
    return out, losses
