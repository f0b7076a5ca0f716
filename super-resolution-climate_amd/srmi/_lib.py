"""ctypes binding of the srmi C ABI (include/srmi.h) -> libsrmi.so (in-tree).

The library is the product path: there is no CPU / PyTorch fallback.  If the
shared object is missing, or the device is not a gfx950 GPU, every entry point
raises.  Build it with ``make`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH_DEFAULT = os.path.join(_HERE, "libsrmi.so")
LIB_PATH = os.environ.get("SRMI_LIB") or LIB_PATH_DEFAULT  # SRMI_LIB: diagnostic build

SRMI_ARCH_RCAN = 0
SRMI_ARCH_EDSR = 1
SRMI_DTYPE_BF16 = 0
SRMI_FLAG_NO_RCAB_INFER = 2
SRMI_FLAG_CA_PASS = 4
SRMI_FLAG_DU_PASS = 16
SRMI_DTYPE_F32 = 1
SRMI_LOSS_RMSE = 0
SRMI_LOSS_MEAN = 1
SRMI_INTERP_BILINEAR = 1
SRMI_INTERP_BICUBIC = 2
TILE_LOSS_SUB = 16  # parts per tile of srmi_tile_loss_parts

ERRORS = {-10001: "SRMI_ERR_ARG", -10002: "SRMI_ERR_SHAPE", -10003: "SRMI_ERR_WORKSPACE",
          -10004: "SRMI_ERR_UNSUPPORTED"}


class ModelConfig(C.Structure):
    _fields_ = [("arch", C.c_int), ("nchannels_in", C.c_int), ("nchannels_out", C.c_int),
                ("nfeatures", C.c_int), ("nlayers", C.c_int), ("nblocks", C.c_int), ("reduction", C.c_int),
                ("scale", C.c_int), ("res_scale", C.c_float), ("batch", C.c_int), ("lr_h", C.c_int),
                ("lr_w", C.c_int), ("cu_budget", C.c_int), ("dtype", C.c_int), ("flags", C.c_int)]


class ParamInfo(C.Structure):
    _fields_ = [("offset", C.c_longlong), ("numel", C.c_longlong), ("ndim", C.c_int), ("shape", C.c_int * 4)]


P = C.c_void_p
F = C.POINTER(C.c_float)
_SIGS = {
    "srmi_version": ([], C.c_int),
    "srmi_param_count": ([C.POINTER(ModelConfig), C.POINTER(C.c_longlong), C.POINTER(C.c_int)], C.c_int),
    "srmi_param_table": ([C.POINTER(ModelConfig), C.POINTER(ParamInfo), C.c_int], C.c_int),
    "srmi_workspace_size": ([C.POINTER(ModelConfig), C.c_int, C.POINTER(C.c_size_t)], C.c_int),
    "srmi_engine_create": ([C.POINTER(ModelConfig), P, C.c_size_t, C.c_int, C.POINTER(P)], C.c_int),
    "srmi_engine_destroy": ([P], C.c_int),
    "srmi_pack_weights": ([P, P, P], C.c_int),
    "srmi_forward": ([P, P, P, P, C.c_int, P], C.c_int),
    "srmi_backward": ([P, P, P, P, P, P, P, P, C.POINTER(P), P], C.c_int),
    "srmi_backward_stage_count": ([P], C.c_int),
    "srmi_backward_stages": ([P, P, P, P, P, P, P, P, C.POINTER(P), C.c_int, C.c_int, P], C.c_int),
    "srmi_engine_probe": ([P, C.c_int, C.c_int, P], C.c_int),
    "srmi_rmse_partial": ([P, P, P, C.c_size_t, C.c_double, P, P], C.c_int),
    "srmi_rmse_finalize": ([P, P], C.c_int),
    "srmi_charbonnier_partial": ([P, P, P, C.c_size_t, C.c_double, C.c_float, P, P, P], C.c_int),
    "srmi_loss_finalize": ([P, C.c_int, P], C.c_int),
    "srmi_loss_combine": ([P, P, C.c_int, C.c_int, P], C.c_int),
    "srmi_tile_loss_parts": ([P, P, C.c_int, C.c_longlong, C.c_int, C.c_float, P, P], C.c_int),
    "srmi_loss_from_parts": ([P, C.c_int, C.c_double, C.c_int, P, P], C.c_int),
    "srmi_batch_losses": ([P, P, C.c_int, C.c_longlong, C.c_int, C.c_int, C.c_float, P, P, P], C.c_int),
    "srmi_batch_loss_means": ([P, C.c_int, C.c_longlong, C.c_int, C.c_int, P, P], C.c_int),
    "srmi_downsample": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P], C.c_int),
    "srmi_upsample": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P], C.c_int),
    "srmi_interpolate": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float, C.c_int, P,
                          P], C.c_int),
    "srmi_adam_step": ([P, P, P, P, C.c_size_t, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, P],
                       C.c_int),
    "srmi_conv3x3": ([P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P,
                      C.c_float, C.c_int, P], C.c_int),
    "srmi_conv3x3_nstrips": ([C.c_int, C.c_int], C.c_int),
    "srmi_debug_conv_stamps": ([P], C.c_int),
    "srmi_debug_wgrad_stamps": ([P], C.c_int),
    "srmi_pack_conv": ([P, P, C.c_int, C.c_int, C.c_int, P, P, P, C.c_int, P], C.c_int),
    "srmi_wgrad3x3": ([P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_size_t, C.c_int, C.c_float,
                       P, P, C.c_int, P], C.c_int),
    "srmi_ca_forward": ([P, P, C.c_int, P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, C.c_int, P],
                        C.c_int),
    "srmi_ca_forward_pair": ([P, P, C.c_int, P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P],
                             C.c_int),
    "srmi_ca_backward": ([P, P, C.c_int, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, C.c_int, P], C.c_int),
    "srmi_head_forward": ([P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, C.c_int, P], C.c_int),
    "srmi_tail_forward": ([P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int, P], C.c_int),
    "srmi_axpy": ([P, P, C.c_float, C.c_size_t, P], C.c_int),
    "srmi_region_to_tiles": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P], C.c_int),
    "srmi_tiles_to_region": ([P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P], C.c_int),
    "srmi_batch_prep": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P], C.c_int),
    "srmi_llc_index_map_workspace": ([C.c_longlong, C.POINTER(C.c_size_t)], C.c_int),
    "srmi_llc_index_map": ([P, C.c_longlong, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, C.c_size_t, P],
                           C.c_int),
    "srmi_llc_gather": ([P, C.c_longlong, P, C.c_longlong, P, P], C.c_int),
    "srmi_tiles_nonfinite": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P], C.c_int),
    "srmi_tiles_gather": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int, P, P], C.c_int),
}
EXPORTED = tuple(_SIGS)

_lib: Optional[C.CDLL] = None


class SrmiError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libsrmi.so and declare every prototype.  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SrmiError(f"srmi HIP library not built: {path} is missing (run `make` or __graft_entry__.build()); "
                        "there is no CPU fallback")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, (args, res) in _SIGS.items():
        if path != LIB_PATH_DEFAULT and not hasattr(lib, name):
            continue  # a diagnostic build of an older revision (SRMI_LIB): entry points added since stay unbound
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise SrmiError(f"{what} failed: {ERRORS.get(rc, f'hipError {-rc}' if rc > -10000 else rc)}")
    return rc


def call(name: str, *args) -> int:
    lib = load()
    return check(getattr(lib, name)(*args), name)


def ptr(t) -> Optional[int]:
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
