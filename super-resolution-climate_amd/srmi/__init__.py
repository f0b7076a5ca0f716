"""srmi -- MI355X-native (gfx950) engine for the RCAN/EDSR tiled super-resolution
hot path of nasa-nccs-hpda/super-resolution-climate.

Product path: hand-written HIP kernels in libsrmi.so behind a C ABI
(include/srmi.h), bound with ctypes (srmi._lib).  No CPU fallback.
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401
from .config import ConfigContext, cfg  # noqa: F401
from .engine import Engine, NetSpec, adam_step, downsample, param_names, param_table, upsample  # noqa: F401


def get_model(name: str = "rcan", **config):
    """importlib-style plugin access: srmi.get_model('rcan', nchannels_in=2, ...)."""
    import importlib
    return importlib.import_module(f"srmi.model.{name}.network").get_model(**config)
