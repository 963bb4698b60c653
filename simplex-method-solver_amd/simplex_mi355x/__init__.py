"""simplex_mi355x -- MI355X-native simplex pivot engine (drop-in for src/simplex.py's solver).

The tableau lives in HBM as a row-major fp64 matrix; selection and the rank-1 Gauss-Jordan update
are hand-written gfx950 HIP kernels (csrc/smx_*.hpp + smx_kernels.hip -> libsmx.so, C ABI in include/smx.h)
reached through thin torch custom ops (ops.py).  Importing this package loads libsmx.so and
fails loudly if it has not been built.
"""
from . import _lib

_lib.load()  # no silent fallback: a missing/broken libsmx.so is an import error

from .engine import Error, Info, SimplexMethod  # noqa: E402
from .device import DeviceTableau  # noqa: E402

__all__ = ["SimplexMethod", "Info", "Error", "DeviceTableau"]
