"""Device operators: fused HIP kernels for gfx950 with torch reference implementations."""
from . import _lib
from ._lib import available as native_available, NativeUnavailable

__all__ = ["native_available", "NativeUnavailable"]
