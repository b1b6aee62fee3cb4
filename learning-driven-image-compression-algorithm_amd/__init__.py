"""lic_amd — MI355X-native (gfx950) encode -> quantize -> decode engine for the
learned image codec of xiaobucc/learning-driven-image-compression-algorithm.

Layout mirrors the reference: ``layers/`` (GDN, window attention,
Win_noShift_Attention, compressai blocks), ``model/`` (net_ga, net_unet_ha_hs,
Block_unet, gdn), ``ops/`` (LowerBound, NonNegativeParametrizer).  Every
activation-sized op runs in liblic.so (csrc/, C ABI in include/lic.h) through
``_ffi`` (ctypes); ``functional`` holds the tensor-level wrappers.
"""
from . import _ffi, functional
from ._ffi import LicError

__all__ = ["_ffi", "functional", "LicError", "load_library"]


def load_library():
    """Load liblic.so (raises LicError if it is missing)."""
    return _ffi.load()
