"""bedops_amd — MI355X-native engine for the BEDOPS sorted-interval sweep path.

The product is the C-ABI library ``bedops_amd/lib/libbedgpu.so`` (HIP kernels for
gfx950, declared in ``include/bedgpu.h``) and the drop-in C front-ends
``bedops_amd/bin/{bedops,bedmap}``. This package is the Python host mirror of that
path: it binds the C ABI with ctypes and exposes the reference's operations with the
reference's argument meaning (``bedops -m/-i/-d/-e/-n``, ``bedmap --count/--mean``).
There is no CPU fallback: if the library cannot be loaded, importing the engine
raises.
"""
from .engine import (BedgpuError, Engine, MAP_COUNT, MAP_MEAN, BED3, BED3_REST,  # noqa: F401
                     BED5, lib_path)

__all__ = ["Engine", "BedgpuError", "MAP_COUNT", "MAP_MEAN", "BED3", "BED3_REST", "BED5",
           "lib_path"]
