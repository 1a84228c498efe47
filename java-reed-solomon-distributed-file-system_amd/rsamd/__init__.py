"""rsamd -- MI355X-native Reed-Solomon erasure coding (GF(2^8), poly 0x11D).

Host-side mirror of the reference codec API (Backblaze JavaReedSolomon as used
by hzhou279/Java-Reed-Solomon-Distributed-File-System) over the C-ABI in
include/rs_amd.h.  Every byte of shard data is coded by the HIP kernels in
csrc/kernels.hip; there is no CPU coding path.
"""
from . import _lib  # noqa: F401
from .codec import (  # noqa: F401
    GpuError,
    IllegalArgumentException,
    ReedSolomon,
    checkSomeShards,
    codeSomeShards,
)
from . import device  # noqa: F401

__all__ = ["ReedSolomon", "IllegalArgumentException", "GpuError", "codeSomeShards", "checkSomeShards", "device"]
