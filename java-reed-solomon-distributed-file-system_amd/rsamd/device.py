"""Device-resident batched API (the benchmark path) over the C-ABI.

Stripes live in HBM as ``[stripe][shard][shard_stride]``; every call is
asynchronous on the given HIP stream.  ``torch`` is only plumbing here (device
allocation and streams); the byte work is done by the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Sequence

import numpy as np

from . import _lib
from .codec import ReedSolomon, _bools, check


@dataclass(frozen=True)
class StripeLayout:
    """Byte layout of a stripe batch in device memory."""

    n_stripes: int
    shard_len: int
    shard_stride: int
    stripe_stride: int

    @staticmethod
    def packed(n_stripes: int, total_shards: int, shard_len: int, align: int = 256, pad: int = 0) -> "StripeLayout":
        """Shards back to back at `align`-rounded strides, plus `pad` bytes
        between shards (a 4 KiB pad spreads the 14 streams of 10+4 x 4 MiB
        stripes over more HBM channels)."""
        stride = (shard_len + align - 1) // align * align + pad
        return StripeLayout(n_stripes, shard_len, stride, stride * total_shards)

    @staticmethod
    def recommended(n_stripes: int, total_shards: int, shard_len: int) -> "StripeLayout":
        """Packed shards at rs_shard_stride_recommended's stride (a pad where
        shards a power of two apart contend for HBM channels)."""
        stride = int(_lib.load().rs_shard_stride_recommended(total_shards, shard_len))
        return StripeLayout(n_stripes, shard_len, stride, stride * total_shards)

    @property
    def nbytes(self) -> int:
        return self.n_stripes * self.stripe_stride


def recommended_granule(total_shards: int) -> int:
    """rs_granule_recommended: the granule measured fastest for stripes of
    total_shards shards (4+2: 64 KiB, 10+4: 32 KiB)."""
    return int(_lib.load().rs_granule_recommended(total_shards))


@dataclass(frozen=True)
class GranuleLayout:
    """The granule layout of a stripe batch in HBM (include/rs_amd.h): the
    batch's byte columns (stripe t's column c is batch column
    x = t*shard_len + c) are stored in `granule`-byte pieces, piece j of every
    shard together, so that byte lives at
        (x // granule)*total_shards*granule + s*granule + x % granule.
    The granule divides shard_len (a stripe spans several rows) or shard_len
    divides the granule (a row holds several stripes).  Byte for byte the
    batch is the packed batch `view` of `rows` stripes of granule-byte shards,
    which the batch entry points code unchanged.  It puts a stripe's k+m
    streams `granule` bytes apart instead of shard_len.  Use
    make() to validate and pick the granule."""

    n_stripes: int
    total_shards: int
    shard_len: int
    granule: int

    @staticmethod
    def make(n_stripes: int, total_shards: int, shard_len: int, granule: int = 0) -> "GranuleLayout":
        g = granule or recommended_granule(total_shards)
        if g <= 0 or g % 16 or shard_len <= 0 or (shard_len % g and g % shard_len) or (n_stripes * shard_len) % g:
            raise ValueError(f"granule {g} (a multiple of 16) and shard_len {shard_len} must divide one another, "
                             f"and the granule must divide n_stripes * shard_len")
        return GranuleLayout(n_stripes, total_shards, shard_len, g)

    @property
    def rows(self) -> int:
        """Granule rows of the batch (stripes of the view)."""
        return self.n_stripes * self.shard_len // self.granule

    @property
    def subs_per_stripe(self) -> int:
        """Granule rows per stripe (granule <= shard_len)."""
        if self.shard_len % self.granule:
            raise ValueError("several stripes share a granule row (shard_len < granule)")
        return self.shard_len // self.granule

    @property
    def nbytes(self) -> int:
        return self.n_stripes * self.total_shards * self.shard_len

    @property
    def view(self) -> StripeLayout:
        """The packed batch of granule-byte stripes with the same bytes."""
        g = self.granule
        return StripeLayout(self.rows, g, g, self.total_shards * g)


def _kernel_layout(lay) -> StripeLayout:
    return lay.view if isinstance(lay, GranuleLayout) else lay


def copy_shard(lay: GranuleLayout, dev_base: int, stripe: int, shard: int, buf: int, to_granules: bool,
               stream=None) -> None:
    """rs_granule_copy_shard: one shard between a contiguous buffer `buf`
    (host or device address, shard_len bytes) and the granule batch.
    ValueError for a stripe or shard outside the batch (the library checks
    them too, with RS_E_INVALID)."""
    if not 0 <= stripe < lay.n_stripes:
        raise ValueError(f"stripe {stripe} outside [0, {lay.n_stripes})")
    if not 0 <= shard < lay.total_shards:
        raise ValueError(f"shard {shard} outside [0, {lay.total_shards})")
    check(_lib.load().rs_granule_copy_shard(C.c_void_p(dev_base), lay.total_shards, lay.n_stripes, lay.shard_len,
                                            lay.granule, stripe, shard, C.c_void_p(buf), int(bool(to_granules)),
                                            C.c_void_p(_stream_handle(stream))))


def _stream_handle(stream) -> int:
    if stream is None:
        return 0
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)  # torch.cuda.Stream


def encode(codec: ReedSolomon, dev_base: int, lay: StripeLayout, stream=None) -> None:
    lay = _kernel_layout(lay)
    check(_lib.load().rs_encode_batch_dev(codec.handle, C.c_void_p(dev_base), lay.n_stripes, lay.shard_len,
                                          lay.shard_stride, lay.stripe_stride, C.c_void_p(_stream_handle(stream))))


def decode(codec: ReedSolomon, dev_base: int, present: Sequence, lay: StripeLayout, stream=None) -> None:
    lay = _kernel_layout(lay)
    p = _bools(present)
    check(_lib.load().rs_decode_batch_dev(codec.handle, C.c_void_p(dev_base), p.ctypes.data_as(_lib.u8p),
                                          lay.n_stripes, lay.shard_len, lay.shard_stride, lay.stripe_stride,
                                          C.c_void_p(_stream_handle(stream))))


def decode_masked(codec: ReedSolomon, dev_base: int, present, lay: StripeLayout, stream=None) -> None:
    """Per-stripe presence patterns: present is (n_stripes, k+m) of bools/0-1
    (a C-contiguous bool or uint8 array is passed without a copy).  A
    GranuleLayout takes one pattern per stripe too
    (rs_decode_granule_masked_dev: the kernels find a block's stripe from its
    batch column, so stripes sharing a granule row may differ)."""
    p = present if isinstance(present, np.ndarray) and present.dtype in (np.bool_, np.uint8) else \
        np.asarray(present, dtype=bool)
    p = np.ascontiguousarray(p).view(np.uint8)
    if p.ndim != 2 or p.shape[0] != lay.n_stripes or p.shape[1] != codec.getTotalShardCount():
        raise ValueError(f"present must be ({lay.n_stripes}, {codec.getTotalShardCount()}), got {p.shape}")
    lib, h, st = _lib.load(), C.c_void_p(_stream_handle(stream)), p.ctypes.data_as(_lib.u8p)
    if isinstance(lay, GranuleLayout):
        check(lib.rs_decode_granule_masked_dev(codec.handle, C.c_void_p(dev_base), st, lay.n_stripes, lay.shard_len,
                                               lay.granule, h))
        return
    check(lib.rs_decode_batch_masked_dev(codec.handle, C.c_void_p(dev_base), st, lay.n_stripes, lay.shard_len,
                                         lay.shard_stride, lay.stripe_stride, h))


def decode_masked_bits(codec: ReedSolomon, dev_base: int, dev_bits: int, lay: StripeLayout, dev_bad: int = 0,
                       stream=None) -> None:
    """Per-stripe presence bitmasks already in device memory: dev_bits points
    at n_stripes uint32 words, bit i = shard i present (one word per stripe,
    for a GranuleLayout too).  Undecodable stripes are skipped and each is
    counted once into the device int32 at dev_bad (when given)."""
    lib, h = _lib.load(), C.c_void_p(_stream_handle(stream))
    if isinstance(lay, GranuleLayout):
        check(lib.rs_decode_granule_masked_bits_dev(codec.handle, C.c_void_p(dev_base), C.c_void_p(dev_bits),
                                                    lay.n_stripes, lay.shard_len, lay.granule,
                                                    C.c_void_p(dev_bad or None), h))
        return
    check(lib.rs_decode_batch_masked_bits_dev(codec.handle, C.c_void_p(dev_base), C.c_void_p(dev_bits),
                                              lay.n_stripes, lay.shard_len, lay.shard_stride, lay.stripe_stride,
                                              C.c_void_p(dev_bad or None), h))


def presence_bits(present) -> np.ndarray:
    """(n_stripes, k+m) presence flags -> uint32 bitmask per stripe (bit i = shard i)."""
    p = np.asarray(present, dtype=bool)
    return (p.astype(np.uint32) << np.arange(p.shape[1], dtype=np.uint32)).sum(axis=1, dtype=np.uint32)


def verify(codec: ReedSolomon, dev_base: int, lay: StripeLayout, dev_flag: int, stream=None) -> None:
    lay = _kernel_layout(lay)
    check(_lib.load().rs_verify_batch_dev(codec.handle, C.c_void_p(dev_base), lay.n_stripes, lay.shard_len,
                                          lay.shard_stride, lay.stripe_stride, C.c_void_p(dev_flag),
                                          C.c_void_p(_stream_handle(stream))))


def fill_synthetic(dev_base: int, data_shards: int, lay: StripeLayout, seed: int, stripe0: int = 0,
                   stream=None) -> None:
    """Synthetic data shards; for a GranuleLayout the bytes are generated per
    sub-stripe of its view (stripe0 counts whole stripes)."""
    if isinstance(lay, GranuleLayout):
        if (stripe0 * lay.shard_len) % lay.granule:
            raise ValueError("stripe0 must start a granule row")
        stripe0 = stripe0 * lay.shard_len // lay.granule
        lay = lay.view
    check(_lib.load().rs_fill_synthetic_dev(C.c_void_p(dev_base), data_shards, lay.n_stripes, lay.shard_len,
                                            lay.shard_stride, lay.stripe_stride, seed, stripe0,
                                            C.c_void_p(_stream_handle(stream))))


def copy(dst: int, src: int, n: int, stream=None) -> None:
    check(_lib.load().rs_copy_dev(C.c_void_p(dst), C.c_void_p(src), n, C.c_void_p(_stream_handle(stream))))


class DeviceBuffer:
    """HBM for a stripe pool from rs_dev_alloc: one physically contiguous
    range when contiguous=True and the device has one (else hipMalloc memory;
    `.contiguous` says which).  Exposes data_ptr() / numel() / device like the
    torch tensors the other calls here take pointers from; freed by free() or
    when collected."""

    def __init__(self, nbytes: int, contiguous: bool = True):
        import torch
        p, got = C.c_void_p(), C.c_int(0)
        check(_lib.load().rs_dev_alloc(C.byref(p), nbytes, int(contiguous), C.byref(got)))
        self._ptr, self.nbytes, self.contiguous = p.value, nbytes, bool(got.value)
        self.device = torch.device("cuda", torch.cuda.current_device())

    def data_ptr(self) -> int:
        return self._ptr

    @property
    def __cuda_array_interface__(self):
        """Lets torch.as_tensor(buf, device=...) view the pool as uint8 (no copy)."""
        return {"shape": (self.nbytes,), "typestr": "|u1", "data": (self._ptr, False), "version": 2}

    def tensor(self):
        """A torch uint8 tensor aliasing the pool (valid while the pool lives)."""
        import torch
        return torch.as_tensor(self, device=self.device)

    def numel(self) -> int:
        return self.nbytes

    def free(self) -> None:
        if self._ptr:
            check(_lib.load().rs_dev_free(C.c_void_p(self._ptr)))
            self._ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


def device_count() -> int:
    return _lib.load().rs_device_count()


def view_shards(buf: np.ndarray, lay: StripeLayout, total: int) -> np.ndarray:
    """(n_stripes, total, shard_len) shards of a host copy of the batch: a view
    for a StripeLayout, a gathered copy for a GranuleLayout."""
    if isinstance(lay, GranuleLayout):
        S, G = lay.shard_len, lay.granule
        if S >= G:  # (stripe, row in stripe, shard, G)
            v = buf[: lay.nbytes].reshape(lay.n_stripes, S // G, total, G).transpose(0, 2, 1, 3)
        else:       # (row, shard, stripe in row, S)
            v = buf[: lay.nbytes].reshape(lay.rows, total, G // S, S).transpose(0, 2, 1, 3)
        return np.ascontiguousarray(v).reshape(lay.n_stripes, total, S)
    v = buf[: lay.nbytes].reshape(lay.n_stripes, lay.stripe_stride)
    v = v[:, : total * lay.shard_stride].reshape(lay.n_stripes, total, lay.shard_stride)
    return v[:, :, : lay.shard_len]


class HostBuffer:
    """Pinned host memory from rs_host_alloc (page-locked, mapped for the
    device, placed by the calling thread's NUMA policy): shards and files kept
    here are coded in place across the link by the host calls, with no host
    copies.  `.array` is a NumPy uint8 view that keeps the buffer alive (its
    base holds a reference to this object, so `HostBuffer(n).array` and its
    slices stay valid); freed by free() -- after which every view dangles --
    or when the buffer and every view are collected."""

    def __init__(self, nbytes: int):
        import numpy as np
        p = C.c_void_p()
        check(_lib.load().rs_host_alloc(C.byref(p), nbytes))
        self._ptr, self.nbytes = p.value, nbytes
        raw = (C.c_uint8 * max(nbytes, 1)).from_address(p.value)
        raw._owner = self  # the view's base (raw) keeps this buffer from being collected
        self.array = np.frombuffer(raw, dtype=np.uint8)[:nbytes]

    def data_ptr(self) -> int:
        return self._ptr

    def free(self) -> None:
        if self._ptr:
            self.array = None
            check(_lib.load().rs_host_free(C.c_void_p(self._ptr)))
            self._ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass
