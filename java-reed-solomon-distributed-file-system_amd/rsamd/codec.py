"""Python mirror of the reference codec API over the C-ABI.

Mirrors (paths under /root/reference/src/main/java/edu/cmu/reedsolomon/):
  ReedSolomon.create / getters          ReedSolomon.java:30-78
  ReedSolomon.encodeParity              ReedSolomon.java:90-104
  ReedSolomon.isParityCorrect (x2)      ReedSolomon.java:115-164
  ReedSolomon.decodeMissing             ReedSolomon.java:175-272
  CodingLoop.codeSomeShards / checkSomeShards   CodingLoop.java:79-117
with the same argument meaning, the same in-place mutation of the shard
buffers, and IllegalArgumentException (a ValueError here) carrying the Java
message text.  All coding runs on the GPU through librsamd.so.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _lib

RS_OK = 0
RS_E_WRONG_NSHARDS = -1
RS_E_SIZE_MISMATCH = -2
RS_E_NEG_OFFSET = -3
RS_E_NEG_COUNT = -4
RS_E_TOO_SMALL = -5
RS_E_NOT_ENOUGH = -6
RS_E_TOO_MANY_SHARDS = -7
RS_E_SINGULAR = -8
RS_E_HIP = -9
RS_E_INVALID = -10
RS_E_TEMP_TOO_SMALL = -11
RS_E_NO_DEVICE = -12


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException, as thrown by the reference codec."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


class GpuError(RuntimeError):
    """A HIP failure or no visible device (the engine has no CPU path)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


def check(rc: int) -> int:
    if rc < 0:
        msg = _lib.last_error()
        if rc in (RS_E_HIP, RS_E_NO_DEVICE):
            raise GpuError(rc, msg)
        raise IllegalArgumentException(rc, msg)
    return rc


_U8 = np.dtype(np.uint8)


class _Buffers:
    """Pins Python buffers (numpy uint8 arrays, bytearray) as a uint8_t* array.

    Addresses come from the buffer protocol (ctypes ``from_buffer``, ~0.4 us
    an array) rather than ``ndarray.ctypes`` (~2 us: it builds a ctypes helper
    object per array), so a small call's marshalling stays a few microseconds
    next to the library's ~11 us."""

    def __init__(self, bufs: Sequence, writable: bool = True):
        self.keep = []
        addrs, lens = [], []
        for b in bufs:
            p, n = self._ptr(b, writable)
            addrs.append(p)
            lens.append(n)
        n = max(1, len(addrs))
        self.lens = (C.c_int64 * n)(*lens)
        # (cast keeps the address array alive; ptrs[i] is a uint8_t*)
        self.ptrs = C.cast((C.c_void_p * n)(*addrs), _lib.u8pp)

    def _ptr(self, b, writable):
        if b is None:
            return None, 0
        if isinstance(b, np.ndarray):
            if b.dtype != _U8 or b.ndim != 1 or not b.flags.c_contiguous:
                raise TypeError("shards must be 1-D contiguous uint8 arrays")
            w = b.flags.writeable
            if writable and not w:
                raise TypeError("shard array is read-only")
            n = b.shape[0]
            if n and w:
                v = C.c_char.from_buffer(b)  # (holds the array)
                self.keep.append(v)
                return C.addressof(v), n
            self.keep.append(b)
            return b.__array_interface__["data"][0], n
        if isinstance(b, bytearray):
            arr = (C.c_uint8 * len(b)).from_buffer(b) if len(b) else (C.c_uint8 * 1)()
            self.keep.append(arr)
            return C.addressof(arr), len(b)
        if isinstance(b, (bytes, memoryview)) and not writable:
            a = np.frombuffer(b, dtype=np.uint8)
            self.keep.append(a)
            return a.__array_interface__["data"][0], a.shape[0]
        raise TypeError(f"unsupported shard buffer type {type(b).__name__}")


def _bools(flags: Sequence) -> np.ndarray:
    return np.array([1 if f else 0 for f in flags], dtype=np.uint8)


def _flag_array(flags: Sequence):
    """The flags as a ctypes uint8_t array (passes as a uint8_t*; ~1 us
    against ~4 us through a numpy array's ctypes pointer)."""
    return (C.c_uint8 * max(1, len(flags)))(*[1 if f else 0 for f in flags])


class ReedSolomon:
    """ReedSolomon.java on the GPU.  Thread-safe; share one instance like the
    reference's ``private static final ReedSolomon REED_SOLOMON``."""

    def __init__(self, data_shard_count: int, parity_shard_count: int):
        h = C.c_void_p()
        check(_lib.load().rs_codec_create(data_shard_count, parity_shard_count, C.byref(h)))
        self._h = h

    @classmethod
    def create(cls, data_shard_count: int, parity_shard_count: int) -> "ReedSolomon":
        """ReedSolomon.create (ReedSolomon.java:30-32)."""
        return cls(data_shard_count, parity_shard_count)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            try:
                _lib.load().rs_codec_destroy(h)
            except (TypeError, AttributeError):
                pass  # interpreter shutdown: module globals already torn down

    @property
    def handle(self):
        return self._h

    def getDataShardCount(self) -> int:
        return _lib.load().rs_codec_data_shard_count(self._h)

    def getParityShardCount(self) -> int:
        return _lib.load().rs_codec_parity_shard_count(self._h)

    def getTotalShardCount(self) -> int:
        return _lib.load().rs_codec_total_shard_count(self._h)

    def matrix(self) -> np.ndarray:
        t, k = self.getTotalShardCount(), self.getDataShardCount()
        out = np.zeros((t, k), dtype=np.uint8)
        check(_lib.load().rs_codec_matrix(self._h, out.ctypes.data_as(_lib.u8p)))
        return out

    def decode_matrix(self, shard_present: Sequence):
        """(survivors, missing, rows) of the fused single-pass decode."""
        t, k = self.getTotalShardCount(), self.getDataShardCount()
        p = _bools(shard_present)
        surv = (C.c_int * k)()
        miss = (C.c_int * t)()
        nm = C.c_int()
        rows = np.zeros((t, k), dtype=np.uint8)
        check(_lib.load().rs_codec_decode_matrix(self._h, p.ctypes.data_as(_lib.u8p), len(p), surv, miss,
                                                 C.byref(nm), rows.ctypes.data_as(_lib.u8p)))
        return list(surv), list(miss)[: nm.value], rows[: nm.value].copy()

    def encodeParity(self, shards: Sequence, offset: int, byteCount: int) -> None:
        """ReedSolomon.encodeParity (ReedSolomon.java:90-104)."""
        b = _Buffers(shards)
        check(_lib.load().rs_encode_parity(self._h, b.ptrs, len(shards), b.lens, offset, byteCount))

    def isParityCorrect(self, shards: Sequence, firstByte: int, byteCount: int, tempBuffer=None) -> bool:
        """ReedSolomon.isParityCorrect (ReedSolomon.java:115-164)."""
        b = _Buffers(shards, writable=False)
        t = _Buffers([tempBuffer], writable=False) if tempBuffer is not None else None
        r = C.c_int(0)
        check(_lib.load().rs_is_parity_correct(self._h, b.ptrs, len(shards), b.lens, firstByte, byteCount,
                                               t.ptrs[0] if t else None, t.lens[0] if t else 0, C.byref(r)))
        return bool(r.value)

    def decodeMissing(self, shards: Sequence, shardPresent: Sequence, offset: int, byteCount: int) -> None:
        """ReedSolomon.decodeMissing (ReedSolomon.java:175-272)."""
        b = _Buffers(shards)
        if len(shardPresent) < len(shards):  # the Java reads shardPresent[i] for every shard index
            raise IndexError("shardPresent shorter than shards")
        check(_lib.load().rs_decode_missing(self._h, b.ptrs, len(shards), b.lens, _flag_array(shardPresent),
                                            offset, byteCount))


def _rows_buffers(matrix_rows, count):
    rows = [np.ascontiguousarray(np.asarray(r, dtype=np.uint8)) for r in list(matrix_rows)[:count]]
    return _Buffers(rows, writable=False)


def codeSomeShards(matrixRows, inputs, inputCount: int, outputs, outputCount: int, offset: int,
                   byteCount: int) -> None:
    """CodingLoop.codeSomeShards (CodingLoop.java:79-85) on the GPU."""
    r = _rows_buffers(matrixRows, outputCount)
    i = _Buffers(list(inputs)[:inputCount], writable=False)
    o = _Buffers(list(outputs)[:outputCount])
    check(_lib.load().rs_code_some_shards(r.ptrs, i.ptrs, inputCount, o.ptrs, outputCount, offset, byteCount))


def checkSomeShards(matrixRows, inputs, inputCount: int, toCheck, checkCount: int, offset: int, byteCount: int,
                    tempBuffer=None) -> bool:
    """CodingLoop.checkSomeShards (CodingLoop.java:110-117) on the GPU."""
    r = _rows_buffers(matrixRows, checkCount)
    i = _Buffers(list(inputs)[:inputCount], writable=False)
    t = _Buffers(list(toCheck)[:checkCount], writable=False)
    res = C.c_int(0)
    check(_lib.load().rs_check_some_shards(r.ptrs, i.ptrs, inputCount, t.ptrs, checkCount, offset, byteCount,
                                           C.byref(res)))
    return bool(res.value)
