"""ctypes loader for oracle/build/librs_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It wraps the C restatement in rs_oracle.c (see its header for the
reference file:line map).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "librs_oracle.so")
_lib = None

u8p = C.POINTER(C.c_uint8)


def build() -> str:
    """Compile the oracle with its Makefile (gcc only, no GPU)."""
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_init.restype = C.c_int
        L.orc_last_error.restype = C.c_char_p
        L.orc_log_table.restype = C.POINTER(C.c_int16)
        L.orc_exp_table.restype = u8p
        L.orc_mul_table.restype = u8p
        L.orc_gal_multiply.restype = C.c_uint8
        L.orc_gal_multiply.argtypes = [C.c_uint8, C.c_uint8]
        L.orc_gal_divide.restype = C.c_int
        L.orc_gal_divide.argtypes = [C.c_uint8, C.c_uint8]
        L.orc_gal_exp.restype = C.c_uint8
        L.orc_gal_exp.argtypes = [C.c_uint8, C.c_int]
        L.orc_build_matrix.argtypes = [C.c_int, C.c_int, u8p]
        L.orc_matrix_invert.argtypes = [u8p, C.c_int, u8p]
        L.orc_codec_create.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        L.orc_codec_destroy.argtypes = [C.c_void_p]
        L.orc_codec_matrix.restype = u8p
        L.orc_codec_matrix.argtypes = [C.c_void_p]
        L.orc_code_some_shards.argtypes = [C.c_int, C.POINTER(u8p), C.POINTER(u8p), C.c_int,
                                           C.POINTER(u8p), C.c_int, C.c_long, C.c_long]
        L.orc_check_some_shards.argtypes = [C.POINTER(u8p), C.POINTER(u8p), C.c_int, C.POINTER(u8p),
                                            C.c_int, C.c_long, C.c_long, u8p]
        L.orc_encode_parity.argtypes = [C.c_void_p, C.POINTER(u8p), C.c_int, C.POINTER(C.c_long),
                                        C.c_long, C.c_long]
        L.orc_decode_missing.argtypes = [C.c_void_p, C.POINTER(u8p), C.c_int, C.POINTER(C.c_long),
                                         u8p, C.c_long, C.c_long]
        L.orc_is_parity_correct.argtypes = [C.c_void_p, C.POINTER(u8p), C.c_int, C.POINTER(C.c_long),
                                            C.c_long, C.c_long, u8p, C.c_long, C.POINTER(C.c_int)]
        L.orc_decode_rows.argtypes = [C.c_void_p, u8p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                      C.POINTER(C.c_int), u8p]
        L.orc_padded_size.restype = C.c_long
        L.orc_padded_size.argtypes = [C.c_long, C.c_int, C.c_int]
        L.orc_file_encode.restype = C.c_long
        L.orc_file_encode.argtypes = [C.c_void_p, u8p, C.c_long, C.c_int, u8p]
        L.orc_file_decode.argtypes = [C.c_void_p, u8p, C.c_long, u8p, C.c_int, C.c_long, u8p]
        L.orc_fill_synthetic.argtypes = [u8p, C.c_long, C.c_uint64, C.c_uint64, C.c_long]
        L.orc_code_stripes.argtypes = [C.c_void_p, u8p, C.c_long, C.c_long, C.c_long, C.c_long, u8p, C.c_int]
        L.orc_all_possible_polynomials.argtypes = [C.POINTER(C.c_int)]
        L.orc_init()
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u8p)


def ptr_array(arrs):
    P = (u8p * max(1, len(arrs)))()
    for i, a in enumerate(arrs):
        P[i] = ptr(a)
    return P


class OracleError(ValueError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def _rc(rc: int):
    if rc < 0:
        raise OracleError(rc, lib().orc_last_error().decode())
    return rc


def log_table() -> np.ndarray:
    return np.ctypeslib.as_array(lib().orc_log_table(), shape=(256,)).copy()


def exp_table() -> np.ndarray:
    return np.ctypeslib.as_array(lib().orc_exp_table(), shape=(510,)).copy()


def mul_table() -> np.ndarray:
    return np.ctypeslib.as_array(lib().orc_mul_table(), shape=(256, 256)).copy()


def build_matrix(k: int, total: int) -> np.ndarray:
    out = np.zeros((total, k), dtype=np.uint8)
    _rc(lib().orc_build_matrix(k, total, ptr(out)))
    return out


def matrix_invert(m: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros_like(m)
    _rc(lib().orc_matrix_invert(ptr(m), m.shape[0], ptr(out)))
    return out


def code_some_shards(loop_id: int, rows: np.ndarray, inputs, outputs, offset: int, byte_count: int):
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    R = ptr_array([rows[i] for i in range(rows.shape[0])])
    lib().orc_code_some_shards(loop_id, R, ptr_array(inputs), len(inputs), ptr_array(outputs),
                               len(outputs), offset, byte_count)


def check_some_shards(rows, inputs, to_check, offset, byte_count, temp=None) -> bool:
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    R = ptr_array([rows[i] for i in range(rows.shape[0])])
    return bool(lib().orc_check_some_shards(R, ptr_array(inputs), len(inputs), ptr_array(to_check),
                                            len(to_check), offset, byte_count,
                                            ptr(temp) if temp is not None else None))


class Codec:
    """The C restatement of ReedSolomon.java (loop_id < 0: default loop)."""

    def __init__(self, k: int, m: int, loop_id: int = -1):
        h = C.c_void_p()
        _rc(lib().orc_codec_create(k, m, loop_id, C.byref(h)))
        self.h, self.k, self.m, self.total = h, k, m, k + m

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_codec_destroy(self.h)
            self.h = None

    def matrix(self) -> np.ndarray:
        return np.ctypeslib.as_array(lib().orc_codec_matrix(self.h), shape=(self.total, self.k)).copy()

    @staticmethod
    def _lens(shards):
        return (C.c_long * max(1, len(shards)))(*[len(s) for s in shards])

    def encode_parity(self, shards, offset, byte_count):
        _rc(lib().orc_encode_parity(self.h, ptr_array(shards), len(shards), self._lens(shards), offset, byte_count))

    def decode_missing(self, shards, present, offset, byte_count):
        p = np.array([1 if x else 0 for x in present], dtype=np.uint8)
        _rc(lib().orc_decode_missing(self.h, ptr_array(shards), len(shards), self._lens(shards), ptr(p),
                                     offset, byte_count))

    def is_parity_correct(self, shards, offset, byte_count, temp=None) -> bool:
        r = C.c_int(0)
        _rc(lib().orc_is_parity_correct(self.h, ptr_array(shards), len(shards), self._lens(shards), offset,
                                        byte_count, ptr(temp) if temp is not None else None,
                                        len(temp) if temp is not None else 0, C.byref(r)))
        return bool(r.value)

    def decode_rows(self, present):
        p = np.array([1 if x else 0 for x in present], dtype=np.uint8)
        surv = (C.c_int * self.k)()
        miss = (C.c_int * self.total)()
        nm = C.c_int(0)
        rows = np.zeros((max(1, self.m), self.k), dtype=np.uint8)
        _rc(lib().orc_decode_rows(self.h, ptr(p), surv, miss, C.byref(nm), ptr(rows)))
        return list(surv), list(miss)[: nm.value], rows[: nm.value].copy()

    def file_encode(self, data: bytes, block: int = 1000):
        buf = np.frombuffer(bytes(data), dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        padded = lib().orc_padded_size(len(data), self.k, block)
        S = padded // self.k
        out = np.zeros((self.total, max(S, 1)), dtype=np.uint8)
        S2 = _rc(lib().orc_file_encode(self.h, ptr(buf), len(data), block, ptr(out)))
        assert S2 == S
        return out[:, :S].copy()

    def file_decode(self, shards: np.ndarray, present, file_size: int, block: int = 1000) -> bytes:
        shards = np.ascontiguousarray(shards, dtype=np.uint8).copy()
        p = np.array([1 if x else 0 for x in present], dtype=np.uint8)
        out = np.zeros(max(1, file_size), dtype=np.uint8)
        _rc(lib().orc_file_decode(self.h, ptr(shards), shards.shape[1], ptr(p), block, file_size, ptr(out)))
        return out[:file_size].tobytes()

    def code_stripes(self, base: np.ndarray, n_stripes, S, shard_stride, stripe_stride, present=None, threads=1):
        p = None
        if present is not None:
            pa = np.array([1 if x else 0 for x in present], dtype=np.uint8)
            p = ptr(pa)
        _rc(lib().orc_code_stripes(self.h, ptr(base), n_stripes, S, shard_stride, stripe_stride, p, threads))


def fill_synthetic(n_bytes: int, seed: int, stripe: int, start_byte: int = 0) -> np.ndarray:
    out = np.zeros(n_bytes, dtype=np.uint8)
    lib().orc_fill_synthetic(ptr(out), n_bytes, seed, stripe, start_byte)
    return out


def synthetic_shards(k: int, S: int, seed: int, stripe: int, granule: int = 0) -> np.ndarray:
    """The k data shards (k x S) that rs_fill_synthetic_dev writes for global
    stripe `stripe`: packed batches generate k*S bytes per stripe; a granule
    batch (rsamd.device.fill_synthetic on a GranuleLayout) generates k*G bytes
    per granule row of its view, row r = (stripe*S + c) // G for column c."""
    if not granule:
        return fill_synthetic(k * S, seed, stripe).reshape(k, S)
    out = np.empty((k, S), dtype=np.uint8)
    c = 0
    while c < S:
        x = stripe * S + c
        r, o = divmod(x, granule)
        n = min(granule - o, S - c)
        row = fill_synthetic(k * granule, seed, r).reshape(k, granule)
        out[:, c:c + n] = row[:, o:o + n]
        c += n
    return out
