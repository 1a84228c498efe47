"""Loads librsamd.so (the C-ABI of include/rs_amd.h) with ctypes.

The library is built in-tree by csrc/Makefile (``__graft_entry__.build()``).
There is no fallback: if the library is missing, importing the binding fails
loudly.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_ROOT, "lib", "librsamd.so")
CSRC = os.path.join(PKG_ROOT, "csrc")

ABI_VERSION = 7  # include/rs_amd.h RS_AMD_ABI_VERSION, which SIGNATURES follows
u8p = C.POINTER(C.c_uint8)
u8pp = C.POINTER(u8p)

# Every exported symbol with (restype, argtypes) -- kept in sync with include/rs_amd.h
# (tests/test_capi_host.py::test_header_symbols_exported parses the header and checks this table).
SIGNATURES = {
    "rs_codec_create": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "rs_codec_destroy": (None, [C.c_void_p]),
    "rs_codec_data_shard_count": (C.c_int, [C.c_void_p]),
    "rs_codec_parity_shard_count": (C.c_int, [C.c_void_p]),
    "rs_codec_total_shard_count": (C.c_int, [C.c_void_p]),
    "rs_codec_matrix": (C.c_int, [C.c_void_p, u8p]),
    "rs_codec_decode_matrix": (C.c_int, [C.c_void_p, u8p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                         C.POINTER(C.c_int), u8p]),
    "rs_abi_version": (C.c_int, []),
    "rs_last_error_message": (C.c_char_p, []),
    "rs_thread_release": (None, []),
    "rs_device_count": (C.c_int, []),
    "rs_encode_parity": (C.c_int, [C.c_void_p, u8pp, C.c_int, C.POINTER(C.c_int64), C.c_int32, C.c_int32]),
    "rs_decode_missing": (C.c_int, [C.c_void_p, u8pp, C.c_int, C.POINTER(C.c_int64), u8p, C.c_int32, C.c_int32]),
    "rs_is_parity_correct": (C.c_int, [C.c_void_p, u8pp, C.c_int, C.POINTER(C.c_int64), C.c_int32, C.c_int32, u8p,
                                       C.c_int64, C.POINTER(C.c_int)]),
    "rs_check_buffers_and_sizes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int64), C.c_int64, C.c_int64]),
    "rs_code_some_shards": (C.c_int, [u8pp, u8pp, C.c_int, u8pp, C.c_int, C.c_int32, C.c_int32]),
    "rs_check_some_shards": (C.c_int, [u8pp, u8pp, C.c_int, u8pp, C.c_int, C.c_int32, C.c_int32,
                                       C.POINTER(C.c_int)]),
    "rs_encode_batch_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                      C.c_void_p]),
    "rs_decode_batch_dev": (C.c_int, [C.c_void_p, C.c_void_p, u8p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                      C.c_void_p]),
    "rs_decode_batch_masked_dev": (C.c_int, [C.c_void_p, C.c_void_p, u8p, C.c_size_t, C.c_size_t, C.c_size_t,
                                             C.c_size_t, C.c_void_p]),
    "rs_decode_batch_masked_bits_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                                  C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p]),
    "rs_decode_granule_masked_dev": (C.c_int, [C.c_void_p, C.c_void_p, u8p, C.c_size_t, C.c_size_t, C.c_size_t,
                                               C.c_void_p]),
    "rs_decode_granule_masked_bits_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                                    C.c_size_t, C.c_void_p, C.c_void_p]),
    "rs_decode_groups_shard_major_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, u8p,
                                                   C.c_void_p]),
    "rs_decode_groups_shard_major": (C.c_int, [C.c_void_p, u8pp, C.c_int, C.POINTER(C.c_int64), C.c_size_t,
                                               C.c_size_t, u8p]),
    "rs_set_relocator": (C.c_int, [C.c_void_p]),
    "rs_shard_stride_recommended": (C.c_size_t, [C.c_int, C.c_size_t]),
    "rs_verify_batch_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                      C.c_void_p, C.c_void_p]),
    "rs_file_layout": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "rs_file_encode": (C.c_int, [C.c_void_p, u8p, C.c_int64, C.c_int32, u8pp, C.c_int, C.POINTER(C.c_int64)]),
    "rs_file_decode": (C.c_int, [C.c_void_p, u8pp, C.c_int, C.POINTER(C.c_int64), u8p, C.c_int32, C.c_int32, u8p,
                                 C.c_int64]),
    "rs_file_encode_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_size_t,
                                     C.c_void_p]),
    "rs_file_decode_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, u8p, C.c_size_t, C.c_void_p,
                                     C.c_size_t, C.c_int, C.c_void_p]),
    "rs_fill_synthetic_dev": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                        C.c_uint64, C.c_uint64, C.c_void_p]),
    "rs_copy_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "rs_granule_recommended": (C.c_size_t, [C.c_int]),
    "rs_granule_copy_shard": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                        C.c_int, C.c_void_p, C.c_int, C.c_void_p]),
    "rs_dev_alloc": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t, C.c_int, C.POINTER(C.c_int)]),
    "rs_dev_free": (C.c_int, [C.c_void_p]),
    "rs_host_alloc": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    "rs_host_free": (C.c_int, [C.c_void_p]),
}

_lib = None


def load():
    """Return the loaded library (raises OSError if it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 (soname
        # libamdhip64.so.7, loaded by file name "libamdhip64.so").  If torch is
        # loaded first, librsamd's DT_NEEDED libamdhip64.so.7 binds to that same
        # runtime; loaded the other way round the process would get two runtimes
        # and torch would see no GPU.  Without torch, /opt/rocm's runtime is used.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise OSError(f"librsamd.so not built at {LIB_PATH}; run __graft_entry__.build() "
                          f"(make -C {CSRC})")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rs_abi_version() != ABI_VERSION:
            raise OSError(f"{LIB_PATH} has ABI version {lib.rs_abi_version()}; this binding was written for "
                          f"{ABI_VERSION} (include/rs_amd.h RS_AMD_ABI_VERSION): rebuild it")
        _lib = lib
    return _lib


def last_error() -> str:
    return load().rs_last_error_message().decode()
