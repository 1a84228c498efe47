"""ctypes binding of the mock JNI environment (tests/jni_mock/mock_env.c over
jni/rs_jni_core.c and librsamd): the Java-array harness of the JNI tests and
of bench.py's JNI and small-call legs.  Test and bench infrastructure only."""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SO = os.path.join(ROOT, "build", "jni_mock", "libmockjni.so")
P = C.c_void_p

SIGNATURES = [
    ("mock_new_bytes", P, [C.c_int]), ("mock_new_bools", P, [C.c_int]), ("mock_new_objects", P, [C.c_int]),
    ("mock_set", None, [P, C.c_int, P]), ("mock_data", P, [P]), ("mock_reset", None, []),
    ("mock_fail_critical", None, [C.c_int]), ("mock_force_copy", None, [C.c_int]),
    ("mock_moving", None, [C.c_int]), ("mock_moves", C.c_longlong, []), ("mock_hugepages", None, [C.c_int]),
    ("mock_exc_class", C.c_char_p, []), ("mock_exc_message", C.c_char_p, []),
    ("mock_stats", None, [C.POINTER(C.c_longlong)]),
    ("mock_encode_parity", None, [C.c_int, P, P, C.c_int32, C.c_int32]),
    ("mock_decode_missing", None, [C.c_int, P, P, P, C.c_int32, C.c_int32]),
    ("mock_is_parity_correct", C.c_int, [C.c_int, P, P, C.c_int32, C.c_int32, P]),
    ("mock_code_some_shards", None, [C.c_int, P, P, C.c_int32, P, C.c_int32, C.c_int32, C.c_int32]),
    ("mock_check_some_shards", C.c_int, [C.c_int, P, P, C.c_int32, P, C.c_int32, C.c_int32, C.c_int32]),
    ("mock_recover_groups_shard_major", None, [C.c_int, P, C.c_int64, C.c_int64, C.c_int32, C.c_int64, P, C.c_int64]),
    ("mock_recover_groups_shard_major_host", None, [C.c_int, P, P, C.c_int32, C.c_int32, P]),
    ("mock_recover_groups_shard_major_direct", None, [C.c_int, P, P, C.c_int32, C.c_int32, P]),
    ("mock_shard_major_record", None, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint8), C.c_int]),
    ("mock_shard_major_rc", None, [C.c_int]),
    ("mock_file_encode", None, [C.c_int, P, P, C.c_int32, P]),
    ("mock_file_decode", None, [C.c_int, P, P, P, C.c_int32, C.c_int32, P, C.c_int32]),
    ("mock_file_record", None, [C.POINTER(C.c_int64), C.c_int]),
    ("mock_new_direct", P, [P, C.c_int]), ("mock_host_live", C.c_int, []), ("mock_drop_local", None, []),
    ("mock_alloc_pinned", P, [C.c_int, C.c_int32]), ("mock_free_pinned", None, [C.c_int, P]),
    ("mock_encode_parity_direct", None, [C.c_int, P, P, C.c_int32, C.c_int32]),
    ("mock_decode_missing_direct", None, [C.c_int, P, P, P, C.c_int32, C.c_int32]),
    ("mock_file_encode_direct", None, [C.c_int, P, P, C.c_int32, C.c_int32, P]),
    ("mock_file_decode_direct", None, [C.c_int, P, P, P, C.c_int32, C.c_int32, P, C.c_int32]),
    ("mock_time_jni", C.c_double, [C.c_int, P, P, P, C.c_int32, C.c_int]),
    ("mock_time_capi", C.c_double, [C.c_int, P, P, C.c_int, P, P, C.c_int32, C.c_int]),
    ("mock_time_capi_file", C.c_double, [C.c_int, P, P, C.c_int64, C.c_int32, P, C.c_int, P, P, P, C.c_int]),
]

_lib = None


def build():
    """make -C tests/jni_mock (rebuilds only when a source is newer)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    """The loaded library (built first when missing or stale; librsamd and the
    HIP runtime are loaded before it, as rsamd._lib.load does)."""
    global _lib
    if _lib is None:
        from rsamd import _lib as rs_lib
        rs_lib.load()
        build()
        lib = C.CDLL(SO)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib
