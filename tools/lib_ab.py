#!/usr/bin/env python3
"""A/B of two builds of librsamd.so on the same shapes, one process per build
and repetition (so each build gets a fresh allocation), alternating:
  python tools/lib_ab.py LIB_A LIB_B [reps]
Each child times encode on configs[4] (4+2 x 4 KiB x 1 M stripes), configs[1]
(4+2 x 1 MiB x 4096) and 10+4 x 4 MiB x 128 through the plain C-ABI (ctypes;
no rsamd import, so older builds load too)."""
import ctypes as C
import json
import subprocess
import sys

SHAPES = [("4p2_4KiB_x1M", 4, 2, 4096, 1 << 20), ("4p2_1MiB_x4096", 4, 2, 1 << 20, 4096),
          ("10p4_4MiB_x128", 10, 4, 4 << 20, 128)]


def child(lib_path):
    import torch
    lib = C.CDLL(lib_path)
    P = C.c_void_p
    lib.rs_codec_create.argtypes = [C.c_int, C.c_int, C.POINTER(P)]
    lib.rs_encode_batch_dev.argtypes = [P, P, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, P]
    lib.rs_fill_synthetic_dev.argtypes = [P, C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_uint64,
                                          C.c_uint64, P]
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)
    out = {"lib": lib_path}
    for name, k, m, S, B in SHAPES:
        h = P()
        assert lib.rs_codec_create(k, m, C.byref(h)) == 0
        stride = (S + 255) // 256 * 256
        buf = torch.empty(B * (k + m) * stride, dtype=torch.uint8, device="cuda:0")
        assert lib.rs_fill_synthetic_dev(P(buf.data_ptr()), k, B, S, stride, stride * (k + m), 0x5EED, 0, sp) == 0

        def enc():
            assert lib.rs_encode_batch_dev(h, P(buf.data_ptr()), B, S, stride, stride * (k + m), sp) == 0
        for _ in range(5):
            enc()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            enc()
        e1.record(st)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10 * 1e-3
        out[name] = round((k + m) * S * B / t / 8e12, 4)
        del buf
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2])
    libs, reps = sys.argv[1:3], int(sys.argv[3]) if len(sys.argv) > 3 else 3
    for _ in range(reps):
        for lib in libs:
            subprocess.run([sys.executable, __file__, "--child", lib], check=True)


if __name__ == "__main__":
    main()
