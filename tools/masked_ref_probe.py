#!/usr/bin/env python3
"""Row f2's gap, separated on ONE contiguous pool (10+4 x 4 MiB x B):
  masked      product per-stripe-pattern decode, 4 random erasures per stripe
  masked_ref  tools/masked_ref.hip: the same loads and stores, XOR only
  uniform     product decode {0,1,2,3}
  uniform_ref masked_ref with every stripe's bitmask = {0,1,2,3} absent
All with the product's block order for this geometry (3/8-stripe rotation at
<= 256 stripes, none beyond).  Fraction of 8 TB/s, one JSON line per rep; the
product masked decode runs last and the batch is verified after.
Needs tools/bin/libmasked_ref.so (build line in tools/masked_ref.hip).
Usage: python tools/masked_ref_probe.py [stripes] [reps]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import numpy as np
    import torch

    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    ref = C.CDLL(os.path.join(ROOT, "tools", "bin", "libmasked_ref.so"))
    ref.masked_ref_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                      C.c_uint32, C.c_void_p]
    st = torch.cuda.current_stream()
    k, m, S = 10, 4, 4 << 20
    chunks = S // 1024
    rot = 3 * chunks // 8 - 1 if B <= 256 else 0
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
    rdev.fill_synthetic(pool.data_ptr(), k, lay, bench.SEED, 0, st)
    rdev.encode(rs, pool.data_ptr(), lay, st)
    rng = np.random.default_rng(0)
    present = np.ones((B, k + m), dtype=bool)
    for t in range(B):
        present[t, rng.choice(k + m, 4, replace=False)] = False
    bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
    uni_present = np.array([[i >= 4 for i in range(k + m)]] * B)
    ubits = torch.from_numpy(rdev.presence_bits(uni_present).view(np.int32)).to("cuda:0")
    alg = 14 * S * B  # 10 reads + 4 writes per stripe in every leg
    uni = [i >= 4 for i in range(k + m)]

    def launch_ref(b):
        rc = ref.masked_ref_launch(pool.data_ptr(), b.data_ptr(), B, S, lay.shard_stride, lay.stripe_stride, rot,
                                   st.cuda_stream)
        assert rc == 0, rc

    legs = [("uniform", lambda: rdev.decode(rs, pool.data_ptr(), uni, lay, st)),
            ("uniform_ref", lambda: launch_ref(ubits)),
            ("masked_ref", lambda: launch_ref(bits)),
            ("masked", lambda: rdev.decode_masked_bits(rs, pool.data_ptr(), bits.data_ptr(), lay, 0, st))]
    for rep in range(reps):
        out = {"rep": rep, "stripes": B, "rot": rot}
        for name, fn in legs:
            out[name] = round(alg / bench.timed(torch, st, fn, 8) / 8e12, 4)
        print(json.dumps(out), flush=True)
    # the reference wrote XOR into the uniform-pattern shards {0..3}: re-encode, then masked decode, then verify
    rdev.encode(rs, pool.data_ptr(), lay, st)
    rdev.decode_masked_bits(rs, pool.data_ptr(), bits.data_ptr(), lay, 0, st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    rdev.verify(rs, pool.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    pool.free()


if __name__ == "__main__":
    main()
