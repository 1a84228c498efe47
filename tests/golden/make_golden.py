"""Generate the committed golden fixtures under tests/golden/.

Every vector is produced by the numpy restatement (oracle/numpy_ref.py) and
asserted equal to the C restatement (oracle/rs_oracle.c) before it is written.
The restatements themselves are pinned by galois_tables.json (literal tables of
Galois.java), the upstream Backblaze 5+5 known-answer vector, and the
reference's round-trip tests (see tests/test_oracle.py).

Outputs:
  rs_4_2_s4096_b8.npz    4+2, 8 stripes x 4096 B (BASELINE config-2 shape, scaled down)
  rs_10_4_s1024_b4.npz   10+4, 4 stripes x 1024 B (config-4 shape, scaled down)
  rs_17_3_s512_b2.npz    17+3, 2 stripes x 512 B (the upstream benchmark shape, CodingLoop.java:20-24)
  rs_ragged.npz          4+2 single stripes at ragged lengths (1, 3, 15, 17, 1000, 4097 B)
  rs_small.json          matrices, decode rows, 5+5 KAT, reference test.txt shard digests
  reference_test.txt     /root/reference/ClientClusterCommTestFiles/Files/test.txt (fixture data)

Synthetic data: stripe t's k*S data bytes are little-endian splitmix64(SEED ^ t)
outputs 1, 2, ... (the same definition as rs_fill_synthetic_dev).
"""
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import c_ref  # noqa: E402
from oracle import numpy_ref as nr  # noqa: E402

SEED = 0x5EED
REF_TXT = "/root/reference/ClientClusterCommTestFiles/Files/test.txt"


def batch(k, m, S, B):
    rs = nr.ReedSolomonRef(k, m)
    cc = c_ref.Codec(k, m)
    out = np.zeros((B, k + m, S), dtype=np.uint8)
    for t in range(B):
        out[t, :k] = nr.synthetic_stripe(SEED, t, k, S)
        assert np.array_equal(out[t, :k].reshape(-1), c_ref.fill_synthetic(k * S, SEED, t))
        sh = [out[t, i] for i in range(k + m)]
        rs.encode_parity(sh, 0, S)
        chk = [out[t, i].copy() for i in range(k + m)]
        for p in range(m):
            chk[k + p][:] = 0
        cc.encode_parity(chk, 0, S)
        assert all(np.array_equal(chk[i], out[t, i]) for i in range(k + m))
    return rs, out


def decode_rows_json(rs, cc, masks):
    res = {}
    for miss in masks:
        present = [i not in miss for i in range(rs.total)]
        surv, missing, rows = rs.decode_rows(present)
        s2, m2, r2 = cc.decode_rows(present)
        assert surv == s2 and missing == m2 and np.array_equal(rows, r2)
        res[",".join(map(str, miss))] = {"survivors": surv, "missing": missing, "rows": rows.tolist()}
    return res


def main():
    rs42, b42 = batch(4, 2, 4096, 8)
    np.savez_compressed(os.path.join(HERE, "rs_4_2_s4096_b8.npz"), shards=b42, matrix=rs42.matrix)
    rs104, b104 = batch(10, 4, 1024, 4)
    np.savez_compressed(os.path.join(HERE, "rs_10_4_s1024_b4.npz"), shards=b104, matrix=rs104.matrix)
    rs173, b173 = batch(17, 3, 512, 2)
    np.savez_compressed(os.path.join(HERE, "rs_17_3_s512_b2.npz"), shards=b173, matrix=rs173.matrix)

    ragged = {}
    for n in (1, 3, 15, 17, 1000, 4097):
        words = nr.splitmix64_words(SEED ^ (0xA000 + n), 1, (4 * n + 7) // 8)
        data = words.view(np.uint8)[: 4 * n].reshape(4, n)
        sh = [data[i].copy() for i in range(4)] + [np.zeros(n, np.uint8) for _ in range(2)]
        rs42.encode_parity(sh, 0, n)
        ragged[f"len_{n}"] = np.stack(sh)
    np.savez_compressed(os.path.join(HERE, "rs_ragged.npz"), **ragged)

    cc42, cc104 = c_ref.Codec(4, 2), c_ref.Codec(10, 4)
    kat_data = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]]
    kat = [np.array(d, np.uint8) for d in kat_data] + [np.zeros(2, np.uint8) for _ in range(5)]
    nr.ReedSolomonRef(5, 5).encode_parity(kat, 0, 2)

    with open(REF_TXT, "rb") as f:
        txt = f.read()
    shutil.copyfile(REF_TXT, os.path.join(HERE, "reference_test.txt"))
    shards = nr.split_file(txt, 4, 2, 1000)
    sh = [shards[i] for i in range(6)]
    rs42.encode_parity(sh, 0, shards.shape[1])
    assert np.array_equal(shards, cc42.file_encode(txt))

    small = {
        "seed": SEED,
        "generator_4_2": rs42.matrix.tolist(),
        "generator_10_4": rs104.matrix.tolist(),
        "generator_17_3_row0": rs173.matrix[17].tolist(),
        "decode_4_2": decode_rows_json(rs42, cc42, [(0,), (0, 1), (0, 5), (2, 3), (4,), (5,), (1, 4)]),
        "decode_10_4": decode_rows_json(rs104, cc104, [(0, 1, 2, 3), (0,), (10, 11, 12, 13), (3, 9, 12)]),
        "kat_5_5": {"data": kat_data, "parity": [s.tolist() for s in kat[5:]],
                    "source": "upstream Backblaze JavaReedSolomon 'one encode' test (not vendored in the reference)"},
        "reference_test_txt": {
            "sha256": hashlib.sha256(txt).hexdigest(),
            "file_size": len(txt),
            "padded_size": nr.padded_size(len(txt)),
            "shard_len": int(shards.shape[1]),
            "shard_sha256": [hashlib.sha256(shards[i].tobytes()).hexdigest() for i in range(6)],
        },
    }
    with open(os.path.join(HERE, "rs_small.json"), "w") as f:
        json.dump(small, f, indent=1)
    print("golden fixtures written")


if __name__ == "__main__":
    main()
