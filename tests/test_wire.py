"""Row f4: wire / on-disk chunk format adapters (rsamd/wire.py).

CPU tests pin the naming and ordering rules to the reference
(FileMetadataHelper.java:127-147, NodeHelper.java:12-21, Client.java:206-220,
MasterImpl.java:795-799); GPU tests run a simulated DFS write -> per-server
chunk files -> read / master recovery through the GPU decode paths.
"""
import os

import numpy as np
import pytest


def test_chunk_names_and_order():
    from rsamd import wire
    assert wire.chunk_file_name("dir/test.txt", 0, 9) == "dir/test.txt.0-9"
    assert wire.chunk_index("test.txt.0-9") == 9
    assert wire.chunk_index("a-b.3-120") == 120  # the LAST '-'
    with pytest.raises(ValueError, match="has some problems"):
        wire.chunk_index("nodash")
    with pytest.raises(ValueError, match="has some problems"):
        wire.chunk_index("trailing-")
    # numeric, not lexicographic, order (Client.java:208-212)
    m = {"f.0-10": b"C", "f.0-4": b"B", "f.0-9": b"X", "f.0-2": b"A"}
    assert wire.assemble_shard(m) == b"ABXC"


def test_split_and_server_files():
    from rsamd import wire
    shard = bytes(range(256)) * 10  # 2560 bytes -> 2 chunks, tail of 560 dropped like the Java
    chunks = wire.split_shard_to_chunks(shard)
    assert [len(c) for c in chunks] == [1000, 1000] and chunks[1] == shard[1000:2000]
    files = wire.server_chunk_files("p", 2, 4, shard)
    assert sorted(files) == ["p.2-10", "p.2-4"]  # chunkIdx = 6*row + server
    assert wire.assemble_shard(files) == shard[:2000]
    assert wire.write_request_payload([b"ab", bytearray(b"c")]) == [b"ab", b"c"]


@pytest.mark.gpu
def test_dfs_write_read_recover_round_trip(gpu, golden_dir):
    from rsamd import wire
    from rsamd.layout import ReedSolomonEncoder
    for data in (open(os.path.join(golden_dir, "reference_test.txt"), "rb").read(),
                 np.random.default_rng(3).integers(0, 256, 1_234_567, dtype=np.uint8).tobytes()):
        enc = ReedSolomonEncoder(data)
        enc.encode()
        disks = [wire.server_chunk_files("test.txt", 0, s, enc.getShards()[s]) for s in range(6)]
        assert wire.read_file(disks, len(data)) == data
        for off in ([0], [5, 0], [2, 3], [4, 5]):
            resp = [None if s in off else disks[s] for s in range(6)]
            assert wire.read_file(resp, len(data)) == data, off
            rec = wire.recover_offline_chunks(resp, off, "test.txt.0")
            assert rec == {n: b for s in off for n, b in disks[s].items()}, off
    assert wire.read_file([None] * 6, 10) is None
