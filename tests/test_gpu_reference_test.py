"""The reference's own codec test, mirrored at its full size on the GPU
(src/test/java/edu/cmu/reedsolomonfs/ReedSolomonTest.java:24-110).

setUpFileData (:44-56) writes FILE_SIZE = 200 * MB (MB = 1 000 000) random
bytes to Files/test.txt; setUp (:58-67) encodes it through
ReedSolomonEncoder(FILE_PATH, ALL_DISK_PATHS) and store()s the six disk files;
testBasicEncodingAndDecoding (:69-74) decodes them all back,
testDecodeMissingShards (:76-93) first deletes ParityDiskTwo and DataDiskOne
(the {0, 5} pattern); compareDecodedAndOriginalFile (:95-) stores the decoded
file and compares it with the original on disk.  The Java test's data comes
from an unseeded java.util.Random; here it is seeded.  The encoded shards are
also checked against the oracle.
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB = 1000000
FILE_SIZE = 200 * MB
DISKS = ["DataDiskOne", "DataDiskTwo", "DataDiskThree", "DataDiskFour", "ParityDiskOne", "ParityDiskTwo"]


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    root = tmp_path_factory.mktemp("ReedSolomonTestFiles")
    for d in ("Disks", "Files", "FilesRead"):
        (root / d).mkdir()
    data = np.random.default_rng(200).integers(0, 256, FILE_SIZE, dtype=np.uint8).tobytes()
    (root / "Files" / "test.txt").write_bytes(data)
    return root, data


def _encode_and_store(root):
    from rsamd.layout import ReedSolomonEncoder
    disks = [str(root / "Disks" / f"{n}.txt") for n in DISKS]
    enc = ReedSolomonEncoder(str(root / "Files" / "test.txt"), disks)
    enc.encode()
    enc.store()
    return enc, disks


def test_basic_encoding_and_decoding(gpu, oracle_lib, files):
    from rsamd.layout import ReedSolomonDecoder
    root, data = files
    enc, disks = _encode_and_store(root)
    shards = enc.getShards()
    assert [os.path.getsize(p) for p in disks] == [FILE_SIZE // 4] * 6  # 200 MB is a multiple of 4000
    # parity against the oracle on a slice of block rows (the full 200 MB on the
    # scalar oracle would take minutes); every data byte is checked by the round trip
    rows = slice(0, 1000 * 1000)
    ref = [s[rows].copy() for s in shards]
    for p in (4, 5):
        ref[p][:] = 0
    oracle_lib.Codec(4, 2).encode_parity(ref, 0, len(ref[0]))
    assert all(np.array_equal(a[rows], b) for a, b in zip(shards, ref))
    dec = ReedSolomonDecoder(str(root / "FilesRead" / "test.txt"), disks, FILE_SIZE)
    dec.decode()
    assert enc.getFileData() == dec.getFileData()


def test_decode_missing_shards(gpu, files):
    from rsamd.layout import ReedSolomonDecoder
    root, data = files
    enc, disks = _encode_and_store(root)
    digests = [hashlib.sha256(s.tobytes()).hexdigest() for s in enc.getShards()]
    for name in ("ParityDiskTwo", "DataDiskOne"):  # ReedSolomonTest.java:78-80
        os.remove(root / "Disks" / f"{name}.txt")
    dec = ReedSolomonDecoder(str(root / "FilesRead" / "test.txt"), disks, FILE_SIZE)
    dec.decode()
    assert enc.getFileData() == dec.getFileData()
    # compareDecodedAndOriginalFile: store, then compare the files on disk
    dec.store()
    assert (root / "FilesRead" / "test.txt").read_bytes() == (root / "Files" / "test.txt").read_bytes()
    # decodeMissing rebuilt the two absent shards in the decoder's arrays too
    assert [hashlib.sha256(s.tobytes()).hexdigest() for s in dec._shards] == digests
