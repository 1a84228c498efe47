"""CPU tests of the disk-file forms of the client layout classes
(rsamd.layout; ReedSolomonEncoder.java:32-54, ReedSolomonDecoder.java:41-90)
that need no GPU: argument handling and the decoder's refusal when no shard
file can be read.  The GPU round trips are in tests/test_gpu_reference_test.py."""
import pytest

from rsamd import IllegalArgumentException
from rsamd.layout import ReedSolomonDecoder, ReedSolomonEncoder


def test_decoder_without_any_disk_file(tmp_path):
    disks = [str(tmp_path / f"disk{i}.txt") for i in range(6)]
    dec = ReedSolomonDecoder(str(tmp_path / "read.txt"), disks, 10)
    with pytest.raises(IllegalArgumentException, match="^There is not enough data to decode$"):
        dec.decode()


def test_encoder_reads_the_file(tmp_path):
    f = tmp_path / "test.txt"
    f.write_bytes(b"test " * 7)
    disks = [str(tmp_path / f"disk{i}.txt") for i in range(6)]
    enc = ReedSolomonEncoder(str(f), disks)
    assert enc.getFileData() == b"test " * 7 and enc.getFileSize() == 35
    enc2 = ReedSolomonEncoder(f, diskPaths=disks)  # os.PathLike works too
    assert enc2.getFileData() == enc.getFileData()
