"""Python mirror of the reference client's file <-> shard layout classes.

  ReedSolomonEncoder(fileData).encode(); getShards(); getPaddedFileSize() ...
  ReedSolomonEncoder(filePath, diskPaths).encode(); store()
      client/ReedSolomonEncoder.java:13-109
  ReedSolomonDecoder(shards, shardPresent, byteCntInShard, fileSize).getFileData()
  ReedSolomonDecoder(filePath, diskPaths, fileSize).decode(); store()
      client/ReedSolomonDecoder.java:13-103
(Java's overloaded constructors are told apart by the type of the first
argument: a path string or os.PathLike selects the disk-file form.)
  constants  ConfigVariables.java:4-9  (BLOCK_SIZE 1000, 4 data + 2 parity)

pad + split + encode (and decode + merge + trim) run on the GPU through
rs_file_encode / rs_file_decode; for k == 4 the split and merge happen inside
the coding kernels.  Device-resident versions: encode_file_dev / decode_file_dev.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

from . import _lib
from .codec import RS_E_INVALID, IllegalArgumentException, ReedSolomon, _bools, _Buffers, _flag_array, check
from .device import _stream_handle

BLOCK_SIZE = 1000         # ConfigVariables.BLOCK_SIZE
DATA_SHARD_COUNT = 4      # ConfigVariables.DATA_SHARD_COUNT
PARITY_SHARD_COUNT = 2    # ConfigVariables.PARITY_SHARD_COUNT
TOTAL_SHARD_COUNT = DATA_SHARD_COUNT + PARITY_SHARD_COUNT
FILE_SIZE_MULTIPLE = DATA_SHARD_COUNT * BLOCK_SIZE

_CODECS: dict = {}


def _codec(k: int, m: int) -> ReedSolomon:
    """One shared codec per shape, like the reference's static final REED_SOLOMON."""
    if (k, m) not in _CODECS:
        _CODECS[(k, m)] = ReedSolomon.create(k, m)
    return _CODECS[(k, m)]


def file_layout(codec: ReedSolomon, file_len: int, block: int = BLOCK_SIZE):
    """(padded_len, shard_len) of ReedSolomonEncoder.pad (ReedSolomonEncoder.java:76-85)."""
    p, s = C.c_int64(), C.c_int64()
    check(_lib.load().rs_file_layout(codec.handle, file_len, block, C.byref(p), C.byref(s)))
    return p.value, s.value


def file_encode_into(codec: ReedSolomon, file_data: np.ndarray, shards_out: Sequence, block: int = BLOCK_SIZE) -> None:
    """rs_file_encode into caller-provided shard buffers (no allocation)."""
    src = _Buffers([file_data if len(file_data) else np.zeros(1, np.uint8)], writable=False)
    b = _Buffers(shards_out)
    check(_lib.load().rs_file_encode(codec.handle, src.ptrs[0], len(file_data), block, b.ptrs, len(shards_out),
                                     b.lens))


def _is_path(x) -> bool:
    return isinstance(x, (str, os.PathLike))


class ReedSolomonEncoder:
    """client/ReedSolomonEncoder.java: ReedSolomonEncoder(byte[] fileData)
    (:27-30), or ReedSolomonEncoder(String filePath, String[] diskPaths)
    (:32-41), which reads the file and names the k+m shard files store()
    writes (:43-54)."""

    def __init__(self, fileData, data_shards=DATA_SHARD_COUNT, parity_shards: int = PARITY_SHARD_COUNT,
                 block: int = BLOCK_SIZE, diskPaths: Sequence = None):
        self._file_path, self._disk_paths = None, None
        if _is_path(fileData):  # (filePath, diskPaths): Files.readAllBytes(Path.of(filePath))
            if not isinstance(data_shards, int):  # diskPaths given positionally, as in the Java
                diskPaths, data_shards = data_shards, DATA_SHARD_COUNT
            self._file_path, self._disk_paths = fileData, list(diskPaths)
            with open(fileData, "rb") as f:
                fileData = f.read()
        self._file = bytes(fileData)
        self._k, self._m, self._block = data_shards, parity_shards, block
        self._shards = None
        self._padded = None

    def encode(self) -> None:
        """pad -> split -> encodeParity (ReedSolomonEncoder.java:56-60), on the GPU."""
        codec = _codec(self._k, self._m)
        padded, S = file_layout(codec, len(self._file), self._block)
        shards = [np.zeros(S, dtype=np.uint8) for _ in range(self._k + self._m)]
        src = np.frombuffer(self._file, dtype=np.uint8) if self._file else np.zeros(1, np.uint8)
        b = _Buffers(shards)
        check(_lib.load().rs_file_encode(codec.handle, src.ctypes.data_as(_lib.u8p), len(self._file), self._block,
                                         b.ptrs, len(shards), b.lens))
        self._shards, self._padded = shards, padded

    def getShards(self):
        return self._shards

    def store(self) -> None:
        """Each shard to its disk path (ReedSolomonEncoder.java:43-54; the Java
        prints and carries on when a write fails)."""
        for path, shard in zip(self._disk_paths, self._shards):
            try:
                with open(path, "wb") as f:
                    f.write(shard.tobytes())
            except OSError as e:
                print(e)

    def getPaddedFileSize(self) -> int:
        return self._padded

    def getFileSize(self) -> int:
        return len(self._file)

    def getFileData(self) -> bytes:
        return self._file

    def getPaddedFileData(self) -> bytes:
        return self._file + bytes(self._padded - len(self._file))

    def getLastChunkIdx(self) -> int:
        """blockCnt - 1 (ReedSolomonEncoder.java:72)."""
        return self._padded // self._block - 1


def file_decode_into(codec: ReedSolomon, shards: Sequence, shardPresent: Sequence, byteCntInShard: int,
                     file_out: np.ndarray, block: int = BLOCK_SIZE) -> None:
    """ReedSolomonDecoder's work into a caller-owned uint8 buffer of fileSize =
    len(file_out) bytes: absent shards filled in place, data merged and trimmed
    (rs_file_decode; no per-call host allocation)."""
    if not (isinstance(file_out, np.ndarray) and file_out.dtype == np.uint8 and file_out.flags.c_contiguous):
        raise TypeError("file_out must be a C-contiguous uint8 numpy array")
    b = _Buffers(shards)
    out = _Buffers([file_out])
    check(_lib.load().rs_file_decode(codec.handle, b.ptrs, len(shards), b.lens, _flag_array(shardPresent),
                                     byteCntInShard, block, out.ptrs[0], len(file_out)))


class ReedSolomonDecoder:
    """client/ReedSolomonDecoder.java.

    ReedSolomonDecoder(shards, shardPresent, byteCntInShard, fileSize) (:33-39)
    decodes at once: decodeMissing fills the absent shards IN PLACE (as the
    Java does), then the data shards are merged and trimmed to fileSize.

    ReedSolomonDecoder(filePath, diskPaths, fileSize) (:41-48) decodes on
    decode() (:70-81): every readable disk file is a present shard
    (retrieveShards, :50-60), the others are zero-filled and rebuilt; store()
    writes the file (:83-90)."""

    def __init__(self, shards, shardPresent, byteCntInShard: int = None, fileSize: int = None,
                 data_shards: int = DATA_SHARD_COUNT, parity_shards: int = PARITY_SHARD_COUNT,
                 block: int = BLOCK_SIZE):
        self._k, self._m, self._block = data_shards, parity_shards, block
        self._data = None
        if _is_path(shards):  # (filePath, diskPaths, fileSize)
            self._file_path, self._disk_paths, self._file_size = shards, list(shardPresent), byteCntInShard
            self._shards, self._present, self._byte_cnt = [None] * len(self._disk_paths), [False] * len(
                self._disk_paths), 0
            return
        self._decode(shards, shardPresent, byteCntInShard, fileSize)

    def _decode(self, shards, shardPresent, byteCntInShard, fileSize):
        codec = _codec(self._k, self._m)
        b = _Buffers(shards)
        p = _bools(shardPresent)
        out = np.zeros(max(1, fileSize), dtype=np.uint8)
        check(_lib.load().rs_file_decode(codec.handle, b.ptrs, len(shards), b.lens, p.ctypes.data_as(_lib.u8p),
                                         byteCntInShard, self._block, out.ctypes.data_as(_lib.u8p), fileSize))
        self._data = out[:fileSize].tobytes()

    def retrieveShards(self) -> None:
        """Read every disk file; a readable one is a present shard and sets
        byteCntInShard (the last one read wins, as in the Java)."""
        for i, path in enumerate(self._disk_paths):
            try:
                with open(path, "rb") as f:
                    self._shards[i] = np.frombuffer(f.read(), dtype=np.uint8).copy()
            except OSError:
                continue
            self._present[i] = True
            self._byte_cnt = len(self._shards[i])

    def decode(self) -> None:
        self.retrieveShards()
        if self._byte_cnt == 0:
            raise IllegalArgumentException(RS_E_INVALID, "There is not enough data to decode")
        for i in range(len(self._shards)):
            if self._shards[i] is None:
                self._shards[i] = np.zeros(self._byte_cnt, dtype=np.uint8)
        self._decode(self._shards, self._present, self._byte_cnt, self._file_size)

    def store(self) -> None:
        """The decoded file to filePath (ReedSolomonDecoder.java:83-90)."""
        try:
            with open(self._file_path, "wb") as f:
                f.write(self._data)
        except OSError as e:
            print(e)

    def getFileData(self) -> bytes:
        return self._data


def encode_file_dev(codec: ReedSolomon, dev_file: int, file_len: int, dev_shards: int, shard_stride: int,
                    block: int = BLOCK_SIZE, stream=None) -> None:
    """Device file -> k+m device shards (rs_file_encode_dev)."""
    check(_lib.load().rs_file_encode_dev(codec.handle, C.c_void_p(dev_file), file_len, block, C.c_void_p(dev_shards),
                                         shard_stride, C.c_void_p(_stream_handle(stream))))


def decode_file_dev(codec: ReedSolomon, dev_shards: int, shard_len: int, shard_stride: int, present: Sequence,
                    dev_file_out: int, file_size: int, block: int = BLOCK_SIZE, write_missing: bool = False,
                    stream=None) -> None:
    """Device survivors -> device file (rs_file_decode_dev)."""
    p = _bools(present)
    check(_lib.load().rs_file_decode_dev(codec.handle, C.c_void_p(dev_shards), shard_len, shard_stride,
                                         p.ctypes.data_as(_lib.u8p), block, C.c_void_p(dev_file_out), file_size,
                                         1 if write_missing else 0, C.c_void_p(_stream_handle(stream))))
