"""Python mirror of the reference client's file <-> shard layout classes.

  ReedSolomonEncoder(fileData).encode(); getShards(); getPaddedFileSize() ...
      client/ReedSolomonEncoder.java:13-109
  ReedSolomonDecoder(shards, shardPresent, byteCntInShard, fileSize).getFileData()
      client/ReedSolomonDecoder.java:13-103
  constants  ConfigVariables.java:4-9  (BLOCK_SIZE 1000, 4 data + 2 parity)

pad + split + encode (and decode + merge + trim) run on the GPU through
rs_file_encode / rs_file_decode; for k == 4 the split and merge happen inside
the coding kernels.  Device-resident versions: encode_file_dev / decode_file_dev.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _lib
from .codec import ReedSolomon, _bools, _Buffers, check
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
    src = file_data if len(file_data) else np.zeros(1, np.uint8)
    b = _Buffers(shards_out)
    check(_lib.load().rs_file_encode(codec.handle, src.ctypes.data_as(_lib.u8p), len(file_data), block, b.ptrs,
                                     len(shards_out), b.lens))


class ReedSolomonEncoder:
    """client/ReedSolomonEncoder.java (the in-memory constructor, :27-30)."""

    def __init__(self, fileData: bytes, data_shards: int = DATA_SHARD_COUNT,
                 parity_shards: int = PARITY_SHARD_COUNT, block: int = BLOCK_SIZE):
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
    p = _bools(shardPresent)
    check(_lib.load().rs_file_decode(codec.handle, b.ptrs, len(shards), b.lens, p.ctypes.data_as(_lib.u8p),
                                     byteCntInShard, block, file_out.ctypes.data_as(_lib.u8p), len(file_out)))


class ReedSolomonDecoder:
    """client/ReedSolomonDecoder.java, the shards constructor (:33-39):
    decodeMissing fills the absent shards IN PLACE (as the Java does), then the
    data shards are merged and trimmed to fileSize."""

    def __init__(self, shards: Sequence, shardPresent: Sequence, byteCntInShard: int, fileSize: int,
                 data_shards: int = DATA_SHARD_COUNT, parity_shards: int = PARITY_SHARD_COUNT,
                 block: int = BLOCK_SIZE):
        codec = _codec(data_shards, parity_shards)
        b = _Buffers(shards)
        p = _bools(shardPresent)
        out = np.zeros(max(1, fileSize), dtype=np.uint8)
        check(_lib.load().rs_file_decode(codec.handle, b.ptrs, len(shards), b.lens, p.ctypes.data_as(_lib.u8p),
                                         byteCntInShard, block, out.ctypes.data_as(_lib.u8p), fileSize))
        self._data = out[:fileSize].tobytes()

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
