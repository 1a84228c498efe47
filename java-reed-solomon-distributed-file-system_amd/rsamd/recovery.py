"""Chunkserver recovery: the reference's per-chunk-group decode, on the GPU.

ChunkserverDiskRecoveryMachine mirrors
server/Chunkserver/ChunkserverDiskRecoveryMachine.java:14-57 one call at a
time (same checks, messages and quirks; decodeMissing runs on the GPU).  The
master drives it once per 6 x 1000-byte chunk group (MasterImpl.java:794-839);
recover_chunk_groups_dev does all of a server's chunk groups in one batched
launch, each group with its own presence pattern (rs_decode_batch_masked_dev),
in the group-major layout [group][server][chunk]; recover_groups_shard_major_dev
takes the layout the master's loop itself implies -- one array per server,
groups back to back -- where a run of groups with one pattern is one long
stripe (rs_decode_groups_shard_major_dev), and recover_groups_shard_major is
the same on host arrays, the form the master holds them in after its reads
(rs_decode_groups_shard_major; NativeReedSolomon.recoverGroupsShardMajor).
"""
from __future__ import annotations

import numpy as np

import ctypes as C

from . import _lib
from .codec import IllegalArgumentException, RS_E_INVALID, RS_E_NOT_ENOUGH, _Buffers, check
from .device import StripeLayout, _stream_handle, decode_masked
from .layout import DATA_SHARD_COUNT, PARITY_SHARD_COUNT, TOTAL_SHARD_COUNT, _codec


class ChunkserverDiskRecoveryMachine:
    """ChunkserverDiskRecoveryMachine.java:14-57."""

    def __init__(self):
        self._data = [None] * TOTAL_SHARD_COUNT
        self._present = [False] * TOTAL_SHARD_COUNT
        self._present_cnt = 0
        self._byte_cnt = 0
        self._rs = _codec(DATA_SHARD_COUNT, PARITY_SHARD_COUNT)

    def addChunkserverDisksData(self, serverIdx: int, chunkserverDiskData) -> None:
        """:22-32 (adding an index twice counts twice, as in the Java)."""
        if serverIdx < 0 or serverIdx >= TOTAL_SHARD_COUNT:
            raise IllegalArgumentException(RS_E_INVALID, "Given server index does not exist")
        data = np.frombuffer(bytes(chunkserverDiskData), dtype=np.uint8)
        if self._byte_cnt != 0 and len(data) != self._byte_cnt:
            raise IllegalArgumentException(RS_E_INVALID, "Number of bytes in different chunkserver disks mismatch")
        self._byte_cnt = len(data)
        self._data[serverIdx] = data.copy()
        self._present[serverIdx] = True
        self._present_cnt += 1

    def recoverChunkserverDiskData(self) -> None:
        """:34-48."""
        if self._present_cnt < DATA_SHARD_COUNT:
            raise IllegalArgumentException(RS_E_NOT_ENOUGH, "There is not enough disk data to perform the recovery")
        if self._byte_cnt == 0:
            raise IllegalArgumentException(RS_E_INVALID, "There is no data to recover")
        if self._present_cnt == TOTAL_SHARD_COUNT:
            return
        for i in range(TOTAL_SHARD_COUNT):
            if not self._present[i]:
                self._data[i] = np.zeros(self._byte_cnt, dtype=np.uint8)
        self._rs.decodeMissing(self._data, self._present, 0, self._byte_cnt)
        for i in range(TOTAL_SHARD_COUNT):
            self._present[i] = True

    def retrieveRecoveredDiskData(self, serverIdx: int) -> bytes:
        """:50-57."""
        if serverIdx < 0 or serverIdx >= TOTAL_SHARD_COUNT:
            raise IllegalArgumentException(RS_E_INVALID, "Given server index does not exist")
        if not self._present[serverIdx]:
            self.recoverChunkserverDiskData()
        return self._data[serverIdx].tobytes()


def recover_chunk_groups_dev(dev_base: int, present, lay: StripeLayout, stream=None,
                             data_shards: int = DATA_SHARD_COUNT, parity_shards: int = PARITY_SHARD_COUNT) -> None:
    """Reconstruct every absent chunk of every chunk group in one batched call.

    The groups are stripes of a [group][server][chunk] device layout (chunk =
    ConfigVariables.BLOCK_SIZE bytes in the DFS); present is (groups, k+m).
    """
    decode_masked(_codec(data_shards, parity_shards), dev_base, present, lay, stream)


def recover_groups_shard_major_dev(dev_base: int, server_stride: int, present, chunk_len: int = 1000, stream=None,
                                   data_shards: int = DATA_SHARD_COUNT,
                                   parity_shards: int = PARITY_SHARD_COUNT) -> None:
    """MasterImpl.recoverOfflineChunkserver (MasterImpl.java:733-743, 794-839)
    over n_groups chunk groups at once, in the master's own layout: chunk g of
    server s at dev_base + s*server_stride + g*chunk_len.  present is
    (n_groups, k+m): group g's servers that answered (the offline set, grown
    where a read failed mid-loop).  Every absent chunk is rebuilt in place, as
    ChunkserverDiskRecoveryMachine.recoverChunkserverDiskData does per group
    (:34-48); each run of groups with one pattern is one launch (past one run per
    128 MiB of the batch, one launch of the per-stripe pattern kernels)."""
    p = np.ascontiguousarray(np.asarray(present, dtype=bool)).view(np.uint8)
    T = data_shards + parity_shards
    if p.ndim != 2 or p.shape[1] != T:
        raise ValueError(f"present must be (n_groups, {T}), got {p.shape}")
    check(_lib.load().rs_decode_groups_shard_major_dev(
        _codec(data_shards, parity_shards).handle, C.c_void_p(dev_base), server_stride, chunk_len, p.shape[0],
        p.ctypes.data_as(_lib.u8p), C.c_void_p(_stream_handle(stream))))


def recover_groups_shard_major(servers, present, chunk_len: int = 1000, data_shards: int = DATA_SHARD_COUNT,
                               parity_shards: int = PARITY_SHARD_COUNT) -> None:
    """MasterImpl.recoverOfflineChunkserver's loop (MasterImpl.java:733-743,
    794-839) on HOST arrays: servers[s] holds server s's chunks of n_groups
    groups back to back (chunk g at byte g*chunk_len; a NumPy uint8 array,
    pageable or from rsamd.device.HostBuffer), present is (n_groups, k+m).
    Every absent chunk is rebuilt in place (ChunkserverDiskRecoveryMachine.java:
    34-48 per group); a run of groups with one pattern is one decodeMissing of
    run-long shards (rs_decode_groups_shard_major)."""
    p = np.ascontiguousarray(np.asarray(present, dtype=bool)).view(np.uint8)
    T = data_shards + parity_shards
    if p.ndim != 2 or p.shape[1] != T:
        raise ValueError(f"present must be (n_groups, {T}), got {p.shape}")
    b = _Buffers(servers)
    check(_lib.load().rs_decode_groups_shard_major(_codec(data_shards, parity_shards).handle, b.ptrs, len(servers),
                                                   b.lens, chunk_len, p.shape[0], p.ctypes.data_as(_lib.u8p)))
