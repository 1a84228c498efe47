"""Wire / on-disk chunk formats around the codec.

The reference stores each server's shard as 1000-byte chunk files and moves
shards as protobuf byte lists; nothing here is coded on the host -- these
adapters only name, slice and order bytes so they can go straight to the GPU
decode paths:

  WriteRequest.payload = the k+m shards           reedsolomonfs.proto:17-27, Client.java:307-332
  chunks of a shard (BLOCK_SIZE each)              datatype/NodeHelper.java:12-21
  chunk file name "<filePath>.<version>-<chunkIdx>" datatype/FileMetadataHelper.java:127-147
  chunkIdx of server s, row r = 6*r + s            datatype/FileMetadataHelper.java:72-114 (nodes round-robin)
  read: ValueResponse.chunkDataMap sorted by the int after the last '-', concatenated
                                                   client/Client.java:202-228, chunkserver.proto:31-39
  read: decode + merge + trim                      client/Client.java:235-241
  recovery: chunk group g = chunks 6g..6g+5 of the six servers  MasterImpl.java:794-839
"""
from __future__ import annotations

from typing import Dict, List, Mapping, Optional, Sequence

import numpy as np

from .layout import BLOCK_SIZE, DATA_SHARD_COUNT, PARITY_SHARD_COUNT, TOTAL_SHARD_COUNT, ReedSolomonDecoder


def chunk_file_name(file_path: str, version: int, chunk_idx: int) -> str:
    """FileMetadataHelper.retrieveFileChunkPaths (:127-147)."""
    return f"{file_path}.{version}-{chunk_idx}"


def chunk_index(name: str) -> int:
    """The integer after the last '-' (Client.java:208-212, MasterImpl.java:795-799)."""
    last = name.rfind("-")
    if last == -1 or last >= len(name) - 1:
        raise ValueError(f"The naming of file {name} has some problems")
    return int(name[last + 1:])


def split_shard_to_chunks(shard, block: int = BLOCK_SIZE) -> List[bytes]:
    """NodeHelper.splitShardToChunks: floor(len / block) chunks (a partial tail is dropped)."""
    b = bytes(shard)
    return [b[i * block:(i + 1) * block] for i in range(len(b) // block)]


def server_chunk_files(file_path: str, version: int, server_idx: int, shard,
                       total: int = TOTAL_SHARD_COUNT, block: int = BLOCK_SIZE) -> Dict[str, bytes]:
    """What chunkserver `server_idx` writes for one file version
    (ChunkserverStateMachine.java:277-310): its shard's chunks under chunkIdx 6*r + s."""
    return {chunk_file_name(file_path, version, total * r + server_idx): c
            for r, c in enumerate(split_shard_to_chunks(shard, block))}


def assemble_shard(chunk_data_map: Mapping[str, bytes]) -> bytes:
    """Client.java:206-220: sort by chunk index, concatenate."""
    return b"".join(bytes(chunk_data_map[n]) for n in sorted(chunk_data_map, key=chunk_index))


def write_request_payload(shards: Sequence) -> List[bytes]:
    """WriteRequest.payload: one bytes entry per shard, in shard order (Client.java:312-314)."""
    return [bytes(s) for s in shards]


def read_file(chunk_maps: Sequence[Optional[Mapping[str, bytes]]], file_size: int,
              data_shards: int = DATA_SHARD_COUNT, parity_shards: int = PARITY_SHARD_COUNT,
              block: int = BLOCK_SIZE) -> Optional[bytes]:
    """Client.readRequest after the six RPCs (Client.java:158-242): assemble each
    server's shard, mark empty/failed servers absent, zero-fill them, decode on
    the GPU, merge and trim.  Returns None when no server answered ("File does
    not exist")."""
    total = data_shards + parity_shards
    shards: List[Optional[np.ndarray]] = [None] * total
    present = [False] * total
    n = 0
    for s in range(total):
        m = chunk_maps[s] if s < len(chunk_maps) else None
        if m:
            shards[s] = np.frombuffer(assemble_shard(m), dtype=np.uint8).copy()
            present[s] = True
            n = len(shards[s])
    if n == 0:
        return None
    for s in range(total):
        if shards[s] is None:
            shards[s] = np.zeros(n, dtype=np.uint8)
    return ReedSolomonDecoder(shards, present, n, file_size, data_shards, parity_shards, block).getFileData()


def recover_offline_chunks(chunk_maps: Sequence[Optional[Mapping[str, bytes]]], offline: Sequence[int],
                           file_path_version: str, data_shards: int = DATA_SHARD_COUNT,
                           parity_shards: int = PARITY_SHARD_COUNT, block: int = BLOCK_SIZE) -> Dict[str, bytes]:
    """MasterImpl.recoverOfflineChunkserver (:730-845), batched: every chunk group
    g (chunk indices 6g..6g+5) of `file_path_version` ("<path>.<version>") is one
    stripe of a [group][server][block] device batch; all groups are decoded in one
    masked launch and the offline servers' chunks are returned by file name."""
    import torch
    from .device import StripeLayout
    from .recovery import recover_chunk_groups_dev

    total = data_shards + parity_shards
    if len(offline) > parity_shards:
        raise ValueError("The number of offline chunkservers exceed the maximum number to recover")
    groups = 0
    for s in range(total):
        if s in offline or not chunk_maps[s]:
            continue
        for name in chunk_maps[s]:
            groups = max(groups, chunk_index(name) // total + 1)
    if groups == 0:
        return {}
    stride = (block + 15) // 16 * 16
    # Staged through page-locked host buffers (torch's pinned allocator): the
    # copies are plain DMA, with no pageable copy for the runtime to lock in
    # place.
    host_t = torch.zeros(groups * total * stride, dtype=torch.uint8, pin_memory=True)
    host = host_t.numpy().reshape(groups, total, stride)
    present = np.zeros((groups, total), dtype=bool)
    for s in range(total):
        if s in offline or not chunk_maps[s]:
            continue
        for name, data in chunk_maps[s].items():
            g = chunk_index(name) // total
            host[g, s, :block] = np.frombuffer(bytes(data), dtype=np.uint8)
            present[g, s] = True
    dev = host_t.to("cuda")
    lay = StripeLayout(groups, block, stride, stride * total)
    recover_chunk_groups_dev(dev.data_ptr(), present, lay, torch.cuda.current_stream(), data_shards, parity_shards)
    host_t.copy_(dev)  # synchronous: the recovered chunks are in host_t on return
    out = host
    return {f"{file_path_version}-{g * total + s}": out[g, s, :block].tobytes()
            for g in range(groups) for s in offline}
