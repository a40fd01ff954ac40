"""Multi-GPU sharding and host-side map-shard merge.

Packets are independent units: GPU g of G processes the contiguous range
[g*N/G, (g+1)*N/G) of the global stream with a private copy of every map.
No data-path collective exists; after the batch the host merges the map
shards:
  * array counters     final = initial + sum_g (shard_g - initial)   (u64 words)
  * hash (additive)    key union, values merged by the same delta rule
  * per-CPU maps       virtual-CPU slots are global ((unit // 64) % ncpu),
                       so per-slot deltas add up the same way
The array rule runs in libbpftime_amd (bpftime_amd_merge_delta_u64).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """[first, count) of rank's contiguous shard."""
    base, rem = divmod(n_total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def merge_array_delta(init: np.ndarray, shards: List[np.ndarray]) -> np.ndarray:
    """final = init + sum(shard - init) over u64 words, via the C++ merge."""
    from ._lib import lib
    init = np.ascontiguousarray(init, dtype=np.uint8)
    acc = init.copy()
    for s in shards:
        s = np.ascontiguousarray(s, dtype=np.uint8)
        if s.nbytes != init.nbytes or init.nbytes % 8:
            raise ValueError("shard size mismatch")
        if lib().bpftime_amd_merge_delta_u64(acc.ctypes.data, init.ctypes.data, s.ctypes.data, acc.nbytes):
            raise ValueError("merge failed")
    return acc


def merge_hash_additive(init: Dict[bytes, bytes], shards: List[Dict[bytes, bytes]],
                        max_entries: int) -> Dict[bytes, bytes]:
    """Key union; values (u64 words) merged by the additive delta rule.
    A union larger than max_entries is order dependent in the reference
    (bpftime_hash_map.hpp:153-156) and is rejected."""
    out = dict(init)
    for sh in shards:
        for k, v in sh.items():
            base = init.get(k, bytes(len(v)))
            nw = len(v) // 8
            cur = np.frombuffer(out.get(k, base), dtype=np.uint64, count=nw)
            delta = np.frombuffer(v, dtype=np.uint64, count=nw) - np.frombuffer(base, dtype=np.uint64, count=nw)
            merged = (cur + delta).tobytes() + v[nw * 8:]
            out[k] = merged
    if len(out) > max_entries:
        raise ValueError(f"merged hash map has {len(out)} keys > max_entries {max_entries}")
    return out


def u64(b: bytes, i: int = 0) -> int:
    return struct.unpack_from("<Q", b, 8 * i)[0]
