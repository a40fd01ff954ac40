"""Multi-GPU sharding and host-side map-shard merge.

Packets are independent units: GPU g of G processes the contiguous range
[g*N/G, (g+1)*N/G) of the global stream with a private copy of every map.
No data-path collective exists; after the batch the host merges the map
shards:
  * array counters     final = initial + sum_g (shard_g - initial), counter by
                       counter at the map's counter width (u64 words by default)
  * hash (additive)    key union, values merged by the same delta rule
  * per-CPU maps       virtual-CPU slots are global ((unit // 64) % ncpu),
                       so per-slot deltas add up the same way
The array rule runs in libbpftime_amd (bpftime_amd_merge_delta).
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


def counter_width(value_size: int, width: int = 0) -> int:
    """The counter width a map's values are merged at: `width` when given,
    else 8 when the value is a whole number of u64 words (the xdp-counter /
    flow / syscount layouts), else 4 for u32 words; other layouts must name
    their width (the map carries no field layout)."""
    if width:
        if width not in (1, 2, 4, 8) or value_size % width:
            raise ValueError(f"counter width {width} does not divide value size {value_size}")
        return width
    for w in (8, 4):
        if value_size % w == 0:
            return w
    raise ValueError(f"value size {value_size}: pass the counter width explicitly")


def merge_array_delta(init: np.ndarray, shards: List[np.ndarray], width: int = 8) -> np.ndarray:
    """final = init + sum(shard - init), counter by counter at `width` bytes,
    via the C++ merge (bpftime_amd_merge_delta)."""
    from ._lib import lib
    init = np.ascontiguousarray(init, dtype=np.uint8)
    acc = init.copy()
    for s in shards:
        s = np.ascontiguousarray(s, dtype=np.uint8)
        if s.nbytes != init.nbytes or init.nbytes % width:
            raise ValueError("shard size mismatch")
        if lib().bpftime_amd_merge_delta(acc.ctypes.data, init.ctypes.data, s.ctypes.data, acc.nbytes, width):
            raise ValueError("merge failed")
    return acc


_DT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def merge_hash_additive(init: Dict[bytes, bytes], shards: List[Dict[bytes, bytes]],
                        max_entries: int, width: int = 0) -> Dict[bytes, bytes]:
    """Key union; values merged by the additive delta rule at the counter
    width (counter_width).  A union larger than max_entries is order
    dependent in the reference (bpftime_hash_map.hpp:153-156) and is rejected."""
    out = dict(init)
    for sh in shards:
        for k, v in sh.items():
            dt = _DT[counter_width(len(v), width)]
            base = init.get(k, bytes(len(v)))
            cur = np.frombuffer(out.get(k, base), dtype=dt)
            delta = np.frombuffer(v, dtype=dt) - np.frombuffer(base, dtype=dt)
            out[k] = (cur + delta).astype(dt).tobytes()
    if len(out) > max_entries:
        raise ValueError(f"merged hash map has {len(out)} keys > max_entries {max_entries}")
    return out


def u64(b: bytes, i: int = 0) -> int:
    return struct.unpack_from("<Q", b, 8 * i)[0]
