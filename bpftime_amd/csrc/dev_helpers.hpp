// bpftime_amd: device-side helpers of the interpreter (maps, XDP helpers,
// wave utilities).  Included by interp.hip only.
#pragma once
#include <hip/hip_runtime.h>
#include "common.hpp"

namespace bpftime_amd {

__device__ __forceinline__ bool is_lds_addr(uint64_t a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_is_shared((const void *)a);
#else
  return false;
#endif
}
__device__ __forceinline__ bool is_scratch_addr(uint64_t a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_is_private((const void *)a);
#else
  return false;
#endif
}

typedef uint16_t u16u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint64_t u64u __attribute__((aligned(1)));

// Sized load/store on a flat address (LDS, scratch or global); the size is
// wave-uniform so the switch is a scalar branch.
__device__ __forceinline__ uint64_t mem_load(uint64_t a, uint32_t sz) {
  switch (sz) {
    case 1: return *(const volatile uint8_t *)a;
    case 2: return *(const u16u *)a;
    case 4: return *(const u32u *)a;
    default: return *(const u64u *)a;
  }
}
__device__ __forceinline__ void mem_store(uint64_t a, uint32_t sz, uint64_t v) {
  switch (sz) {
    case 1: *(uint8_t *)a = (uint8_t)v; break;
    case 2: *(u16u *)a = (uint16_t)v; break;
    case 4: *(u32u *)a = (uint32_t)v; break;
    default: *(u64u *)a = v; break;
  }
}

// Global windows a program may access: the batch, the map arena, and the
// lanes' scratch words (PROG_ARRAY lookup copies; C++ tier only -- the asm
// window check leaves those accesses to it).
struct Win {
  uint64_t lo1, hi1, lo2, hi2, lo3, hi3;
  bool checked;
  __device__ __forceinline__ bool ok(uint64_t a, uint32_t sz) const {
    if (!checked) return true;
    if (is_lds_addr(a) || is_scratch_addr(a)) return true;
    uint64_t e = a + sz;
    return (a >= lo1 && e <= hi1 && e >= a) || (a >= lo2 && e <= hi2 && e >= a) ||
           (a >= lo3 && e <= hi3 && e >= a);
  }
};

// ---------------------------------------------------------------------------
// Device maps (helpers 1/2/3).  Semantics follow the reference helper view:
//   array_map.cpp:27-64, fix_hash_map.cpp:27-45 over bpftime_hash_map.hpp,
//   per_cpu_array_map.cpp:34-80, per_cpu_hash_map.cpp:48-107.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t key_hash(uint64_t key, uint32_t ks) {
  // bpftime_hash_map.hpp:40-47: h = h*31 + byte over size_t
  uint64_t h = 0;
  for (uint32_t i = 0; i < ks; i++) h = h * 31 + *(const volatile uint8_t *)(key + i);
  return h;
}

// Hash-table words are shared between workgroups on different XCDs while a
// batch runs: every access is a GLOBAL (address_space(1)) agent-scope atomic
// (sc1), never a flat access (MI355X_MICROARCH.md, inter-workgroup visibility).
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
#define G32(a) ((gu32 *)(uintptr_t)(a))
#define G64(a) ((gu64 *)(uintptr_t)(a))

__device__ __forceinline__ uint32_t ald32(uint64_t a) {
  return __hip_atomic_load(G32(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint8_t ald8(uint64_t a) {
  uint64_t w = a & ~3ull;
  uint32_t v = ald32(w);
  return (uint8_t)(v >> ((a & 3) * 8));
}

// Coherent read: an atomic is performed at the coherence point, so it sees
// every store another XCD has drained, even when this XCD's L2 still holds
// an older copy of the line (an sc1 load is served by the local L2).
__device__ __forceinline__ uint32_t acoh32(uint64_t a) {
  return __hip_atomic_fetch_or(G32(a), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Compare the program-side key (any alignment, any memory) with a slot key
// (8-aligned, published with agent-scope stores).  `coh` selects coherent
// reads: needed when the slot's FILLED state was learned from an atomic
// rather than from a load of the same (line-contained) slot.
__device__ __forceinline__ bool key_eq(uint64_t slot_key, uint64_t key, uint32_t ks, bool coh) {
  uint32_t i = 0;
  for (; i + 4 <= ks; i += 4) {
    uint32_t kv = *(const u32u *)(key + i);
    if ((coh ? acoh32(slot_key + i) : ald32(slot_key + i)) != kv) return false;
  }
  for (; i < ks; i++) {
    uint64_t w = (slot_key + i) & ~3ull;
    uint32_t v = coh ? acoh32(w) : ald32(w);
    if ((uint8_t)(v >> (((slot_key + i) & 3) * 8)) != *(const volatile uint8_t *)(key + i)) return false;
  }
  return true;
}

__device__ __forceinline__ void copy_bytes_publish(uint64_t dst, uint64_t src, uint32_t n) {
  // dst is 8-aligned device memory; src is any flat address.
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4)
    __hip_atomic_store(G32(dst + i), *(const u32u *)(src + i), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (i < n) {
    uint32_t w = 0;
    for (uint32_t j = 0; i + j < n; j++) w |= (uint32_t)(*(const volatile uint8_t *)(src + i + j)) << (8 * j);
    __hip_atomic_store(G32(dst + i), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void copy_bytes(uint64_t dst, uint64_t src, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    *(volatile uint8_t *)(dst + i) = *(const volatile uint8_t *)(src + i);
}

constexpr uint32_t ST_EMPTY = 0, ST_FILLED = 1, ST_BUSY = 2;

__device__ __forceinline__ uint64_t ald64(uint64_t a) {
  return __hip_atomic_load(G64(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// An insert into a table whose lookup index is valid (common.hpp kIxRes),
// holding the index entry `ea` reserved for its key, which is absent: claim
// the first EMPTY bucket of the reference probe from h % nb
// (bpftime_hash_map.hpp:127-180) -- found through the table's bucket bitmap
// (64 buckets per word, a stale bit is only a failed claim), claimed by
// compare-and-swap on its state -- publish key and value, then the index
// entry.  Never waits on another lane: a lane of the same wave that waits on
// the reservation re-reads it on its next loop trip (hash_find_ix).
#ifdef BPFTIME_AMD_INSERT_STATS
// (experiment build only: insert-path counters, tools/insert_stats.py)
__device__ unsigned long long g_istats[8];
#define ISTAT(i, v) atomicAdd(&g_istats[i], (unsigned long long)(v))
#define ISTAT_MAX(i, v) atomicMax(&g_istats[i], (unsigned long long)(v))
#else
#define ISTAT(i, v) ((void)0)
#define ISTAT_MAX(i, v) ((void)0)
#endif
__device__ uint64_t ix_insert(const DMap &m, uint64_t key, uint64_t h, uint64_t ea, uint64_t init,
                              uint32_t init_bytes, bool *inserted, uint64_t part, uint32_t part_off,
                              uint32_t part_bytes) {
  const uint64_t nb = m.nbuckets, bm = ix_bitmap(m.ix, m.ix_mask, m.key_size), nw = (nb + 63) >> 6;
  uint64_t b = h % nb, left = nb;
  uint32_t words = 0;
  while (left) {
    // the next kScan bitmap words at once (one memory round trip for 64 *
    // kScan buckets: the late inserts of a nearly full table scan far), then
    // the first clear bit in probe order
    constexpr uint32_t kScan = 8;
    uint64_t wv[kScan];
    {
      uint64_t w = b >> 6;
#pragma unroll
      for (uint32_t k = 0; k < kScan; k++) {
        wv[k] = ald64(bm + 8 * w);
        w = w + 1 == nw ? 0 : w + 1;
      }
    }
    bool found = false;
#pragma unroll
    for (uint32_t k = 0; k < kScan; k++) {
      if (!left) break;
      words++;
      const uint64_t o = b & 63;
      uint64_t span = 64 - o;
      if (span > left) span = left;
      if (span > nb - b) span = nb - b;
      uint64_t freeb = ~wv[k] >> o;
      if (span < 64) freeb &= (1ull << span) - 1;
      if (freeb) {
        const uint64_t i = (uint64_t)__builtin_ctzll(freeb);
        b += i;
        left -= i;
        found = true;
        break;
      }
      b += span;
      left -= span;
      if (b == nb) b = 0;
    }
    if (!found) continue;
    const uint64_t s = m.data + b * (uint64_t)m.slot_size;
    const uint64_t bit = 1ull << (b & 63);
    uint32_t prev = ST_EMPTY;
    __hip_atomic_compare_exchange_strong(G32(s), &prev, ST_BUSY, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or(G64(bm + 8 * (b >> 6)), bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == ST_EMPTY) {
      // the element count check (bpftime_hash_map.hpp:153-156) by the lane
      // that owns the bucket, as in hash_find
      unsigned long long c = __hip_atomic_fetch_add(G64(m.count_addr), 1ull, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
      if (c >= m.max_entries) {
        __hip_atomic_fetch_add(G64(m.count_addr), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(G32(s), ST_EMPTY, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_and(G64(bm + 8 * (b >> 6)), ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      copy_bytes_publish(s + m.key_off, key, m.key_size);
      if (init)
        copy_bytes_publish(s + m.val_off, init, init_bytes);
      else
        for (uint32_t k = 0; k < init_bytes; k += 4)
          __hip_atomic_store(G32(s + m.val_off + k), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (part) copy_bytes_publish(s + m.val_off + part_off, part, part_bytes);
      // a keyed index (common.hpp ix_key_stride): the key at the entry's
      // position before the entry is published
      // (one 8- or 16-B store: a reader's line holds all of it or none, so a
      // stale key line reads zero, gen_fast.py index_probe)
      if (const uint32_t ks = ix_key_stride(m.key_size)) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t i = 0; i < m.key_size; i++) ((uint8_t *)w)[i] = *(const volatile uint8_t *)(key + i);
        const uint64_t ka = ix_keys(m.ix, m.ix_mask) + (ea - m.ix) / 4 * ks;
        typedef __attribute__((ext_vector_type(2))) uint32_t v2u;
        typedef __attribute__((ext_vector_type(4))) uint32_t v4u;
        if (ks == 8)
          *(__attribute__((address_space(1))) v2u *)(uintptr_t)ka = v2u{w[0], w[1]};
        else
          *(__attribute__((address_space(1))) v4u *)(uintptr_t)ka = v4u{w[0], w[1], w[2], w[3]};
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // key/value stores drained first
      __hip_atomic_store(G32(s), ST_FILLED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(G32(ea), (uint32_t)b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      *inserted = true;
      ISTAT(0, 1);
      ISTAT(1, words);
      ISTAT_MAX(4, words);
      return s;
    }
    ISTAT(2, 1);
    // claimed by another insert: go on after it
    b = b + 1 == nb ? 0 : b + 1;
    left--;
  }
  // full: the reservation goes back (a lane waiting on it tries its own)
  __hip_atomic_store(G32(ea), 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  return 0;
}

// hash_find over a valid lookup index: the index holds exactly the keys the
// reference probe reaches (maps.cpp ix_rebuild; device inserts index what
// they publish), so walking it from ix_pos(h) to an empty entry decides
// presence without the reference probe's walk of a nearly full table (config
// 3: 65,536 flows in 65,537 buckets).  An empty entry is confirmed at the
// coherence point (a line of this XCD's L2 may predate another XCD's
// insert).  An insert reserves the empty entry that proved its key absent
// (0 -> kIxRes): any other insert of the same key walks the same entries and
// waits at the reservation until it holds the new bucket, so two inserts of
// one key meet in one element; lookups pass reserved entries (an insert in
// flight).  Waiting is re-reading on the next loop trip, never a spin inside
// a trip, so a lane never waits on a lane of its own wave.
__device__ uint64_t hash_find_ix(const DMap &m, uint64_t key, uint64_t h, bool insert, uint64_t init,
                                 uint32_t init_bytes, bool *inserted, uint64_t part, uint32_t part_off,
                                 uint32_t part_bytes) {
  uint32_t p = ix_pos(h, m.ix_mask), spins = 0;
  const uint32_t ks = ix_key_stride(m.key_size);
  ISTAT(insert ? 5 : 6, 1);
  for (uint32_t t = 0; t <= m.ix_mask;) {
    ISTAT(7, 1);
    const uint64_t ea = m.ix + 4ull * p;
    uint32_t e = ald32(ea);
    // an empty entry is confirmed at the coherence point; a reservation is
    // polled with loads, confirmed every 16th trip (thousands of lanes may
    // wait on a hot new key's: same-address atomics serialize)
    if (e == 0 || (e == kIxRes && (spins & 15) == 15)) e = acoh32(ea);
    if (e == 0) {
      if (!insert) return 0;
      uint32_t z = 0;
      if (__hip_atomic_compare_exchange_strong(G32(ea), &z, kIxRes, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        return ix_insert(m, key, h, ea, init, init_bytes, inserted, part, part_off, part_bytes);
      e = z;
    }
    if (e == kIxRes) {
      if (insert) {  // maybe this key's: read the entry again on the next trip
        ISTAT(3, 1);
        if (++spins > (1u << 22)) return 0;  // bounded: never hang the GPU
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
    } else if (ks) {
      // a keyed index: the entry's key was published before the entry (read
      // coherently when the entry was: ix_insert)
      if (key_eq(ix_keys(m.ix, m.ix_mask) + (uint64_t)p * ks, key, m.key_size, true))
        return m.data + (uint64_t)(e - 1) * m.slot_size;
    } else {
      const uint64_t s = m.data + (uint64_t)(e - 1) * m.slot_size;
      uint32_t st = ald32(s);
      bool coh = false;
      if (st != ST_FILLED) {
        st = acoh32(s);
        coh = true;
      }
      if (st == ST_FILLED && key_eq(s + m.key_off, key, m.key_size, coh)) return s;
    }
    p = (p + 1) & m.ix_mask;
    t++;
  }
  return 0;
}

// Find `key`; if absent and `insert`, claim a slot and publish key + init
// value (init == 0 -> zero).  Returns slot address or 0.  A table with a
// valid lookup index goes through it (hash_find_ix); the rest of this
// function is the reference probe, for tables without one.  *inserted tells
// whether this lane created the element.  The probe order is the
// reference's: start at hash % nbuckets, linear, wrap once
// (bpftime_hash_map.hpp:127-180).  Lanes never wait on a lane of their own
// wave: a BUSY slot is re-read on the next loop trip, by which time the
// claiming lane (same wave, same trip) has published it.
// (part / part_off / part_bytes: bytes written over the zero-initialised
// value of a new element before it is published -- a per-CPU element's
// value for the inserting lane's CPU, which a lane adding to that CPU's
// slot right after the publish must not see overwritten)
__device__ uint64_t hash_find(const DMap &m, uint64_t key, bool insert, uint64_t init,
                              uint32_t init_bytes, bool *inserted, uint64_t part = 0, uint32_t part_off = 0,
                              uint32_t part_bytes = 0) {
  *inserted = false;
  const uint64_t nb = m.nbuckets;
  const uint64_t h = key_hash(key, m.key_size);
  if (m.ix) return hash_find_ix(m, key, h, insert, init, init_bytes, inserted, part, part_off, part_bytes);
  uint64_t idx = h % nb;
  uint64_t start = idx;
  uint32_t spins = 0;
  for (;;) {
    uint64_t s = m.data + idx * (uint64_t)m.slot_size;
    // A slot never straddles a 128-B line (maps.cpp slot sizing), so a
    // FILLED state read by a load comes with the key bytes of that same
    // line snapshot.  Anything else is confirmed at the coherence point: a
    // stale EMPTY from this XCD's L2 would end the probe with a false miss.
    uint32_t st = ald32(s);
    bool coh = false;
    if (st != ST_FILLED) {
      st = acoh32(s);
      coh = true;
    }
    if (st == ST_EMPTY) {
      if (!insert) return 0;
      uint32_t prev = ST_EMPTY;
      __hip_atomic_compare_exchange_strong(G32(s), &prev, ST_BUSY, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (prev == ST_EMPTY) {
        // Element count check (bpftime_hash_map.hpp:153-156), made only by
        // the lane that owns the slot: reserving before the claim lets
        // thousands of concurrent losers over-count a table that is not full.
        unsigned long long c = __hip_atomic_fetch_add(G64(m.count_addr), 1ull, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
        if (c >= m.max_entries) {
          __hip_atomic_fetch_add(G64(m.count_addr), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(G32(s), ST_EMPTY, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          return 0;
        }
        copy_bytes_publish(s + m.key_off, key, m.key_size);
        if (init)
          copy_bytes_publish(s + m.val_off, init, init_bytes);
        else
          for (uint32_t i = 0; i < init_bytes; i += 4)
            __hip_atomic_store(G32(s + m.val_off + i), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (part) copy_bytes_publish(s + m.val_off + part_off, part, part_bytes);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // key/value stores drained first
        __hip_atomic_store(G32(s), ST_FILLED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        *inserted = true;
        return s;
      }
      st = prev;  // lost the claim: BUSY or FILLED, learned at the coherence point
    }
    if (st == ST_BUSY) {
      if (++spins > (1u << 22)) return 0;  // bounded: never hang the GPU
      __builtin_amdgcn_s_sleep(1);
      continue;  // re-read the same slot on the next trip
    }
    if (key_eq(s + m.key_off, key, m.key_size, coh)) return s;
    idx = idx + 1 == nb ? 0 : idx + 1;
    if (idx == start) return 0;
  }
}

// ---------------------------------------------------------------------------
// LRU hash (runtime/src/bpf_map/userspace/lru_var_hash_map.cpp) over the
// HASH slot layout with tombstones and per-bucket last-use stamps (common.hpp
// DMap, kLruSeqShift).  Every state and key read is made at the coherence
// point: slots change owner within a launch (evictions, deletions, reuse).
//   lookup  (:27-41)  a hit raises the element's stamp (move_to_head)
//   update  (:43-90)  exact flags 0/1/2; an existing key: value + stamp; a new
//                     key claims the first tombstone / empty bucket of its
//                     probe, and past max_entries evicts the smallest stamp:
//                     over every bucket when the batch is ORDERED (the
//                     reference's list tail), over kLruScan buckets from a
//                     hashed start in parallel batches
//   delete  (:92-103) the element becomes a tombstone, ENOENT when absent
// Two parallel inserts of one key converge on one bucket (the first free
// bucket of the same probe), except when a deletion or eviction frees an
// earlier bucket between their probes; the later-probing copy then folds
// itself into the earlier one after publishing (lru_dedup).
// ---------------------------------------------------------------------------
constexpr uint32_t ST_TOMB = 3;

__device__ __forceinline__ uint64_t lru_stamp_at(const DMap &m, uint64_t idx) { return m.count_addr + 128 + 8 * idx; }

__device__ __forceinline__ void lru_touch(const DMap &m, uint64_t idx, uint64_t stamp) {
  __hip_atomic_fetch_max(G64(lru_stamp_at(m, idx)), (unsigned long long)stamp, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}

// the FILLED bucket holding key (-1 absent, -2 gave up on a BUSY bucket);
// *free_idx = the first tombstone or empty bucket of the probe (-1 none)
__device__ int64_t lru_probe(const DMap &m, uint64_t key, int64_t *free_idx, uint32_t *free_st) {
  const uint64_t nb = m.nbuckets;
  uint64_t idx = key_hash(key, m.key_size) % nb;
  const uint64_t start = idx;
  *free_idx = -1;
  *free_st = ST_EMPTY;
  uint32_t spins = 0;
  for (;;) {
    const uint64_t s = m.data + idx * (uint64_t)m.slot_size;
    const uint32_t st = acoh32(s);
    if (st == ST_BUSY) {
      if (++spins > (1u << 22)) return -2;  // bounded: never hang the GPU
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (st == ST_EMPTY || st == ST_TOMB) {
      if (*free_idx < 0) {
        *free_idx = (int64_t)idx;
        *free_st = st;
      }
      if (st == ST_EMPTY) return -1;
    } else if (key_eq(s + m.key_off, key, m.key_size, true)) {
      return (int64_t)idx;
    }
    idx = idx + 1 == nb ? 0 : idx + 1;
    if (idx == start) return -1;
  }
}

__device__ __forceinline__ bool lru_kill(const DMap &m, uint64_t idx) {
  uint32_t prev = ST_FILLED;
  if (!__hip_atomic_compare_exchange_strong(G32(m.data + idx * (uint64_t)m.slot_size), &prev, ST_TOMB,
                                            __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return false;
  __hip_atomic_fetch_add(G64(m.count_addr), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(G64(m.count_addr + 8), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// evict one element: the smallest stamp among the FILLED buckets examined
__device__ bool lru_evict(const DMap &m, uint64_t h, uint64_t stamp, bool exact) {
  const uint64_t nb = m.nbuckets;
  const uint64_t span = exact || nb <= kLruScan ? nb : kLruScan;
  for (uint32_t attempt = 0; attempt < 16; attempt++) {
    const uint64_t start = span == nb ? 0 : ((h ^ (stamp * 0x9E3779B97F4A7C15ull)) + attempt * span) % nb;
    int64_t best = -1;
    uint64_t bs = ~0ull;
    for (uint64_t k = 0, i = start; k < span; k++, i = i + 1 == nb ? 0 : i + 1) {
      if (acoh32(m.data + i * (uint64_t)m.slot_size) != ST_FILLED) continue;
      const uint64_t t = __hip_atomic_load(G64(lru_stamp_at(m, i)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t < bs) {
        bs = t;
        best = (int64_t)i;
      }
    }
    if (best >= 0 && lru_kill(m, (uint64_t)best)) return true;
  }
  return false;
}

// After publishing bucket f for key: another copy of key on the probe
// (possible only when a deletion or eviction freed an earlier bucket between
// two inserts' probes) is resolved by probe position, the earlier copy
// staying.  Each insert scans the whole probe once its own copy is visible,
// so of two copies at least the later-scanning insert sees the other one.
// The dropped copy's value is dropped with it, as if its insert had come
// first and the other one had overwritten it.
__device__ void lru_dedup(const DMap &m, uint64_t key, uint64_t f, uint64_t stamp) {
  const uint64_t nb = m.nbuckets;
  const uint64_t home = key_hash(key, m.key_size) % nb;
  const uint64_t fdist = (f + nb - home) % nb;
  uint64_t idx = home;
  uint32_t spins = 0;
  for (uint64_t k = 0; k < nb;) {
    const uint64_t s = m.data + idx * (uint64_t)m.slot_size;
    const uint32_t st = acoh32(s);
    if (st == ST_BUSY && idx != f) {
      if (++spins > (1u << 22)) return;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (st == ST_EMPTY) return;
    if (idx != f && st == ST_FILLED && key_eq(s + m.key_off, key, m.key_size, true)) {
      if (k < fdist) {  // an earlier copy: this one goes
        if (lru_kill(m, f)) lru_touch(m, idx, stamp);
        return;
      }
      lru_kill(m, idx);  // a later copy goes
    }
    idx = idx + 1 == nb ? 0 : idx + 1;
    k++;
  }
}

__device__ uint64_t lru_lookup(const DMap &m, uint64_t key, uint64_t stamp) {
  int64_t fi;
  uint32_t fst;
  const int64_t idx = lru_probe(m, key, &fi, &fst);
  if (idx < 0) return 0;
  lru_touch(m, (uint64_t)idx, stamp);
  return m.data + (uint64_t)idx * m.slot_size + m.val_off;
}

__device__ uint64_t lru_update(const DMap &m, uint64_t key, uint64_t val, uint64_t flags, uint64_t stamp, bool exact,
                               bool keep_existing) {
  if (flags > 2) return (uint64_t)-1;  // is_good_update_flag (:8-11): EINVAL
  for (uint32_t tries = 0; tries < 64; tries++) {
    int64_t fi;
    uint32_t fst;
    const int64_t idx = lru_probe(m, key, &fi, &fst);
    if (idx == -2) return (uint64_t)-1;
    if (idx >= 0) {
      if (flags == 1) return (uint64_t)-1;  // BPF_NOEXIST: EEXIST
      if (!keep_existing) copy_bytes_publish(m.data + (uint64_t)idx * m.slot_size + m.val_off, val, m.value_size);
      lru_touch(m, (uint64_t)idx, stamp);
      return 0;
    }
    if (flags == 2) return (uint64_t)-1;  // BPF_EXIST: ENOENT
    if (fi < 0) return (uint64_t)-1;      // no free bucket on the probe
    const uint64_t s = m.data + (uint64_t)fi * m.slot_size;
    uint32_t prev = fst;
    if (!__hip_atomic_compare_exchange_strong(G32(s), &prev, ST_BUSY, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT))
      continue;  // the bucket changed under the probe: probe again
    if (fst == ST_TOMB)
      __hip_atomic_fetch_add(G64(m.count_addr + 8), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long c =
        __hip_atomic_fetch_add(G64(m.count_addr), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c >= m.max_entries && !lru_evict(m, key_hash(key, m.key_size), stamp, exact)) {
      // nothing evictable (every element in flight): give the bucket back
      __hip_atomic_fetch_add(G64(m.count_addr), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(G64(m.count_addr + 8), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(G32(s), ST_TOMB, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      return (uint64_t)-1;
    }
    copy_bytes_publish(s + m.key_off, key, m.key_size);
    copy_bytes_publish(s + m.val_off, val, m.value_size);
    __hip_atomic_store(G64(lru_stamp_at(m, (uint64_t)fi)), (unsigned long long)stamp, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // key / value / stamp before the state
    __hip_atomic_store(G32(s), ST_FILLED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (!exact) lru_dedup(m, key, (uint64_t)fi, stamp);
    return 0;
  }
  return (uint64_t)-1;
}

__device__ uint64_t lru_delete(const DMap &m, uint64_t key) {
  int64_t fi;
  uint32_t fst;
  for (uint32_t tries = 0; tries < 64; tries++) {
    const int64_t idx = lru_probe(m, key, &fi, &fst);
    if (idx < 0) return (uint64_t)-1;  // ENOENT
    if (lru_kill(m, (uint64_t)idx)) return 0;
  }
  return (uint64_t)-1;
}

// LPM trie lookup on the device replica: the walk of lpm_trie_map.cpp:
// 192-264 (longest prefix match down the trie, the last non-intermediate
// node on the path wins; an exact full-length match ends the walk).  The
// replica changes during a batch only in ORDERED batches of a program that
// updates / deletes (lpm_update / lpm_remove below).
__device__ __forceinline__ uint32_t lpm_bit(const uint8_t *d, uint32_t i) { return (d[i >> 3] >> (7 - (i & 7))) & 1; }

__device__ uint64_t lpm_lookup(const DMap &m, uint64_t key) {
  const uint32_t dsz = m.key_size - 4, maxp = dsz * 8;
  const uint32_t kp = *(const u32u *)key;
  if (kp > maxp) return 0;
  const uint8_t *kd = (const uint8_t *)(uintptr_t)(key + 4);
  if (m.ix && kp == 32 && dsz == 4) {
    // IPv4 full-length key: the flat table (maps.cpp LpmTrie::flat)
    const uint32_t *t = (const uint32_t *)(uintptr_t)m.ix;
    uint32_t e = t[((uint32_t)kd[0] << 16) | ((uint32_t)kd[1] << 8) | kd[2]];
    if (e & 0x80000000u) e = t[(1u << 24) + 256u * (e & 0x7fffffffu) + kd[3]];
    return e ? m.data + 16 + (uint64_t)(e - 1) * m.slot_size + m.val_off : 0;
  }
  int32_t node = *(const int32_t *)(uintptr_t)m.data;
  uint64_t found = 0;
  for (uint32_t guard = 0; node >= 0 && guard <= maxp + 1; guard++) {
    const uint64_t nb = m.data + 16 + (uint64_t)node * m.slot_size;
    const uint32_t np = *(const uint32_t *)(uintptr_t)nb;
    const bool inter = *(const uint32_t *)(uintptr_t)(nb + 4) != 0;
    const uint8_t *nd = (const uint8_t *)(uintptr_t)(nb + m.key_off);
    const uint32_t lim = np < kp ? np : kp;
    uint32_t ml = 0;
    while (ml + 8 <= lim && nd[ml >> 3] == kd[ml >> 3]) ml += 8;  // whole bytes first
    while (ml < lim && lpm_bit(nd, ml) == lpm_bit(kd, ml)) ml++;
    if (ml == maxp) {
      found = inter ? 0 : nb;
      break;
    }
    if (ml < np) break;
    if (!inter) found = nb;
    if (ml >= kp) break;
    node = *(const int32_t *)(uintptr_t)(nb + 8 + 4 * lpm_bit(kd, np));
  }
  return found ? found + m.val_off : 0;
}

// Program-side LPM trie writes, ORDERED batches only (one lane runs the
// units in order; vm_api.cpp refuses other batches of such programs):
// lpm_trie_map.cpp:266-488 (elem_update) and :490-541 (elem_delete, a
// logical deletion: the node becomes intermediate) restated over the
// replica exactly as the host's LpmTrie::update / remove (maps.cpp) do over
// its node pool -- new nodes appended at index `nodes`, the same numbering,
// so the host takes the replica back as its trie after the batch
// (maps.cpp lpm_pull).  Replica header {i32 root, u32 nodes, u32 entries,
// u32 cap}; a node {u32 plen, u32 intermediate, i32 child[2], data at
// key_off, value at val_off}.  Errors return -1 like the reference helper.
struct LpmHdr {
  int32_t root;
  uint32_t nodes, entries, cap;  // (cap | kLpmPoolOut: an update found the pool full)
};

__device__ __forceinline__ uint32_t lpm_match(const DMap &m, uint64_t nb, const uint8_t *kd, uint32_t kp) {
  const uint32_t np = *(const uint32_t *)(uintptr_t)nb;
  const uint8_t *nd = (const uint8_t *)(uintptr_t)(nb + m.key_off);
  const uint32_t lim = np < kp ? np : kp;
  uint32_t ml = 0;
  while (ml < lim && lpm_bit(nd, ml) == lpm_bit(kd, ml)) ml++;
  return ml;
}

__device__ uint64_t lpm_update(const DMap &m, uint64_t key, uint64_t val, uint64_t flags) {
  if (flags != 0 && flags != 1 && flags != 2) return (uint64_t)-1;  // EINVAL
  const uint32_t dsz = m.key_size - 4, maxp = dsz * 8, vsz = m.value_size;
  const uint32_t kp = *(const u32u *)key;
  if (kp > maxp) return (uint64_t)-1;  // EINVAL
  const uint8_t *kd = (const uint8_t *)(uintptr_t)(key + 4);
  LpmHdr *h = (LpmHdr *)(uintptr_t)m.data;
  auto at = [&](int32_t i) { return m.data + 16 + (uint64_t)i * m.slot_size; };
  auto plen = [&](int32_t i) -> uint32_t & { return *(uint32_t *)(uintptr_t)at(i); };
  auto inter = [&](int32_t i) -> uint32_t & { return *(uint32_t *)(uintptr_t)(at(i) + 4); };
  auto child = [&](int32_t i, uint32_t b) -> int32_t & { return *(int32_t *)(uintptr_t)(at(i) + 8 + 4 * b); };
  auto value = [&](int32_t i) { return at(i) + m.val_off; };
  auto need_room = [&]() {
    if (flags == 2) return false;                    // ENOENT
    if (h->entries >= m.max_entries) return false;   // ENOSPC
    // the replica's node pool (maps.cpp): running out of it is no answer
    // the reference gives (its heap grows), so it is flagged in the
    // header and the host fails the batch (maps.cpp lpm_pull)
    if (h->nodes + 2 <= (h->cap & ~kLpmPoolOut)) return true;
    h->cap |= kLpmPoolOut;
    return false;
  };
  auto make = [&](uint32_t p, bool in) -> int32_t {
    const int32_t i = (int32_t)h->nodes++;
    plen(i) = p;
    inter(i) = in ? 1u : 0u;
    child(i, 0) = child(i, 1) = -1;
    copy_bytes(at(i) + m.key_off, (uint64_t)(uintptr_t)kd, dsz);
    for (uint32_t j = 0; j < vsz; j++) ((uint8_t *)(uintptr_t)value(i))[j] = 0;
    if (!in) copy_bytes(value(i), val, vsz);
    return i;
  };
  if (h->root < 0) {
    if (!need_room()) return (uint64_t)-1;
    h->root = make(kp, false);
    h->entries++;
    return 0;
  }
  int32_t parent = -1, cur = h->root;
  uint32_t pbit = 0, ml = 0;
  while (cur >= 0) {
    ml = lpm_match(m, at(cur), kd, kp);
    const uint32_t np = plen(cur);
    if (np != ml || np == kp || np == maxp) break;
    parent = cur;
    pbit = lpm_bit(kd, np);
    cur = child(cur, pbit);
  }
  auto set_slot = [&](int32_t v) {
    if (parent < 0)
      h->root = v;
    else
      child(parent, pbit) = v;
  };
  auto split = [&](int32_t c) {  // an intermediate node at the split point
    const int32_t nn = make(kp, false);
    const int32_t im = make(ml, true);
    const uint32_t b = lpm_bit(kd, ml);
    child(im, b) = nn;
    child(im, b ^ 1) = c;
    set_slot(im);
    h->entries++;
    return (uint64_t)0;
  };
  if (cur >= 0 && plen(cur) == kp) {  // case 1
    if (lpm_match(m, at(cur), kd, kp) == kp) {
      if (flags == 1) return (uint64_t)-1;               // EEXIST
      if (flags == 2 && inter(cur)) return (uint64_t)-1;  // ENOENT
      if (inter(cur)) {
        if (h->entries >= m.max_entries) return (uint64_t)-1;  // ENOSPC
        inter(cur) = 0;
        h->entries++;
      }
      copy_bytes(value(cur), val, vsz);
      return 0;
    }
    if (!need_room()) return (uint64_t)-1;
    return split(cur);
  }
  if (cur < 0) {  // case 2
    if (!need_room()) return (uint64_t)-1;
    set_slot(make(kp, false));
    h->entries++;
    return 0;
  }
  if (ml == kp) {  // case 3: the new prefix becomes cur's parent
    if (!need_room()) return (uint64_t)-1;
    const int32_t nn = make(kp, false);
    child(nn, lpm_bit((const uint8_t *)(uintptr_t)(at(cur) + m.key_off), ml)) = cur;
    set_slot(nn);
    h->entries++;
    return 0;
  }
  if (!need_room()) return (uint64_t)-1;  // case 4
  return split(cur);
}

__device__ uint64_t lpm_remove(const DMap &m, uint64_t key) {
  const uint32_t dsz = m.key_size - 4;
  const uint32_t kp = *(const u32u *)key;
  if (kp > dsz * 8) return (uint64_t)-1;  // EINVAL
  const uint8_t *kd = (const uint8_t *)(uintptr_t)(key + 4);
  LpmHdr *h = (LpmHdr *)(uintptr_t)m.data;
  auto at = [&](int32_t i) { return m.data + 16 + (uint64_t)i * m.slot_size; };
  int32_t cur = h->root, last = -1;
  while (cur >= 0) {
    last = cur;
    const uint32_t np = *(const uint32_t *)(uintptr_t)at(cur);
    if (np != lpm_match(m, at(cur), kd, kp) || np == kp) break;
    cur = *(const int32_t *)(uintptr_t)(at(cur) + 8 + 4 * lpm_bit(kd, np));
    last = cur;
  }
  if (last < 0) return (uint64_t)-1;  // ENOENT
  const uint64_t nb = at(last);
  uint32_t *in = (uint32_t *)(uintptr_t)(nb + 4);
  if (*(const uint32_t *)(uintptr_t)nb != kp || lpm_match(m, nb, kd, kp) != kp || *in) return (uint64_t)-1;
  *in = 1;
  for (uint32_t j = 0; j < m.value_size; j++) ((uint8_t *)(uintptr_t)(nb + m.val_off))[j] = 0;
  if (h->entries) h->entries--;
  return 0;
}

// ---------------------------------------------------------------------------
// Ring buffer (runtime/src/bpf_map/userspace/ringbuf_map.cpp, helpers
// bpf_helper.cpp:451-504).  Records are [u32 len | BUSY | DISCARD][i32 fd]
// + data, 8-aligned, at data + (pos & mask).  A reservation moves the
// producer position with a CAS after checking room against the consumer
// position, like ringbuf::reserve under its spin lock.  The lanes of a wave
// that reserve from one ring take one CAS for all of them (their records are
// laid out in lane order); a ring too full for the whole wave falls back to
// lane-by-lane reservations, so each reservation succeeds or fails exactly
// as a serial one would at that point.
// ---------------------------------------------------------------------------
constexpr uint32_t RB_BUSY = 0x80000000u, RB_DISCARD = 0x40000000u, RB_HDR = 8;
constexpr uint64_t kRbMaxWaves = 256 * 32;                 // CUs x resident waves per CU (upper bound)
constexpr uint64_t kRbWaveMax = 4096;                      // largest wave reservation on the fast path
constexpr uint64_t kRbSlack = kRbMaxWaves * kRbWaveMax;    // 32 MiB

// Block staging of ring-buffer records.  A block does not move the ring's
// producer position per record (a same-address atomic at the memory side,
// ~40 ns each under the whole chip's contention: it bounded the sampler at
// 1.5 Gpps).  Its first reservation, when the ring has ample room (the fast
// path's condition, counting promises), PROMISES itself kRbStageRec bytes:
// an add to the ring's promise counter (at data + 192), no ring position.
// The block's waves then claim records inside that budget with an LDS
// compare-and-swap on the bytes used, writing them to a per-block staging
// area.  When the block ends it reserves exactly the bytes it used with one
// fetch-and-add of the producer position, copies its records there and
// returns its promise: no ring byte is ever wasted, so a ring that goes from
// ample room to full inside one launch accepts exactly what a serial run
// accepts (the reference's ringbuf::reserve, ringbuf_map.cpp:262-295).
// Every reservation counts the outstanding promises as taken
// (rb_room), so a promised byte is always there at the block's end.  A
// reservation that does not fit while promises are outstanding first closes
// its own block's staging (the block's used bytes are reserved at once, its
// promise returned: a closed block's waves reserve directly) and then waits
// for the other blocks' promises to come back -- they do when those blocks
// end or close; no new promise is made that close to full -- so it fails only
// when the ring is really full, as a serial reservation would.  A wave whose
// records do not fit the block's budget reserves directly.  The consumer,
// bpftime_amd_ringbuf_fetch, synchronizes the device before it reads.
// Consumers see the same records in another parallel order.
// (sizes: common.hpp kRbStage*)
constexpr uint32_t kRbClosed = 0x80000000u;  // RbStage::used: the block's staging is closed
struct RbLds {       // LDS: the block's staging counters
  uint32_t used;     // bytes claimed (| kRbClosed)
  uint32_t nrec;     // records
  int32_t fd;        // the ring of the block's promise (-1 undecided, -3 deciding, -2 none)
  uint32_t pad;
  uint64_t base;     // the ring position of the block's records (set when it closes)
};
// (two pointers, passed by value: a struct the helpers take by reference
// lives in scratch, written by every lane of every launch)
struct RbStage {
  uint8_t *buf = nullptr;  // this block's area: records, then u32 offsets (nullptr: no staging)
  RbLds *lds = nullptr;
};

// the ring's room for a reservation: capacity - (producer - consumer) -
// the bytes blocks have promised themselves (RbStage)
__device__ __forceinline__ int64_t rb_room(const DMap &m, uint64_t *prod_out = nullptr) {
  const uint64_t cons = __hip_atomic_load(G64(m.data), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t prod = __hip_atomic_load(G64(m.data + 128), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t prom = __hip_atomic_load(G64(m.data + 192), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prod_out) *prod_out = prod;
  return (int64_t)m.max_entries - (int64_t)(prod - cons) - (int64_t)prom;
}

// Close the block's staging (a reservation of the block needs the exact
// path): no claim succeeds after this, the bytes claimed so far are
// reserved in the ring now (rb_publish copies them there) and the promise
// is returned.
__device__ void rb_close(const DMap &m, RbStage st) {
  if (!st.buf || st.lds->fd < 0) return;
  const uint32_t u = __hip_atomic_fetch_or(&st.lds->used, kRbClosed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (u & kRbClosed) return;  // (closed by another wave of the block)
  st.lds->base = u ? __hip_atomic_fetch_add(G64(m.data + 128), (uint64_t)u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
               : 0;
  __hip_atomic_fetch_add(G64(m.data + 192), (uint64_t)0 - kRbStageRec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t rb_cas_reserve(const DMap *maps, const DMap &m, uint64_t total, RbStage st,
                                                   int32_t fd) {
  // returns the old producer position, or ~0 if total does not fit.  The
  // loop ends by a successful CAS or a failed room check, as the
  // reference's spin-locked reserve does: the consumer position does not
  // move while a launch runs (its only consumer, bpftime_amd_ringbuf_fetch,
  // synchronizes the device first), every lost CAS means another
  // reservation moved the producer position by >= 8 bytes, and promises
  // only come back.  A room that only the outstanding promises take is
  // waited for, this block's own promise returned first (rb_close) -- on
  // whichever ring it is: a block waiting on ring B while it holds a
  // promise on ring A could otherwise wait for a block that waits on A
  // (ADVICE r04), so no block waits holding a promise.
  uint32_t backoff = 1;
  const uint64_t bound = (uint64_t)m.max_entries / 8 + (1u << 20);
  for (uint64_t spin = 0; spin < bound; spin++) {
    uint64_t p;
    const int64_t room = rb_room(m, &p);
    if (room < (int64_t)total) {
      const uint64_t prom = __hip_atomic_load(G64(m.data + 192), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!prom) return ~0ull;  // full, with nothing promised: the serial answer
      // (a launch without staging waits only)
      if (st.buf) {
        const int32_t pfd = __hip_atomic_load(&st.lds->fd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (pfd >= 0 && pfd < (int32_t)kMaxFds) rb_close(pfd == fd ? m : maps[pfd], st);
      }
    } else {
      unsigned long long e = p;
      if (__hip_atomic_compare_exchange_strong(G64(m.data + 128), &e, p + total, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return p;
    }
    // lost to another wave, or waiting for promises: back off (thousands of
    // waves share these words)
    for (uint32_t i = 0; i < backoff; i++) __builtin_amdgcn_s_sleep(2);
    backoff = backoff < 64 ? 2 * backoff : 64;
  }
  return ~0ull;
}

// The calling lanes that reserve from one ring (rb_reserve groups them).
__device__ uint64_t rb_reserve_ring(const DMap *maps, uint64_t fd, uint64_t size, RbStage st) {
  const bool ok = fd < kMaxFds && maps[fd < kMaxFds ? fd : 0].type == MT_RINGBUF &&
                  !(size & (RB_BUSY | RB_DISCARD));
  const DMap m = maps[ok ? fd : 0];
  const uint64_t total = ok ? (size + RB_HDR + 7) / 8 * 8 : 0;
  const bool fits = ok && total <= m.max_entries;
  // one CAS for the wave when every calling lane reserves from the same ring
  const uint64_t active = __ballot(1);
  const uint32_t me = __lane_id(), leader = (uint32_t)__builtin_ctzll(active);
  const uint64_t lfd = __shfl(fd, leader);
  uint64_t pos = ~0ull;
  if (__ballot(!fits || fd != lfd) == 0) {
    uint64_t before = 0, sum = 0;
    for (uint64_t rest = active; rest; rest &= rest - 1) {
      const uint32_t l = (uint32_t)__builtin_ctzll(rest);
      const uint64_t t = __shfl(total, l);
      if (l < me) before += t;
      sum += t;
    }
    if (st.buf) {
      // block staging (RbStage): the block's first reservation reserves
      // its chunk (a wave arriving while another decides reserves directly)
      int32_t sfd = __shfl(__hip_atomic_load(&st.lds->fd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), leader);
      if (sfd == -1) {
        if (me == leader) {
          int32_t cur = -1;
          if (__hip_atomic_compare_exchange_strong(&st.lds->fd, &cur, -3, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP)) {
            int32_t got = -2;
            // the fast path's condition (below), for a block's budget
            if (m.max_entries >= 2 * kRbSlack && rb_room(m) >= (int64_t)(kRbStageRec + kRbSlack)) {
              __hip_atomic_fetch_add(G64(m.data + 192), (uint64_t)kRbStageRec, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
              got = (int32_t)fd;
            }
            __hip_atomic_store(&st.lds->fd, got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            cur = got;
          }
          sfd = cur;
        }
        sfd = __shfl(sfd, leader);
      }
      if (sfd == (int32_t)fd) {
        uint32_t base = ~0u, rbase = 0;
        const uint32_t cnt = (uint32_t)__builtin_popcountll(active);
        if (me == leader) {
          // claim sum bytes of the budget (a compare-and-swap, so the used
          // count is exactly the claimed bytes: rb_close reserves them)
          uint32_t u = __hip_atomic_load(&st.lds->used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          for (;;) {
            if ((u & kRbClosed) || (uint64_t)u + sum > kRbStageRec) {
              base = ~0u;  // closed, or the budget is spent: direct
              break;
            }
            if (__hip_atomic_compare_exchange_strong(&st.lds->used, &u, u + (uint32_t)sum, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
              base = u;  // (then the record slots fit too: >= 8 B each)
              rbase = __hip_atomic_fetch_add(&st.lds->nrec, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            }
          }
        }
        base = __shfl(base, leader);
        rbase = __shfl(rbase, leader);
        if (base != ~0u) {
          const uint32_t off = base + (uint32_t)before;
          const uint32_t rank = (uint32_t)__builtin_popcountll(active & ((1ull << me) - 1));
          uint8_t *rec = st.buf + off;
          *(uint32_t *)rec = (uint32_t)size | RB_BUSY;
          *(int32_t *)(rec + 4) = (int32_t)fd;
          ((uint32_t *)(st.buf + kRbStageRec))[rbase + rank] = off;
          return (uint64_t)(uintptr_t)(rec + RB_HDR);
        }
      }
    }
    uint64_t base = ~0ull;
    if (me == leader) {
      // Plenty of room: a fetch-and-add (same-address atomics serialize at
      // the memory side, ~12 ns each, while a CAS retry loop under the
      // contention of thousands of waves costs microseconds per record).
      // Safe because at most kRbMaxWaves reservations of <= kRbWaveMax
      // bytes can be between their room check and their add, so an add
      // admitted with kRbSlack bytes to spare never overruns the consumer.
      if (sum <= kRbWaveMax && rb_room(m) >= (int64_t)(sum + kRbSlack))
        base = __hip_atomic_fetch_add(G64(m.data + 128), sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        base = rb_cas_reserve(maps, m, sum, st, (int32_t)fd);
    }
    base = __shfl(base, leader);
    if (base != ~0ull) pos = base + before;
  }
  if (pos == ~0ull && fits) {  // lane by lane (full ring, mixed rings)
    for (uint64_t rest = __ballot(1); rest; rest &= rest - 1)
      if ((uint32_t)__builtin_ctzll(rest) == me) pos = rb_cas_reserve(maps, m, total, st, (int32_t)fd);
  }
  if (pos == ~0ull) return 0;
  const uint64_t mask = m.max_entries - 1, d = m.data + 256;
  __hip_atomic_store(G32(d + (pos & mask)), (uint32_t)size | RB_BUSY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(G32(d + (pos & mask) + 4), (uint32_t)fd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return d + ((pos + RB_HDR) & mask);
}

// bpf_ringbuf_reserve (bpf_helper.cpp:468-474) for the calling lanes: one
// group per distinct ring fd, each reserved the wave way (a wave whose lanes
// write two rings took the lane-by-lane path for all of them: one
// contended compare-and-swap per record)
__device__ uint64_t rb_reserve(const DMap *maps, uint64_t fd, uint64_t size, RbStage st) {
  const uint64_t all = __ballot(1);
  uint64_t done = 0, out = 0;
  while (all & ~done) {
    const uint64_t f0 = __shfl(fd, (uint32_t)__builtin_ctzll(all & ~done));
    if (fd == f0) out = rb_reserve_ring(maps, fd, size, st);
    done |= __ballot(fd == f0);
  }
  return out;
}

// fd < 0: the ring named by the record header's fd, ptr[-1]
// (bpf_helper.cpp:478-479, bpf_ringbuf_submit / _discard); for a record
// whose data wrapped to the ring's first byte that word is the zeroed end of
// the position area, fd 0, as the reference reads the zeroed end of its
// producer page.  bpf_ringbuf_output passes the fd it reserved from
// (bpf_helper.cpp:460-465).
__device__ void rb_submit(const DMap *maps, uint64_t sample, bool discard, RbStage st, int32_t fd = -1) {
  if (st.buf && sample >= (uint64_t)(uintptr_t)st.buf + RB_HDR &&
      sample < (uint64_t)(uintptr_t)st.buf + kRbStageRec) {  // a staged record: published at block end
    uint32_t *h = (uint32_t *)(uintptr_t)(sample - RB_HDR);
    *h = (*h & ~RB_BUSY) | (discard ? RB_DISCARD : 0u);
    return;
  }
  if (fd < 0) fd = *(const int32_t *)(uintptr_t)(sample - 4);
  if (fd < 0 || fd >= (int32_t)kMaxFds) return;
  const DMap m = maps[fd];
  if (m.type != MT_RINGBUF) return;
  const uint64_t mask = m.max_entries - 1, d = m.data + 256;
  const uint64_t hdr = d + ((mask + 1 + (sample - d) - RB_HDR) & mask);
  const uint32_t v = __hip_atomic_load(G32(hdr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the record's bytes before its header
  __hip_atomic_exchange(G32(hdr), (v & ~RB_BUSY) | (discard ? RB_DISCARD : 0u), __ATOMIC_RELEASE,
                        __HIP_MEMORY_SCOPE_AGENT);
}

__device__ uint64_t rb_output(const DMap *maps, uint64_t fd, uint64_t data, uint64_t size, RbStage st) {
  const uint64_t buf = rb_reserve(maps, fd, size, st);
  if (!buf) return (uint64_t)-1;
  copy_bytes(buf, data, (uint32_t)size);
  rb_submit(maps, buf, false, st, (int32_t)fd);
  return 0;
}

// The block's staged records into the ring (every wave of the block is
// done; called by every thread of the block): thread 0 reserves exactly the
// bytes the block used (unless a wave closed the block's staging, which
// reserved them then) and returns the block's promise; then one thread per
// record copies it, with the flags submit / discard gave it.
__device__ void rb_publish(const DMap *maps, RbStage st, uint32_t tid, uint32_t nthreads) {
  if (!st.buf) return;
  const int32_t fd = st.lds->fd;
  if (fd < 0) return;
  const DMap m = maps[fd];
  const uint32_t used = st.lds->used & ~kRbClosed;
  if (tid == 0 && !(st.lds->used & kRbClosed)) {
    st.lds->base = used ? __hip_atomic_fetch_add(G64(m.data + 128), (uint64_t)used, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                    : 0;
    __hip_atomic_fetch_add(G64(m.data + 192), (uint64_t)0 - kRbStageRec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint64_t base = st.lds->base, mask = m.max_entries - 1, d = m.data + 256;
  const uint32_t n = min(st.lds->nrec, kRbStageMaxRec);
  const uint32_t *offs = (const uint32_t *)(st.buf + kRbStageRec);
  for (uint32_t i = tid; i < n; i += nthreads) {
    const uint32_t off = offs[i];
    const uint32_t h = *(const uint32_t *)(st.buf + off);
    const uint32_t total = ((h & ~(RB_BUSY | RB_DISCARD)) + RB_HDR + 7) / 8 * 8;
    const uint64_t *src = (const uint64_t *)(st.buf + off);
    // where a direct reservation puts them (rb_reserve): the header at the
    // position, the data contiguous from the position after it -- at the
    // ring's start when the header takes its last 8 bytes (the ring area is
    // 2 x max_entries bytes, as the reference's is)
    const uint64_t pos = base + off;
    *(uint64_t *)(uintptr_t)(d + (pos & mask)) = src[0];
    uint64_t *dst = (uint64_t *)(uintptr_t)(d + ((pos + RB_HDR) & mask));
    for (uint32_t w = 1; w < total / 8; w++) dst[w - 1] = src[w];
  }
}

struct LaneEnv {
  uint64_t vcpu;
  uint64_t lru_stamp;  // this unit's LRU stamp base (common.hpp kLruSeqShift)
  uint32_t lru_ops;    // LRU operations the unit has made (the stamp's low byte)
  bool exact;          // ORDERED batch: LRU evictions scan every bucket
  uint64_t scratch;  // this lane's scratch word (KParams::lane_scratch), 0 = none
  // last lookup miss (map fd, key hash) for the lookup_or_try_init race rule
  int32_t miss_fd;
  uint64_t miss_hash;
  RbStage rb;        // the block's ring-buffer staging (RbStage)
  // syscall dispatch state of this unit (KParams::sys_state / sys_ret), the
  // bit this batch's phase sets; null outside a dispatch
  uint32_t *ovr_state;
  int64_t *ovr_val;
  uint32_t ovr_bit;
  uint64_t pid_tgid;  // bpf_get_current_pid_tgid's value for this unit
  uint64_t ktime;     // bpf_ktime_get_ns's value for this unit (a replay's recorded clock) ...
  bool kt_on;         // ... when set, else the device clock
};

// bpftime_override_return / bpftime_set_retval (attach/base_attach_impl/
// base_attach_impl.hpp:76-105): the dispatch's return callback records the
// value (syscall_trace_attach_impl.cpp:35-40); with no callback set the
// reference throws, which fails the unit here
__device__ __forceinline__ uint64_t helper_set_retval(uint64_t v, LaneEnv &env, uint32_t *err) {
  if (!env.ovr_state) {
    *err = E_BADOP;
    return 0;
  }
  *env.ovr_state |= env.ovr_bit;
  if (env.ovr_val) *env.ovr_val = (int64_t)v;
  return 0;
}

__device__ __forceinline__ uint64_t lru_next_stamp(LaneEnv &env) {
  const uint32_t op = env.lru_ops < 255 ? env.lru_ops : 255;
  env.lru_ops++;
  return env.lru_stamp | op;
}

// A map's descriptor for a helper call: through the scalar cache when every
// calling lane names the same map (the usual case: an lddw constant), else
// per lane.  The table only changes between launches.
__device__ __forceinline__ DMap load_dmap(const DMap *maps, uint64_t fd) {
  const uint32_t f0 = __builtin_amdgcn_readfirstlane((uint32_t)fd);
  if (__ballot(fd != f0) == 0) {
    typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));
    typedef const u32x4c __attribute__((address_space(4))) *cvec;
    const cvec q = (cvec)(maps + f0);
    const u32x4c w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    DMap m;
    __builtin_memcpy((uint8_t *)&m, &w0, 16);
    __builtin_memcpy((uint8_t *)&m + 16, &w1, 16);
    __builtin_memcpy((uint8_t *)&m + 32, &w2, 16);
    __builtin_memcpy((uint8_t *)&m + 48, &w3, 16);
    return m;
  }
  return maps[fd];
}

__device__ uint64_t helper_lookup(const DMap *maps, uint64_t fd, uint64_t key, LaneEnv &env) {
  if (fd >= kMaxFds) return 0;
  const DMap m = load_dmap(maps, fd);
  switch (m.type) {
    case MT_ARRAY: {
      uint32_t k = *(const u32u *)key;
      if (k >= m.max_entries) return 0;
      return m.data + (uint64_t)k * m.value_size;
    }
    case MT_PERCPU_ARRAY: {
      uint32_t k = *(const u32u *)key;
      if (k >= m.max_entries) return 0;
      return m.data + ((uint64_t)k * m.ncpu + env.vcpu % m.ncpu) * m.value_size;
    }
    case MT_HASH:
    case MT_PERCPU_HASH: {
      bool ins;
      uint64_t s = hash_find(m, key, false, 0, 0, &ins);
      if (!s) {
        env.miss_fd = (int32_t)fd;
        env.miss_hash = key_hash(key, m.key_size);
        return 0;
      }
      uint64_t v = s + m.val_off;
      if (m.type == MT_PERCPU_HASH) v += (env.vcpu % m.ncpu) * m.value_size;
      return v;
    }
    case MT_LPM_TRIE:
      return lpm_lookup(m, key);
    case MT_LRU_HASH: {
      const uint64_t v = lru_lookup(m, key, lru_next_stamp(env));
      if (!v) {
        env.miss_fd = (int32_t)fd;
        env.miss_hash = key_hash(key, m.key_size);
      }
      return v;
    }
    case MT_PROG_ARRAY: {  // prog_array.cpp:113-143: a copy of the slot's prog fd
      const int32_t k = (int32_t)*(const u32u *)key;
      if (k < 0 || (uint32_t)k >= m.max_entries) return 0;
      const int32_t v = *(const volatile int32_t *)(m.data + 4ull * (uint32_t)k);
      if (v < 0) return 0;
      // the copy: this lane's scratch word when the launch has them (the
      // reference's thread-local), else the array's shadow half (maps.cpp);
      // either way a write through the pointer never reaches the array
      const uint64_t c = env.scratch ? env.scratch : m.data + 4ull * m.max_entries + 4ull * (uint32_t)k;
      *(volatile int32_t *)c = v;
      return c;
    }
  }
  return 0;
}

__device__ uint64_t helper_update(const DMap *maps, uint64_t fd, uint64_t key, uint64_t val,
                                  uint64_t flags, LaneEnv &env) {
  if (fd >= kMaxFds) return (uint64_t)-1;
  const DMap m = load_dmap(maps, fd);
  uint64_t base = flags & 0xffffffffull;
  bool flags_ok = base == 0 || base == 1 || base == 2;  // map_common_def.hpp:83-94
  switch (m.type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY: {
      if (!flags_ok) return (uint64_t)-1;
      uint32_t k = *(const u32u *)key;
      if (k < m.max_entries && flags == 1) return (uint64_t)-1;  // EEXIST
      if (k >= m.max_entries) return (uint64_t)-1;               // E2BIG
      uint64_t dst = m.type == MT_ARRAY
                         ? m.data + (uint64_t)k * m.value_size
                         : m.data + ((uint64_t)k * m.ncpu + env.vcpu % m.ncpu) * m.value_size;
      copy_bytes(dst, val, m.value_size);
      return 0;
    }
    case MT_HASH: {
      // fix_hash_map.cpp:34-39: flags ignored, returns 0 even when full.
      bool ins;
      uint32_t vbytes = (m.value_size + 3) & ~3u;
      uint64_t s = hash_find(m, key, true, val, m.value_size, &ins);
      if (s && !ins) {
        // Existing element: overwrite, except in the lookup-miss race (this
        // lane's previous lookup of the same key missed, so in any serial
        // order this update would have created the element): another lane
        // created it first, and overwriting would drop its updates.
        bool race = env.miss_fd == (int32_t)fd && env.miss_hash == key_hash(key, m.key_size);
        if (!race) copy_bytes(s + m.val_off, val, m.value_size);
      }
      (void)vbytes;
      env.miss_fd = -1;
      return 0;
    }
    case MT_PERCPU_HASH: {
      if (!flags_ok) return (uint64_t)-1;
      // per_cpu_hash_map.cpp:66-94: insert zeroed ncpu*vsize, then write
      // the slot (a new element's slot before it is published)
      bool ins;
      const uint32_t off = (uint32_t)(env.vcpu % m.ncpu) * m.value_size;
      uint64_t s = hash_find(m, key, true, 0, m.value_size * m.ncpu, &ins, val, off, m.value_size);
      if (!s) return 0;
      bool race = !ins && env.miss_fd == (int32_t)fd && env.miss_hash == key_hash(key, m.key_size);
      if (!ins && !race) copy_bytes(s + m.val_off + off, val, m.value_size);
      env.miss_fd = -1;
      return 0;
    }
    case MT_LPM_TRIE:
      return env.exact ? lpm_update(m, key, val, flags) : (uint64_t)-1;
    case MT_LRU_HASH: {
      // the lookup-miss race of MT_HASH above: an existing element is not
      // overwritten by the lane whose lookup of the key just missed
      const bool race = env.miss_fd == (int32_t)fd && env.miss_hash == key_hash(key, m.key_size);
      env.miss_fd = -1;
      return lru_update(m, key, val, flags, lru_next_stamp(env), env.exact, race);
    }
  }
  return (uint64_t)-1;
}

__device__ uint64_t helper_delete(const DMap *maps, uint64_t fd, uint64_t key, LaneEnv &env) {
  if (fd >= kMaxFds) return (uint64_t)-1;
  const DMap m = load_dmap(maps, fd);
  switch (m.type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY:
      return (uint64_t)-1;  // EINVAL (array_map.cpp:58-64)
    case MT_HASH: {
      bool ins;
      uint64_t s = hash_find(m, key, false, 0, 0, &ins);
      if (s) {
        uint32_t prev = ST_FILLED;  // no tombstone (bpftime_hash_map.hpp:182-199)
        if (__hip_atomic_compare_exchange_strong(G32(s), &prev, ST_EMPTY, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          __hip_atomic_fetch_add(G64(m.count_addr), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return 0;
    }
    case MT_PERCPU_HASH: {
      // per_cpu_hash_map.cpp:96-107: zeroes [0, cpu*vsize) of the element
      bool ins;
      uint64_t s = hash_find(m, key, false, 0, 0, &ins);
      if (s) {
        uint64_t n = (env.vcpu % m.ncpu) * m.value_size;
        for (uint64_t i = 0; i < n; i++) *(volatile uint8_t *)(s + m.val_off + i) = 0;
      }
      return 0;
    }
    case MT_LRU_HASH:
      return lru_delete(m, key);
    case MT_LPM_TRIE:
      return env.exact ? lpm_remove(m, key) : (uint64_t)-1;
  }
  return (uint64_t)-1;
}

// bpf_helper.cpp:713-744
__device__ uint64_t helper_csum_diff(uint64_t from, uint64_t from_size_, uint64_t to,
                                     uint64_t to_size_, uint64_t seed_) {
  int from_size = (int)from_size_, to_size = (int)to_size_;
  int csum = -22;
  if ((from_size % 4 != 0) || (to_size % 4 != 0)) return (uint64_t)(int64_t)csum;
  csum = (int)seed_;
  if (to)
    for (int i = 0; i < to_size / 2; i++) csum += (uint16_t)(*(const u16u *)(to + 2 * i));
  if (from)
    for (int i = 0; i < from_size / 2; i++) csum += (uint16_t)(~*(const u16u *)(from + 2 * i));
  if (csum < 0) csum = -22;
  return (uint64_t)(int64_t)csum;
}

// xdp_md_userspace (runtime/extension/userspace_xdp.h:6-17)
struct XdpCtx {
  uint64_t data, data_end;
  uint32_t data_meta, ingress_ifindex, rx_queue_index, egress_ifindex;
  uint64_t buffer_start, buffer_end;
};

// bpf_helper.cpp:748-764
__device__ uint64_t helper_adjust_head(uint64_t ctx, uint64_t off_) {
  volatile XdpCtx *x = (volatile XdpCtx *)ctx;
  int offset = (int)off_;
  uint64_t data = x->data + (int64_t)offset;
  if (data > x->data_end - 14 || data > x->buffer_end) return (uint64_t)(int64_t)-22;
  if (data < x->buffer_start) {
    // memmove(buffer_start + (buffer_start - data), data, data_end - data)
    uint64_t dst = x->buffer_start + (x->buffer_start - data), src = x->data;
    uint64_t n = x->data_end - x->data;
    if (dst > src)
      for (uint64_t i = n; i-- > 0;) *(volatile uint8_t *)(dst + i) = *(volatile uint8_t *)(src + i);
    else
      for (uint64_t i = 0; i < n; i++) *(volatile uint8_t *)(dst + i) = *(volatile uint8_t *)(src + i);
    data = x->buffer_start;
  }
  x->data = data;
  return 0;
}

// bpf_helper.cpp:766-776
__device__ uint64_t helper_adjust_tail(uint64_t ctx, uint64_t delta_) {
  volatile XdpCtx *x = (volatile XdpCtx *)ctx;
  int delta = (int)delta_;
  uint64_t data = x->data_end + (int64_t)delta;
  if (data < x->data || data < x->buffer_start || data > x->buffer_end) return (uint64_t)(int64_t)-22;
  x->data_end = data;
  return 0;
}

// bpf_helper.cpp:778-788 (defined in the reference, not registered by default)
__device__ uint64_t helper_xdp_load_bytes(uint64_t ctx, uint64_t off, uint64_t buf, uint64_t len) {
  volatile XdpCtx *x = (volatile XdpCtx *)ctx;
  uint64_t data = x->data + (uint32_t)off;
  if (data + (uint32_t)len > x->data_end) return (uint64_t)(int64_t)-22;
  copy_bytes(buf, data, (uint32_t)len);
  return 0;
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return readlane64(x, 0);
}

// One lane of the wave adds a cached counter delta (wave-uniform arguments).
__device__ __forceinline__ void flush_delta(uint64_t a, uint32_t sz, uint64_t delta) {
  if (a == 0 || delta == 0) return;
  if ((threadIdx.x & 63) == 0) {
    if (sz == 8)
      __hip_atomic_fetch_add((uint64_t *)a, delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_fetch_add((uint32_t *)a, (uint32_t)delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one tagged delta {address | (4-byte ? 1 : 0), delta} (LDS combining
// table entries, the block's combined wave caches)
__device__ __forceinline__ void flush_delta_tag(uint64_t tag, uint64_t delta) {
  if (!tag || !delta) return;
  if (tag & 1)
    __hip_atomic_fetch_add((uint32_t *)(uintptr_t)(tag & ~1ull), (uint32_t)delta, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  else
    __hip_atomic_fetch_add((uint64_t *)(uintptr_t)tag, delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace bpftime_amd
