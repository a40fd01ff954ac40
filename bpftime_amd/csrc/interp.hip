// bpftime_amd: the gfx950 eBPF interpreter kernel.
//
// Replaces, for batches of packets/records, the per-packet CPU call chain
//   bpftime_prog::bpftime_prog_exec (runtime/src/bpftime_prog.cpp:231-260)
//   -> ebpf_exec (vm/vm-core/src/ebpf-vm.cpp:56-60) -> ubpf_exec
// with one wave64 lane per unit.  Design:
//  * the program is pre-decoded to 16-B DInsn records and fetched with scalar
//    loads: the pc is wave-uniform, so dispatch is a scalar branch tree;
//  * uniform branches take a ballot fast path; a split branch switches the
//    wave to per-lane pcs and min-pc scheduling until the lanes reconverge;
//  * r0-r10 live in LDS, lane-major (conflict-free ds_read_b64);
//  * the XDP ctx (48 B) and a stack sized by the loader's analysis live in
//    LDS; packet bytes and map values are read in place from HBM through
//    flat addresses;
//  * global accesses are confined to the batch window and the map arena
//    (a faulting program fails its lanes, never the GPU).
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

struct Win {
  uint64_t lo1, hi1, lo2, hi2;
  bool checked;
  __device__ __forceinline__ bool ok(uint64_t a, uint32_t sz) const {
    if (!checked) return true;
    if (is_lds_addr(a) || is_scratch_addr(a)) return true;
    uint64_t e = a + sz;
    return (a >= lo1 && e <= hi1 && e >= a) || (a >= lo2 && e <= hi2 && e >= a);
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

__device__ __forceinline__ uint32_t ald32(uint64_t a) {
  return __hip_atomic_load((uint32_t *)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint8_t ald8(uint64_t a) {
  uint64_t w = a & ~3ull;
  uint32_t v = ald32(w);
  return (uint8_t)(v >> ((a & 3) * 8));
}

// Compare the program-side key (any alignment, any memory) with a slot key
// (8-aligned, published with agent-scope stores).
__device__ __forceinline__ bool key_eq(uint64_t slot_key, uint64_t key, uint32_t ks) {
  uint32_t i = 0;
  for (; i + 4 <= ks; i += 4) {
    uint32_t kv = *(const u32u *)(key + i);
    if (ald32(slot_key + i) != kv) return false;
  }
  for (; i < ks; i++) {
    if (ald8(slot_key + i) != *(const volatile uint8_t *)(key + i)) return false;
  }
  return true;
}

__device__ __forceinline__ void copy_bytes_publish(uint64_t dst, uint64_t src, uint32_t n) {
  // dst is 8-aligned device memory; src is any flat address.
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4)
    __hip_atomic_store((uint32_t *)(dst + i), *(const u32u *)(src + i), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (i < n) {
    uint32_t w = 0;
    for (uint32_t j = 0; i + j < n; j++) w |= (uint32_t)(*(const volatile uint8_t *)(src + i + j)) << (8 * j);
    __hip_atomic_store((uint32_t *)(dst + i), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void copy_bytes(uint64_t dst, uint64_t src, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    *(volatile uint8_t *)(dst + i) = *(const volatile uint8_t *)(src + i);
}

constexpr uint32_t ST_EMPTY = 0, ST_FILLED = 1, ST_BUSY = 2;

// Find `key`; if absent and `insert`, claim a slot and publish key + init
// value (init == 0 -> zero).  Returns slot address or 0.  *inserted tells
// whether this lane created the element.  The probe order is the
// reference's: start at hash % nbuckets, linear, wrap once
// (bpftime_hash_map.hpp:127-180).  Lanes never wait on a lane of their own
// wave: a BUSY slot is re-read on the next loop trip, by which time the
// claiming lane (same wave, same trip) has published it.
__device__ uint64_t hash_find(const DMap &m, uint64_t key, bool insert, uint64_t init,
                              uint32_t init_bytes, bool *inserted) {
  *inserted = false;
  uint64_t nb = m.nbuckets;
  uint64_t idx = key_hash(key, m.key_size) % nb;
  uint64_t start = idx;
  uint32_t spins = 0;
  for (;;) {
    uint64_t s = m.data + idx * (uint64_t)m.slot_size;
    uint32_t st = ald32(s);
    if (st == ST_EMPTY) {
      if (!insert) return 0;
      // element count check (bpftime_hash_map.hpp:153-156)
      unsigned long long c = atomicAdd((unsigned long long *)m.count_addr, 1ull);
      if (c >= m.max_entries) {
        atomicAdd((unsigned long long *)m.count_addr, ~0ull);  // undo
        return 0;
      }
      uint32_t prev = atomicCAS((uint32_t *)s, ST_EMPTY, ST_BUSY);
      if (prev == ST_EMPTY) {
        copy_bytes_publish(s + m.key_off, key, m.key_size);
        if (init)
          copy_bytes_publish(s + m.val_off, init, init_bytes);
        else
          for (uint32_t i = 0; i < init_bytes; i += 4)
            __hip_atomic_store((uint32_t *)(s + m.val_off + i), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __hip_atomic_store((uint32_t *)s, ST_FILLED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        *inserted = true;
        return s;
      }
      atomicAdd((unsigned long long *)m.count_addr, ~0ull);  // lost the race: undo
      st = prev;
    }
    if (st == ST_BUSY) {
      if (++spins > (1u << 22)) return 0;  // bounded: never hang the GPU
      __builtin_amdgcn_s_sleep(1);
      continue;  // re-read the same slot on the next trip
    }
    if (key_eq(s + m.key_off, key, m.key_size)) return s;
    idx = idx + 1 == nb ? 0 : idx + 1;
    if (idx == start) return 0;
  }
}

struct LaneEnv {
  uint64_t vcpu;
  // last lookup miss (map fd, key hash) for the lookup_or_try_init race rule
  int32_t miss_fd;
  uint64_t miss_hash;
};

__device__ uint64_t helper_lookup(const DMap *maps, uint64_t fd, uint64_t key, LaneEnv &env) {
  if (fd >= kMaxFds) return 0;
  const DMap m = maps[fd];
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
  }
  return 0;
}

__device__ uint64_t helper_update(const DMap *maps, uint64_t fd, uint64_t key, uint64_t val,
                                  uint64_t flags, LaneEnv &env) {
  if (fd >= kMaxFds) return (uint64_t)-1;
  const DMap m = maps[fd];
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
      // per_cpu_hash_map.cpp:66-94: insert zeroed ncpu*vsize, then write slot
      bool ins;
      uint64_t s = hash_find(m, key, true, 0, m.value_size * m.ncpu, &ins);
      if (!s) return 0;
      bool race = !ins && env.miss_fd == (int32_t)fd && env.miss_hash == key_hash(key, m.key_size);
      if (!race) copy_bytes(s + m.val_off + (env.vcpu % m.ncpu) * m.value_size, val, m.value_size);
      env.miss_fd = -1;
      return 0;
    }
  }
  return (uint64_t)-1;
}

__device__ uint64_t helper_delete(const DMap *maps, uint64_t fd, uint64_t key, LaneEnv &env) {
  if (fd >= kMaxFds) return (uint64_t)-1;
  const DMap m = maps[fd];
  switch (m.type) {
    case MT_ARRAY:
    case MT_PERCPU_ARRAY:
      return (uint64_t)-1;  // EINVAL (array_map.cpp:58-64)
    case MT_HASH: {
      bool ins;
      uint64_t s = hash_find(m, key, false, 0, 0, &ins);
      if (s) {
        uint32_t prev = atomicCAS((uint32_t *)s, ST_FILLED, ST_EMPTY);  // no tombstone
        if (prev == ST_FILLED) atomicAdd((unsigned long long *)m.count_addr, ~0ull);
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
// The interpreter
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
#define RREG(i) Rf[(uint32_t)(i) * kBlock + tid]

template <uint32_t KIND, bool BIGSTACK>
__global__ __launch_bounds__(kBlock) void k_interp(KParams p) {
  __shared__ uint64_t Rf[11 * kBlock];
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  constexpr uint32_t CTXB = KIND == CTX_XDP ? 48 : 0;
  const uint32_t tid = threadIdx.x;
  uint8_t *my_ctx = dyn + tid * CTXB;
  uint8_t *my_stack = dyn + kBlock * CTXB + tid * p.stack_size;
  uint64_t big_stack[BIGSTACK ? kStackSize / 8 : 1];
  const Win win{p.data_lo, p.data_hi, p.arena_lo, p.arena_hi, p.checked != 0};
  // per-wave delta cache for fused counters (wave-uniform, lives in SGPRs)
  uint64_t c0a = 0, c0d = 0, c1a = 0, c1d = 0;
  uint32_t c0s = 0, c1s = 0;
  const uint64_t stack_top = BIGSTACK ? (uint64_t)(uintptr_t)(big_stack + kStackSize / 8)
                                      : (uint64_t)(uintptr_t)(my_stack + p.stack_size);

  const bool ordered = p.ordered != 0;
  const uint64_t ustep = ordered ? 1 : (uint64_t)gridDim.x * kBlock;
  // constant address space: the program is read with scalar (s_load) loads
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 __attribute__((address_space(4))) *prog =
      (const u32x4 __attribute__((address_space(4))) *)p.prog;
  for (uint64_t u0 = ordered ? 0 : (uint64_t)blockIdx.x * kBlock; u0 < p.n; u0 += ustep) {
    const uint64_t unit = ordered ? u0 : u0 + tid;
    const bool active = ordered ? (tid == 0 && blockIdx.x == 0) : unit < p.n;
    const uint64_t slot = (uint64_t)(uintptr_t)p.data + unit * p.stride;
    uint32_t len = p.fixed_len;
    if (active && p.lens) len = p.lens[unit];

    LaneEnv env;
    env.vcpu = (p.first_unit + unit) / 64;
    env.miss_fd = -1;
    env.miss_hash = 0;

    // ---- per-unit setup (r1, r2, r10) ----
    for (uint32_t r = 0; r < 11; r++) RREG(r) = 0;
    if (KIND == CTX_XDP) {
      XdpCtx *c = (XdpCtx *)my_ctx;
      c->data = slot + p.head;
      c->data_end = slot + p.head + len;
      c->data_meta = 0;
      c->ingress_ifindex = p.ifindex;
      c->rx_queue_index = p.rxq;
      c->egress_ifindex = 0;
      c->buffer_start = slot;
      c->buffer_end = slot + p.stride;
      RREG(1) = (uint64_t)(uintptr_t)c;
      RREG(2) = 48;
    } else {
      RREG(1) = slot;
      RREG(2) = KIND == CTX_SYSCALL ? 64 : len;
    }
    RREG(10) = stack_top;

    bool alive = active;
    if (KIND == CTX_SYSCALL && active) {
      // exit / exit_group bypass every callback (syscall_trace_attach_impl.cpp:25)
      int64_t nr = *(const int64_t *)(slot + 8);
      if (nr == 60 || nr == 231) alive = false;
    }
    uint32_t err = E_OK;
    uint32_t pc = 0;      // wave-uniform pc (uniform mode)
    uint32_t lpc = 0;     // per-lane pc (divergent mode)
    bool uni = true;
    uint64_t steps = 0;
    if (__ballot(alive) != 0)
    for (;;) {
      uint32_t cur;
      bool sel;
      if (uni) {
        cur = pc;
        sel = alive;
      } else {
        const uint32_t m = alive ? lpc : 0xffffffffu;
        cur = __reduce_min_sync(~0ull, m);
        if (cur == 0xffffffffu) break;
        sel = alive && lpc == cur;
        if (__ballot(alive && lpc != cur) == 0) uni = true;  // reconverged
      }
      cur = __builtin_amdgcn_readfirstlane(cur);
      if (++steps > p.step_limit) {
        if (alive) err = E_STEPS;
        alive = false;
        break;
      }
      const u32x4 raw = prog[cur];
      DInsn d;
      __builtin_memcpy(&d, &raw, sizeof(d));
      const uint32_t op = __builtin_amdgcn_readfirstlane(d.op);
      uint32_t npc = cur + 1;
      bool jmp = false;
      bool taken = false;
      const uint64_t mask = (d.aux & A_W32) ? 0xffffffffull : ~0ull;

#define OPB() ((d.aux & A_SRCREG) ? RREG(d.src) : (uint64_t)(int64_t)d.imm)
#define ALU(expr)                          \
  if (sel) {                               \
    const uint64_t a = RREG(d.dst);        \
    const uint64_t b = OPB();              \
    (void)a;                               \
    (void)b;                               \
    RREG(d.dst) = (expr);                  \
  }                                        \
  break;
#define JCMP(expr)                          \
  jmp = true;                               \
  if (sel) {                                \
    uint64_t a = RREG(d.dst);               \
    uint64_t b = OPB();                     \
    if (d.aux & A_W32) {                    \
      a = (uint32_t)a;                      \
      b = (uint32_t)b;                      \
    }                                       \
    taken = (expr);                         \
  }                                         \
  break;
#define JSCMP(cmp)                                                   \
  jmp = true;                                                        \
  if (sel) {                                                         \
    int64_t a = (int64_t)RREG(d.dst);                                \
    int64_t b = (int64_t)OPB();                                      \
    if (d.aux & A_W32) {                                             \
      a = (int32_t)a;                                                \
      b = (int32_t)b;                                                \
    }                                                                \
    taken = a cmp b;                                                 \
  }                                                                  \
  break;

      switch (op) {
        case X_ADD: ALU((a + b) & mask)
        case X_SUB: ALU((a - b) & mask)
        case X_MUL: ALU((a * b) & mask)
        case X_OR: ALU((a | b) & mask)
        case X_AND: ALU((a & b) & mask)
        case X_XOR: ALU((a ^ b) & mask)
        case X_MOV: ALU(b & mask)
        case X_DIV64: ALU(b ? a / b : 0)
        case X_MOD64: ALU(b ? a % b : a)
        case X_LSH64: ALU(a << (b & 63))
        case X_RSH64: ALU(a >> (b & 63))
        case X_ARSH64: ALU((uint64_t)((int64_t)a >> (b & 63)))
        case X_NEG64: ALU((uint64_t)(-(int64_t)a))
        case X_DIV32: ALU((uint32_t)b ? (uint64_t)((uint32_t)a / (uint32_t)b) : 0)
        case X_MOD32: ALU((uint32_t)b ? (uint64_t)((uint32_t)a % (uint32_t)b) : (uint64_t)(uint32_t)a)
        case X_LSH32: ALU((uint64_t)(uint32_t)((uint32_t)a << (b & 31)))
        case X_RSH32: ALU((uint64_t)((uint32_t)a >> (b & 31)))
        case X_ARSH32: ALU((uint64_t)(uint32_t)((int32_t)a >> (b & 31)))
        case X_NEG32: ALU((uint64_t)(uint32_t)(-(int64_t)a))
        case X_LE:
          ALU(d.imm == 16 ? (uint64_t)(uint16_t)a : d.imm == 32 ? (uint64_t)(uint32_t)a : a)
        case X_BE:
          ALU(d.imm == 16   ? (uint64_t)__builtin_bswap16((uint16_t)a)
              : d.imm == 32 ? (uint64_t)__builtin_bswap32((uint32_t)a)
              : d.imm == 64 ? __builtin_bswap64(a)
                            : a)
        case X_LDDW:
          if (sel) RREG(d.dst) = (uint64_t)(uint32_t)d.imm | ((uint64_t)(uint32_t)d.hi << 32);
          npc = cur + 2;
          break;
        case X_LDX: {
          const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
          if (sel) {
            const uint64_t a = RREG(d.src) + (int64_t)d.off;
            if (win.ok(a, sz)) {
              RREG(d.dst) = mem_load(a, sz);
            } else {
              err = E_OOB;
              alive = false;
            }
          }
          break;
        }
        case X_ST:
        case X_STX: {
          const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
          if (sel) {
            const uint64_t a = RREG(d.dst) + (int64_t)d.off;
            const uint64_t v = op == X_STX ? RREG(d.src) : (uint64_t)(int64_t)d.imm;
            if (win.ok(a, sz)) {
              mem_store(a, sz, v);
            } else {
              err = E_OOB;
              alive = false;
            }
          }
          break;
        }
        case X_RMW_ADD: {
          // fused ldx/add/stx (loaded register proven dead by the loader)
          // Counters hit by a whole wave (e.g. cntrs_array[0]) are summed across
          // the wave and kept in a per-wave scalar delta cache flushed with one
          // atomic at the end of the launch; otherwise one atomic per lane.
          const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
          uint64_t a = 0, v = 0;
          if (sel) {
            a = RREG(d.dst) + (int64_t)d.off;
            v = OPB();
          }
          const uint64_t selm = __ballot(sel);
          const int first = __builtin_ctzll(selm);
          const uint64_t a0 = readlane64(a, first);
          if (__ballot(sel && a != a0) == 0 && win.ok(a0, sz) && !is_lds_addr(a0) && !is_scratch_addr(a0)) {
            const uint64_t v0 = readlane64(v, first);
            uint64_t total;
            if (__ballot(sel && v != v0) == 0)
              total = v0 * (uint64_t)__builtin_popcountll(selm);
            else
              total = wave_sum64(sel ? v : 0);
            if (c0a == a0 && c0s == sz) {
              c0d += total;
            } else if (c1a == a0 && c1s == sz) {
              c1d += total;
            } else if (c0a == 0) {
              c0a = a0; c0s = sz; c0d = total;
            } else if (c1a == 0) {
              c1a = a0; c1s = sz; c1d = total;
            } else {
              flush_delta(c1a, c1s, c1d);
              c1a = a0; c1s = sz; c1d = total;
            }
          } else if (sel) {
            if (win.ok(a, sz)) {
              if (sz == 8)
                __hip_atomic_fetch_add((uint64_t *)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              else if (sz == 4)
                __hip_atomic_fetch_add((uint32_t *)a, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              else
                mem_store(a, sz, mem_load(a, sz) + v);  // 1/2-byte: not fused by the loader
            } else {
              err = E_OOB;
              alive = false;
            }
          }
          npc = d.tgt;
          break;
        }
        case X_ATOMIC: {
          const bool w64 = ((d.aux >> A_SIZE_SHIFT) & 3) == 3;
          if (sel) {
            const uint64_t a = RREG(d.dst) + (int64_t)d.off;
            const uint64_t v = RREG(d.src);
            if (!win.ok(a, w64 ? 8 : 4)) {
              err = E_OOB;
              alive = false;
            } else if (d.hi == 0xf1) {  // CMPXCHG: r0 = old
              if (w64) {
                uint64_t e = RREG(0);
                __hip_atomic_compare_exchange_strong((uint64_t *)a, &e, v, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                RREG(0) = e;
              } else {
                uint32_t e = (uint32_t)RREG(0);
                __hip_atomic_compare_exchange_strong((uint32_t *)a, &e, (uint32_t)v, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                RREG(0) = e;
              }
            } else if (d.hi == 0xe1) {  // XCHG
              RREG(d.src) = w64 ? __hip_atomic_exchange((uint64_t *)a, v, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)
                                : (uint64_t)__hip_atomic_exchange((uint32_t *)a, (uint32_t)v,
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              uint64_t old = 0;
              const uint32_t aop = d.hi & ~1;
              if (w64) {
                uint64_t *q = (uint64_t *)a;
                if (aop == 0x00) old = __hip_atomic_fetch_add(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (aop == 0x40) old = __hip_atomic_fetch_or(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (aop == 0x50) old = __hip_atomic_fetch_and(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else old = __hip_atomic_fetch_xor(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              } else {
                uint32_t *q = (uint32_t *)a;
                const uint32_t w = (uint32_t)v;
                if (aop == 0x00) old = __hip_atomic_fetch_add(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (aop == 0x40) old = __hip_atomic_fetch_or(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (aop == 0x50) old = __hip_atomic_fetch_and(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else old = __hip_atomic_fetch_xor(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              if (d.hi & 1) RREG(d.src) = old;
            }
          }
          break;
        }
        case X_JA:
          jmp = true;
          taken = sel;
          break;
        case X_JEQ: JCMP(a == b)
        case X_JGT: JCMP(a > b)
        case X_JGE: JCMP(a >= b)
        case X_JSET: JCMP((a & b) != 0)
        case X_JNE: JCMP(a != b)
        case X_JLT: JCMP(a < b)
        case X_JLE: JCMP(a <= b)
        case X_JSGT: JSCMP(>)
        case X_JSGE: JSCMP(>=)
        case X_JSLT: JSCMP(<)
        case X_JSLE: JSCMP(<=)
        case X_CALL: {
          if (sel) {
            const uint64_t a1 = RREG(1), a2 = RREG(2), a3 = RREG(3), a4 = RREG(4), a5 = RREG(5);
            uint64_t r = 0;
            switch (d.hi) {
              case 1: r = helper_lookup(p.maps, a1, a2, env); break;
              case 2: r = helper_update(p.maps, a1, a2, a3, a4, env); break;
              case 3: r = helper_delete(p.maps, a1, a2, env); break;
              case 5: r = (uint64_t)__builtin_amdgcn_s_memrealtime() * 10ull; break;
              case 7: {
                uint64_t x = (p.first_unit + unit) * 0x9E3779B97F4A7C15ull + steps;
                x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
                r = (uint32_t)x;
                break;
              }
              case 8: r = env.vcpu % p.ncpu; break;
              case 28: r = helper_csum_diff(a1, a2, a3, a4, a5); break;
              case 44: r = helper_adjust_head(a1, a2); break;
              case 65: r = helper_adjust_tail(a1, a2); break;
              case 189: r = helper_xdp_load_bytes(a1, a2, a3, a4); break;
              default: err = E_BADOP; alive = false; break;
            }
            RREG(0) = r;
          }
          break;
        }
        case X_EXIT:
          if (sel) {
            alive = false;
            if (err == E_OK) {
              const uint64_t r0 = RREG(0);
              if (p.verdicts) p.verdicts[unit] = (uint32_t)r0;
              if (p.rets) p.rets[unit] = r0;
            }
          }
          npc = 0xffffffffu;
          break;
        default:
          if (sel) {
            err = E_BADOP;
            alive = false;
          }
          break;
      }
#undef ALU
#undef JCMP
#undef JSCMP
#undef OPB

      // ---- next pc ----
      if (op == X_EXIT) {
        if (uni) break;  // every alive lane was selected and has exited
        continue;        // divergent: remaining lanes continue
      }
      if (jmp) {
        const uint64_t tm = __ballot(taken);
        const uint64_t sm = __ballot(sel);
        if (uni) {
          if (tm == 0) {
            pc = npc;
          } else if (tm == sm) {
            pc = d.tgt;
          } else {
            uni = false;
            if (sel) lpc = taken ? (uint32_t)d.tgt : npc;
          }
        } else {
          if (sel) lpc = taken ? (uint32_t)d.tgt : npc;
        }
      } else {
        if (uni)
          pc = npc;
        else if (sel)
          lpc = npc;
      }
      if (!uni && __ballot(alive) == 0) break;
      if (uni && op >= X_LDX && op <= X_RMW_ADD && __ballot(alive) == 0) break;
      if (uni && (op == X_CALL || op == X_BAD || op >= X_NOP) && __ballot(alive) == 0) break;
    }

    if (active) {
      if (err != E_OK) {
        // bpftime_prog.cpp:250-257: a failed exec reports 0
        if (p.verdicts) p.verdicts[unit] = 0;
        if (p.rets) p.rets[unit] = 0;
        atomicAdd(p.err_count, 1u);
      } else if (KIND == CTX_SYSCALL) {
        int64_t nr = *(const int64_t *)(slot + 8);
        if (nr == 60 || nr == 231) {
          if (p.verdicts) p.verdicts[unit] = 0;
          if (p.rets) p.rets[unit] = 0;
        }
      }
      if (KIND == CTX_XDP) {
        const XdpCtx *c = (const XdpCtx *)my_ctx;
        if (p.out_data_off) p.out_data_off[unit] = (int32_t)(c->data - slot);
        if (p.out_len) p.out_len[unit] = (uint32_t)(c->data_end - c->data);
      }
    }
  }
  flush_delta(c0a, c0s, c0d);
  flush_delta(c1a, c1s, c1d);
}
#undef RREG

// ---------------------------------------------------------------------------
// Host-side launch wrappers
// ---------------------------------------------------------------------------
extern "C" hipError_t bpftime_amd_launch_interp(const KParams *p, uint32_t kind, bool big_stack,
                                                uint32_t grid, uint32_t ordered, hipStream_t stream) {
  KParams q = *p;
  q.ordered = ordered;
  const size_t ctxb = kind == CTX_XDP ? 48 : 0;
  const size_t dyn = kBlock * (ctxb + (big_stack ? 0 : p->stack_size));
  dim3 g(grid), b(kBlock);
#define L(K, B) hipLaunchKernelGGL((k_interp<K, B>), g, b, dyn, stream, q)
  if (kind == CTX_XDP) {
    if (big_stack) L(CTX_XDP, true); else L(CTX_XDP, false);
  } else if (kind == CTX_SYSCALL) {
    if (big_stack) L(CTX_SYSCALL, true); else L(CTX_SYSCALL, false);
  } else {
    if (big_stack) L(CTX_RAW, true); else L(CTX_RAW, false);
  }
#undef L
  return hipGetLastError();
}

extern "C" int bpftime_amd_occupancy(uint32_t kind, bool big_stack, size_t dyn_lds) {
  int n = 0;
  hipError_t e;
#define O(K, B) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_interp<K, B>, kBlock, dyn_lds)
  if (kind == CTX_XDP) {
    if (big_stack) O(CTX_XDP, true); else O(CTX_XDP, false);
  } else if (kind == CTX_SYSCALL) {
    if (big_stack) O(CTX_SYSCALL, true); else O(CTX_SYSCALL, false);
  } else {
    if (big_stack) O(CTX_RAW, true); else O(CTX_RAW, false);
  }
#undef O
  return e == hipSuccess ? n : 1;
}

}  // namespace bpftime_amd
