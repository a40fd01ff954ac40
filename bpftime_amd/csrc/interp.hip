// bpftime_amd: the gfx950 eBPF interpreter kernel.
//
// Replaces, for batches of packets/records, the per-packet CPU call chain
//   bpftime_prog::bpftime_prog_exec (runtime/src/bpftime_prog.cpp:231-260)
//   -> ebpf_exec (vm/vm-core/src/ebpf-vm.cpp:56-60) -> ubpf_exec
// with one wave64 lane per unit.  Design:
//  * tier 1, the threaded-code fast path (gen_fast.py -> fast_asm.inc): one
//    inline-asm block whose handlers dispatch through s_setpc_b64 on 32-B
//    FInsn records fetched with scalar loads; eBPF r0-r10 live in VGPRs
//    (s_set_gpr_idx_on), the unit's first bytes are staged in VGPRs, split
//    branches become lane groups scheduled by minimum pc, lookups / counter
//    adds / tail calls / exits run in asm;
//  * tier 2, this file's C++ interpreter (run_loop), for what the asm does
//    not take (other helpers, div/mod, cmpxchg, accesses failing the fast
//    checks, more lane groups than the asm holds): a UNIFORM loop (all live
//    lanes at one pc) and a DIVERGENT loop (per-lane pcs, min-pc
//    scheduling), with branch-free case bodies (lanes that must not act
//    touch a per-lane dummy LDS slot).  It works on a [register][lane]
//    copy of r0-r10 -- in LDS, or in global memory for launches whose LDS
//    goes to a combining table / lookup cache (G) -- written when the asm
//    exits and read when it re-enters;
//  * helper calls leave both loops and run in the outer loop (R_CALL),
//    keeping the helpers' divergent code out of the hot loops;
//  * the XDP ctx (48 B) and a stack sized by the loader's analysis live in
//    LDS (else 512-B scratch); packet bytes and map values are read in
//    place; global accesses are confined to the batch window and the map
//    arena (a faulting program fails its lanes, never the GPU);
//  * counter adds are deferred where the loader proves no later access of
//    the unit observes them: per-wave delta caches and a per-block LDS
//    combining table, flushed when the block ends (k_comb_merge).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "dev_helpers.hpp"
#include "fast_asm.inc"
#include "fast_ops.hpp"

namespace bpftime_amd {

// Helper dispatch (helper id is wave-uniform); returns r0, sets *err.
__device__ __forceinline__ uint64_t call_helper(uint32_t id, uint64_t a1, uint64_t a2, uint64_t a3, uint64_t a4,
                                                uint64_t a5, const DMap *maps, uint32_t ncpu, uint64_t seed,
                                                LaneEnv &env, uint32_t *err) {
  switch (id) {
    case 1: return helper_lookup(maps, a1, a2, env);
    case 2: return helper_update(maps, a1, a2, a3, a4, env);
    case 3: return helper_delete(maps, a1, a2, env);
    case 5: return env.kt_on ? env.ktime : (uint64_t)__builtin_amdgcn_s_memrealtime() * 10ull;
    case 7: {
      uint64_t x = seed * 0x9E3779B97F4A7C15ull;
      x ^= x >> 31;
      x *= 0xBF58476D1CE4E5B9ull;
      x ^= x >> 29;
      return (uint32_t)x;
    }
    case 8: return env.vcpu % ncpu;
    case 14: return env.pid_tgid;  // bpf_get_current_pid_tgid (KParams::pid_off)
    case 28: return helper_csum_diff(a1, a2, a3, a4, a5);
    case 44: return helper_adjust_head(a1, a2);
    case 65: return helper_adjust_tail(a1, a2);
    case 189: return helper_xdp_load_bytes(a1, a2, a3, a4);
    case 130: return rb_output(maps, a1, a2, a3, env.rb);
    case 131: return rb_reserve(maps, a1, a2, env.rb);
    case 132: rb_submit(maps, a1, false, env.rb); return 0;
    case 133: rb_submit(maps, a1, true, env.rb); return 0;
    case 58: return helper_set_retval(a2, env, err);   // bpf_override_return(ctx, value)
    case 187: return helper_set_retval(a1, env, err);  // bpf_set_retval(value)
  }
  *err = E_BADOP;
  return 0;
}

// Copy a wave-uniform value into a fresh SGPR (an explicit s_mov, so the
// result is not tied to the kernel-argument tuple it was loaded into).
__device__ __forceinline__ uint64_t sreg(uint64_t v) {
  uint64_t o;
  asm volatile("s_mov_b64 %0, %1" : "=s"(o) : "s"(v));
  return o;
}
__device__ __forceinline__ uint32_t sreg(uint32_t v) {
  uint32_t o;
  asm volatile("s_mov_b32 %0, %1" : "=s"(o) : "s"(v));
  return o;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(4))) *prog_ptr;

// loop exits
constexpr uint32_t R_DONE = 0, R_DIVERGE = 1, R_RECONV = 2, R_CALL = 3, R_STEP = 4;

// Everything one interpreter loop reads or updates (inlined; SROA'd).
struct Ctx {
  uint64_t *R;           // this lane's register file column: R[i * kBlock]
  prog_ptr prog;
  const FInsn *fast;     // per-launch threaded form (w1: FW_* flags)
  Win win;
  uint64_t dummy;        // flat address of this lane's dummy LDS slot
  uint32_t *verdicts;
  uint64_t *rets;
  uint64_t unit;
  uint32_t step_limit;
  // mutable state
  uint32_t pc;           // uniform loop: the wave's pc
  uint32_t lpc;          // divergent loop: this lane's pc
  uint32_t steps;
  bool alive;
  uint32_t err;
  uint32_t call_pc, call_id;
  uint64_t c0a, c0d, c1a, c1d;  // per-wave fused-counter delta cache
  uint32_t c0s, c1s;
};

#define RG(i) c.R[(uint32_t)(i) * kBlock]

// Runs the program until the wave exits, diverges / reconverges, or calls
// a helper.  UNI: every live lane is at c.pc and selected.  ONE: return
// R_STEP after one instruction (the slow step behind the asm fast path).
template <bool UNI, bool ONE = false>
__device__ __forceinline__ uint32_t run_loop(Ctx &c) {
  for (;;) {
    uint32_t cur;
    bool sel;
    if (UNI) {
      cur = c.pc;
      sel = c.alive;
    } else {
      const uint32_t m = c.alive ? c.lpc : 0xffffffffu;
      cur = __reduce_min_sync(~0ull, m);
      if (cur == 0xffffffffu) return R_DONE;
      if (__ballot(c.alive && c.lpc != cur) == 0) {
        c.pc = cur;
        return R_RECONV;
      }
      sel = c.alive && c.lpc == cur;
    }
    cur = __builtin_amdgcn_readfirstlane(cur);
    if (++c.steps > c.step_limit) {
      c.err = c.alive ? E_STEPS : c.err;
      c.alive = false;
      return R_DONE;
    }
    const u32x4 raw = c.prog[cur];
    DInsn d;
    __builtin_memcpy(&d, &raw, sizeof(d));
    const uint32_t op = d.op;
    const bool srcreg = (d.aux & A_SRCREG) != 0;
    const bool w32 = (d.aux & A_W32) != 0;
    const uint64_t mask = w32 ? 0xffffffffull : ~0ull;
    uint32_t npc = cur + 1;

// write a register: selected lanes only (in the uniform loop the other
// lanes may be parked lane groups, interp kernel loop)
#define WRO(r, val, old) RG(r) = sel ? (uint64_t)(val) : (uint64_t)(old)
#define OPB(rv) (srcreg ? (rv) : (uint64_t)(int64_t)d.imm)
#define ALU(expr)                              \
  {                                            \
    const uint64_t a = RG(d.dst);              \
    const uint64_t b = OPB(RG(d.src));         \
    WRO(d.dst, (expr), a);                     \
    break;                                     \
  }
#define JMP_TAKEN(cond)                        \
  {                                            \
    taken = sel && (cond);                     \
    is_jmp = true;                             \
    break;                                     \
  }
    bool is_jmp = false, taken = false;
    uint64_t ja = 0, jb = 0;
    if (op >= X_JEQ && op <= X_JSLE) {
      ja = RG(d.dst);
      jb = OPB(RG(d.src));
    }
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
      case X_LE: ALU(d.imm == 16 ? (uint64_t)(uint16_t)a : d.imm == 32 ? (uint64_t)(uint32_t)a : a)
      case X_BE:
        ALU(d.imm == 16   ? (uint64_t)__builtin_bswap16((uint16_t)a)
            : d.imm == 32 ? (uint64_t)__builtin_bswap32((uint32_t)a)
            : d.imm == 64 ? __builtin_bswap64(a)
                          : a)
      case X_LDDW: {
        const uint64_t v = (uint64_t)(uint32_t)d.imm | ((uint64_t)(uint32_t)d.hi << 32);
        WRO(d.dst, v, RG(d.dst));
        npc = cur + 2;
        break;
      }
      case X_LDX: {
        const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
        const uint64_t a = RG(d.src) + (int64_t)d.off;
        const bool ok = c.win.ok(a, sz);
        const uint64_t v = mem_load(sel && ok ? a : c.dummy, sz);
        WRO(d.dst, v, RG(d.dst));
        if (__ballot(sel && !ok) != 0) {
          c.err = (sel && !ok) ? E_OOB : c.err;
          c.alive = c.alive && !(sel && !ok);
          if (__ballot(c.alive) == 0) return R_DONE;
        }
        break;
      }
      case X_ST:
      case X_STX: {
        const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
        const uint64_t a = RG(d.dst) + (int64_t)d.off;
        const uint64_t v = op == X_STX ? RG(d.src) : (uint64_t)(int64_t)d.imm;
        const bool ok = c.win.ok(a, sz);
        mem_store(sel && ok ? a : c.dummy, sz, v);
        if (__ballot(sel && !ok) != 0) {
          c.err = (sel && !ok) ? E_OOB : c.err;
          c.alive = c.alive && !(sel && !ok);
          if (__ballot(c.alive) == 0) return R_DONE;
        }
        break;
      }
      case X_RMW_ADD: {
        // Counters hit by a whole wave (e.g. cntrs_array[0]) are summed across
        // the wave into the per-wave delta cache; otherwise one atomic per lane.
        // FW_NODEFER counters (a later access of the unit can observe them,
        // or the batch is ORDERED) and fetch forms reach memory here.
        const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
        const uint64_t a = RG(d.dst) + (int64_t)d.off;
        const uint64_t v = OPB(RG(d.src));
        const bool fetch = (d.aux & A_FETCH) != 0;
        const uint32_t fw = __builtin_amdgcn_readfirstlane(c.fast[cur].w1);  // uniform by construction
        if (fetch || (fw & FW_NODEFER)) {
          const bool ok = c.win.ok(a, sz);
          const bool local = is_lds_addr(a) || is_scratch_addr(a);  // the unit's own stack: no other writer
          uint64_t old = 0;
          if (sel && ok && local) {
            old = mem_load(a, sz);
            mem_store(a, sz, old + v);
          }
          // global: lanes adding to one address take one atomic in lane
          // order (each lane's old value = the leader's result + the adds of
          // the lanes before it: a serial order of the wave's units)
          uint64_t pend = __ballot(sel && ok && !local);
          while (pend) {
            const int leader = __builtin_ctzll(pend);
            const uint64_t la = readlane64(a, leader);
            const bool mine = ((pend >> __lane_id()) & 1) && a == la;
            const uint64_t m = __ballot(mine);
            const uint64_t add = mine ? (sz == 8 ? v : (uint64_t)(uint32_t)v) : 0;
            uint64_t incl = add;
            for (int o = 1; o < 64; o <<= 1) {
              const uint64_t t = __shfl_up(incl, (unsigned)o, 64);
              if ((int)__lane_id() >= o) incl += t;
            }
            const uint64_t total = readlane64(incl, 63);
            uint64_t base = 0;
            if ((int)__lane_id() == leader) {
              if (sz == 8)
                base = __hip_atomic_fetch_add((uint64_t *)la, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              else
                base = __hip_atomic_fetch_add((uint32_t *)la, (uint32_t)total, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            }
            base = readlane64(base, leader);
            if (mine) old = base + incl - add;
            pend &= ~m;
          }
          if (fetch) {
            // ldx zero-extends; the add is 64-bit unless it was ALU32
            const uint64_t o = sz == 8 ? old : (uint64_t)(uint32_t)old;
            const uint64_t r = (d.aux & A_W32) ? (uint64_t)(uint32_t)(o + v) : o + v;
            WRO(d.hi, r, RG(d.hi));
          }
          if (__ballot(sel && !ok) != 0) {
            c.err = (sel && !ok) ? E_OOB : c.err;
            c.alive = c.alive && !(sel && !ok);
            if (__ballot(c.alive) == 0) return R_DONE;
          }
          npc = d.tgt;
          break;
        }
        const uint64_t selm = __ballot(sel);
        const int first = __builtin_ctzll(selm);
        const uint64_t a0 = readlane64(a, first);
        if (__ballot(sel && a != a0) == 0 && c.win.ok(a0, sz) && !is_lds_addr(a0) && !is_scratch_addr(a0)) {
          const uint64_t v0 = readlane64(v, first);
          uint64_t total;
          if (__ballot(sel && v != v0) == 0)
            total = v0 * (uint64_t)__builtin_popcountll(selm);
          else
            total = wave_sum64(sel ? v : 0);
          if (c.c0a == a0 && c.c0s == sz) {
            c.c0d += total;
          } else if (c.c1a == a0 && c.c1s == sz) {
            c.c1d += total;
          } else if (c.c0a == 0) {
            c.c0a = a0;
            c.c0s = sz;
            c.c0d = total;
          } else if (c.c1a == 0) {
            c.c1a = a0;
            c.c1s = sz;
            c.c1d = total;
          } else {
            flush_delta(c.c1a, c.c1s, c.c1d);
            c.c1a = a0;
            c.c1s = sz;
            c.c1d = total;
          }
        } else {
          const bool ok = c.win.ok(a, sz);
          const uint64_t ea = sel && ok ? a : c.dummy;
          if (sz == 8)
            __hip_atomic_fetch_add((uint64_t *)ea, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            __hip_atomic_fetch_add((uint32_t *)ea, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__ballot(sel && !ok) != 0) {
            c.err = (sel && !ok) ? E_OOB : c.err;
            c.alive = c.alive && !(sel && !ok);
            if (__ballot(c.alive) == 0) return R_DONE;
          }
        }
        npc = d.tgt;
        break;
      }
      case X_ATOMIC: {
        const bool w64 = ((d.aux >> A_SIZE_SHIFT) & 3) == 3;
        const uint64_t a = RG(d.dst) + (int64_t)d.off;
        const uint64_t v = RG(d.src);
        const bool ok = c.win.ok(a, w64 ? 8 : 4);
        const uint64_t ea = sel && ok ? a : c.dummy;
        if (d.hi == 0xf1) {  // CMPXCHG: r0 = old
          const uint64_t r0 = RG(0);
          uint64_t res;
          if (w64) {
            uint64_t e = r0;
            __hip_atomic_compare_exchange_strong((uint64_t *)ea, &e, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            res = e;
          } else {
            uint32_t e = (uint32_t)r0;
            __hip_atomic_compare_exchange_strong((uint32_t *)ea, &e, (uint32_t)v, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            res = e;
          }
          WRO(0, res, r0);
        } else if (d.hi == 0xe1) {  // XCHG
          const uint64_t old = w64 ? __hip_atomic_exchange((uint64_t *)ea, v, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)
                                   : (uint64_t)__hip_atomic_exchange((uint32_t *)ea, (uint32_t)v, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT);
          WRO(d.src, old, v);
        } else if (d.hi == 0x00) {
          // add without fetch: lanes adding to one address are summed across
          // the wave and one of them adds (same-address device atomics
          // serialize at the memory side); the final value is the same
          uint64_t pend = __ballot(sel && ok);
          while (pend) {
            const int leader = __builtin_ctzll(pend);
            const uint64_t la = readlane64(a, leader);
            const bool mine = ((pend >> __lane_id()) & 1) && a == la;
            const uint64_t m = __ballot(mine);
            const uint64_t sum = wave_sum64(mine ? (w64 ? v : (uint64_t)(uint32_t)v) : 0);
            if ((int)__lane_id() == leader) {
              if (w64)
                __hip_atomic_fetch_add((uint64_t *)la, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              else
                __hip_atomic_fetch_add((uint32_t *)la, (uint32_t)sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            pend &= ~m;
          }
        } else {
          uint64_t old;
          const uint32_t aop = (uint32_t)d.hi & ~1u;
          if (w64) {
            uint64_t *q = (uint64_t *)ea;
            if (aop == 0x00) old = __hip_atomic_fetch_add(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (aop == 0x40) old = __hip_atomic_fetch_or(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (aop == 0x50) old = __hip_atomic_fetch_and(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else old = __hip_atomic_fetch_xor(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            uint32_t *q = (uint32_t *)ea;
            const uint32_t w = (uint32_t)v;
            if (aop == 0x00) old = __hip_atomic_fetch_add(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (aop == 0x40) old = __hip_atomic_fetch_or(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (aop == 0x50) old = __hip_atomic_fetch_and(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else old = __hip_atomic_fetch_xor(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (d.hi & 1) WRO(d.src, old, v);
        }
        if (__ballot(sel && !ok) != 0) {
          c.err = (sel && !ok) ? E_OOB : c.err;
          c.alive = c.alive && !(sel && !ok);
          if (__ballot(c.alive) == 0) return R_DONE;
        }
        break;
      }
      case X_JA: JMP_TAKEN(true)
      case X_JEQ: JMP_TAKEN((ja & mask) == (jb & mask))
      case X_JNE: JMP_TAKEN((ja & mask) != (jb & mask))
      case X_JGT: JMP_TAKEN((ja & mask) > (jb & mask))
      case X_JGE: JMP_TAKEN((ja & mask) >= (jb & mask))
      case X_JLT: JMP_TAKEN((ja & mask) < (jb & mask))
      case X_JLE: JMP_TAKEN((ja & mask) <= (jb & mask))
      case X_JSET: JMP_TAKEN((ja & jb & mask) != 0)
      case X_JSGT: JMP_TAKEN((w32 ? (int64_t)(int32_t)ja : (int64_t)ja) > (w32 ? (int64_t)(int32_t)jb : (int64_t)jb))
      case X_JSGE: JMP_TAKEN((w32 ? (int64_t)(int32_t)ja : (int64_t)ja) >= (w32 ? (int64_t)(int32_t)jb : (int64_t)jb))
      case X_JSLT: JMP_TAKEN((w32 ? (int64_t)(int32_t)ja : (int64_t)ja) < (w32 ? (int64_t)(int32_t)jb : (int64_t)jb))
      case X_JSLE: JMP_TAKEN((w32 ? (int64_t)(int32_t)ja : (int64_t)ja) <= (w32 ? (int64_t)(int32_t)jb : (int64_t)jb))
      case X_CALL:
        c.call_pc = cur;
        c.call_id = (uint32_t)d.hi;
        return R_CALL;
      case X_EXIT: {
        const uint64_t r0 = RG(0);
        const bool w = sel && c.err == E_OK;
        if (c.verdicts) *(uint32_t *)(w ? (uint64_t)(uintptr_t)(c.verdicts + c.unit) : c.dummy) = (uint32_t)r0;
        if (c.rets) *(uint64_t *)(w ? (uint64_t)(uintptr_t)(c.rets + c.unit) : c.dummy) = r0;
        c.alive = c.alive && !sel;
        if (UNI) return R_DONE;  // every live lane was selected and has exited
        continue;                // divergent: the other lanes continue
      }
      default:
        c.err = sel ? E_BADOP : c.err;
        c.alive = c.alive && !sel;
        if (UNI) return R_DONE;
        continue;
    }
#undef ALU
#undef JMP_TAKEN
#undef OPB
#undef WRO
    // ---- next pc ----
    if (is_jmp) {
      if (UNI) {
        const uint64_t tm = __ballot(taken);
        if (tm == 0) {
          c.pc = npc;
        } else if (tm == __ballot(sel)) {
          c.pc = d.tgt;
        } else {
          c.lpc = sel ? (taken ? (uint32_t)d.tgt : npc) : c.lpc;
          return R_DIVERGE;
        }
      } else {
        c.lpc = sel ? (taken ? (uint32_t)d.tgt : npc) : c.lpc;
      }
    } else {
      if (UNI)
        c.pc = npc;
      else
        c.lpc = sel ? npc : c.lpc;
    }
    if (ONE) return R_STEP;
  }
}
#undef RG

// Threaded-code fast path (gen_fast.py): runs the uniform loop in asm from
// c.pc until an instruction it does not handle; returns 1 if the step limit
// was crossed at a taken jump, else 0 (c.pc = the instruction to run in C++).
struct FastEnv {
  const FInsn *fast;
  const DMap *maps;
  uint64_t dlo, dhi, alo, ahi;
  uint32_t shi, phi;
  uint32_t oflags;  // bit 0: verdicts, bit 1: rets
  uint32_t head;    // batch head: ctx->data = slot + head
  uint32_t comb;    // LDS address of the block's combining table
  uint32_t combn;   // its entries (0: add straight to memory)
  uint32_t rb;      // LDS byte address of this lane's R[0] (G: of its dummy slot)
  uint32_t stage;   // staged bytes per unit (0: no staging)
  uint32_t ncpu;    // virtual CPUs (per-CPU maps)
  uint32_t sstep;   // chained units: slot bytes from one unit of a lane to its next
  uint32_t ustep;   // ... and units (verdict / ret / length array steps)
};

constexpr uint32_t FAST_SLOW = 0, FAST_STEPS = 1, FAST_EXIT = 2, FAST_SPLIT = 3;

// Per-unit inputs of a fresh entry (gen_fast.py: registers from operands,
// optional staging of the slot's first kFastStageBytes bytes).
struct FastUnit {
  uint64_t r1, r10, slot;
  uint32_t r2;
  uint32_t len;    // unit length (ctx->data_end - ctx->data)
  // bit 0: fresh unit, 1: stage the slot, 2: lane groups in asm; chained
  // units (gen_fast.py chain_routine): 3 r1 = slot, 4 r2 = length, 5 lengths
  // from laddr, 6 syscall-record filter, 16.. virtual-cpu step
  uint32_t entry;
  uint32_t vm;     // the unit's virtual CPU mod ncpu (per-CPU array lookups)
  uint64_t vaddr, raddr, laddr;  // the unit's verdict / ret / length addresses (0: none)
  uint32_t chain;  // further units the asm may run for this wave (every lane's unit < n)
};

// adv: units the asm tier finished and moved past (chained); the lanes are
// then in the wave's unit `adv` iterations further on, at c.pc
template <bool G>
__device__ __forceinline__ uint32_t run_fast(Ctx &c, const FastEnv &f, const FastUnit &u, uint32_t chain_in,
                                             uint32_t &adv) {
  // every "s" operand must be provably uniform: readfirstlane what the
  // compiler cannot prove (the values are uniform by construction)
  uint32_t pc = __builtin_amdgcn_readfirstlane(c.pc), steps = __builtin_amdgcn_readfirstlane(c.steps), why;
  uint64_t alive_out;
  uint32_t lpc;
  const uint64_t alive = __ballot(c.alive);
  const uint32_t limit = __builtin_amdgcn_readfirstlane(c.step_limit);
  const uint32_t entry = __builtin_amdgcn_readfirstlane(u.entry);
  // (the wave's counter cache: uniform by construction, but the compiler
  // cannot prove it across the lane-group scheduling loop)
  auto u32 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); };
  auto u64 = [&](uint64_t v) { return (uint64_t)u32((uint32_t)v) | ((uint64_t)u32((uint32_t)(v >> 32)) << 32); };
  uint64_t c0a = u64(c.c0a), c1a = u64(c.c1a);
  uint32_t c0dl = u32((uint32_t)c.c0d), c0dh = u32((uint32_t)(c.c0d >> 32)), c1dl = u32((uint32_t)c.c1d),
           c1dh = u32((uint32_t)(c.c1d >> 32)), c0s = u32(c.c0s), c1s = u32(c.c1s);
  // the wave's virtual cpu for per-CPU array lookups: cpu | ncpu << 16 when
  // every lane shares it (consecutive units), else ~0
  const uint32_t vm0 = __builtin_amdgcn_readfirstlane(u.vm);
  uint32_t vcpu = __ballot(c.alive && u.vm != vm0) == 0 && f.ncpu <= 0xffff ? vm0 | (f.ncpu << 16) : ~0u;
  uint64_t vaddr = u.vaddr, raddr = u.raddr, laddr = u.laddr;
  uint32_t ulen = u.len, chain = __builtin_amdgcn_readfirstlane(chain_in);
  uint32_t m0s;  // M0 across the block (gen_fast.py: saved at the entry, restored at the exit)
#define FAST_OUTS                                                                                             \
  [pc] "+s"(pc), [steps] "+s"(steps), [why] "=s"(why), [aliveout] "=s"(alive_out), [lpc] "=v"(lpc),            \
      [c0a] "+s"(c0a), [c1a] "+s"(c1a), [c0dl] "+s"(c0dl), [c0dh] "+s"(c0dh), [c1dl] "+s"(c1dl),                \
      [c1dh] "+s"(c1dh), [c0s] "+s"(c0s), [c1s] "+s"(c1s), [vaddr] "+v"(vaddr), [raddr] "+v"(raddr),            \
      [laddr] "+v"(laddr), [ulen] "+v"(ulen), [chain] "+s"(chain), [vcpu] "+s"(vcpu), [m0s] "=&s"(m0s)
#define FAST_INS                                                                                              \
  [prog] "s"(f.fast), [maps] "s"(f.maps), [dlo] "s"(f.dlo), [dhi] "s"(f.dhi), [alo] "s"(f.alo),               \
      [ahi] "s"(f.ahi), [shi] "s"(f.shi), [phi] "s"(f.phi), [limit] "s"(limit), [rb] "v"(f.rb),               \
      [alive] "s"(alive), [oflags] "s"(f.oflags), [entry] "s"(entry), [r1lo] "v"((uint32_t)u.r1),               \
      [r1hi] "v"((uint32_t)(u.r1 >> 32)), [r2lo] "v"(u.r2), [r10lo] "v"((uint32_t)u.r10),                       \
      [r10hi] "v"((uint32_t)(u.r10 >> 32)), [slotlo] "v"((uint32_t)u.slot),                                    \
      [slothi] "v"((uint32_t)(u.slot >> 32)), [head] "s"(f.head), [stklo] "v"((uint32_t)u.r10),                 \
      [comb] "s"(f.comb), [combn] "s"(f.combn), [stage] "s"(f.stage), [sstep] "s"(f.sstep), [ustep] "s"(f.ustep)
  if constexpr (G)
    asm volatile(BPFTIME_AMD_FAST_ASM_G : FAST_OUTS : FAST_INS : BPFTIME_AMD_FAST_CLOBBERS);
  else
    asm volatile(BPFTIME_AMD_FAST_ASM : FAST_OUTS : FAST_INS : BPFTIME_AMD_FAST_CLOBBERS);
#undef FAST_OUTS
#undef FAST_INS
  adv = __builtin_amdgcn_readfirstlane(chain_in) - chain;
  c.pc = pc;
  c.steps = steps;
  c.c0a = c0a;
  c.c1a = c1a;
  c.c0d = (uint64_t)c0dl | ((uint64_t)c0dh << 32);
  c.c1d = (uint64_t)c1dl | ((uint64_t)c1dh << 32);
  c.c0s = c0s;
  c.c1s = c1s;
  // lanes that ran exit inside the block are done (verdict stored); after
  // chaining every lane is in a later unit, alive as the asm left it
  c.alive = (adv ? true : c.alive) && ((alive_out >> __lane_id()) & 1);
  if (why == FAST_SPLIT && c.alive) c.lpc = lpc;  // (parked lane groups keep theirs)
  return why;
}

// xdp_md_userspace of one unit (runtime/extension/userspace_xdp.h:6-17)
__device__ __forceinline__ void write_xdp_ctx(XdpCtx *x, uint64_t slot, uint32_t len, uint64_t chunk,
                                              const KParams &p) {
  x->data = slot + p.head;
  x->data_end = slot + p.head + len;
  x->data_meta = 0;
  x->ingress_ifindex = p.ifindex;
  x->rx_queue_index = p.rxq;
  x->egress_ifindex = 0;
  x->buffer_start = chunk;
  x->buffer_end = chunk + (p.descs && !p.stride ? len : p.stride);
}

// IMAGE: a linked tail-call image (lane groups scheduled through the asm tier)
// G: r0..r10's copy for the C++ tier lives in global memory (p.gregs, the
// block's [register][lane] columns) instead of LDS: 22 KiB of LDS per block
// go to residency (launches with a combining table or lookup cache, whose
// units stay in the asm tier)
template <uint32_t KIND, bool BIGSTACK, bool IMAGE, bool G, uint32_t BS>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4))) void k_interp(KParams pin) {
  static_assert(BS == kBlock || (BS == kBigBlock && G && !IMAGE && !BIGSTACK), "big blocks: G launches only");
  // Copy every kernel argument through an SGPR barrier: without it the
  // compiler keeps the argument block as one 16-dword tuple that it spills
  // and reloads whole inside the dispatch loop.
  KParams p;
#define SRP(f) p.f = (decltype(p.f))sreg((uint64_t)(uintptr_t)pin.f)
#define SRV(f) p.f = sreg(pin.f)
  SRP(prog); SRP(fast); SRP(maps); SRP(data); SRP(lens); SRP(verdicts); SRP(rets); SRP(out_data_off); SRP(out_len);
  SRP(err_count); SRV(n); SRV(stride); SRV(first_unit); SRV(data_lo); SRV(data_hi); SRV(arena_lo);
  SRV(arena_hi); SRV(step_limit); SRV(fixed_len); SRV(stack_size); SRV(ncpu); SRV(ifindex); SRV(rxq);
  SRV(checked); SRV(head); SRV(ordered); SRV(fast_div); SRV(comb_entries); SRV(stage); SRV(needs_ctx);
  SRP(descs); SRV(umem_bytes); SRP(tail_entry); SRP(frames); SRV(frame_words); SRV(dbg); SRP(dbg_counts); SRP(flush_log); SRV(log_words); SRP(lane_scratch);
  SRV(lru_seq); SRV(tail_ctx_mask); SRV(tail_stack_mask); SRV(tail_lds); SRV(lcache); SRP(gregs); SRP(rb_stage); SRP(gctx);
  SRP(miss_log); SRP(miss_counts); SRV(miss_cap); SRP(tail_slots); SRV(full_q); SRV(full_r); SRV(step_cpu);
  SRP(sys_state); SRP(sys_ret); SRV(sys_phase); SRV(pid_tgid);
  p.pid_off = (int32_t)sreg((uint64_t)(uint32_t)pin.pid_off);
  SRP(pid_base); SRV(pid_stride); SRP(kt_base); SRV(kt_stride); SRV(ctx_stride); SRV(stack_stride);
  p.sys_nr = (int64_t)sreg((uint64_t)pin.sys_nr);
  p.unwind_idx = (int32_t)sreg((uint64_t)(uint32_t)pin.unwind_idx);
#undef SRP
#undef SRV
  // r0..r10, a dummy slot, and (images) the lane's tail-call depth | its
  // grid lane index << 32 (gen_fast.py tail_env).  (2 KiB of LDS decide
  // between 3 and 4 resident blocks of the headline program: images only.)
  // (G: the dummy and depth slots only)
  constexpr uint32_t kDummy = G ? 0 : 11, kDepth = G ? 1 : 12;
  __shared__ uint64_t Rf[(IMAGE ? kDepth + 1 : kDummy + 1) * BS];
  // r0..r10 columns: [register][lane] per 256 lanes (kBlock), so a block of
  // BS > kBlock lanes (G launches only) holds BS / kBlock such column sets
  uint64_t *const Rg = G ? p.gregs + (uint64_t)blockIdx.x * 11 * BS : Rf;
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  // the lane's XDP ctx: in LDS, or (p.gctx: a program that only reads
  // data / data_end, whose ctx only the C++ tier touches) in global memory
  const uint32_t tid = threadIdx.x;
  // (lane strides: common.hpp lane_stride)
  const uint32_t ctxb = KIND == CTX_XDP && !p.gctx ? p.ctx_stride : 0;
  const uint32_t sstride = p.stack_stride;
  uint8_t *my_ctx = KIND == CTX_XDP && p.gctx ? p.gctx + ((uint64_t)blockIdx.x * BS + tid) * 48 : dyn + tid * ctxb;
  uint8_t *my_stack = dyn + BS * ctxb + tid * sstride;
  // combining table for per-lane counter adds (gen_fast.py comb_add), after
  // the ctx and stack areas: comb_entries u32 tags {16-byte granule's arena
  // offset (8-byte aligned for 8-byte counters) | 2 | (4-byte ? 1 : 0)}
  // (8-way sets), then comb_entries 16-byte
  // delta granules (2 x u64 or 4 x u32), flushed when the block ends; sized 0
  // for programs that never need it
  uint32_t *lcache = (uint32_t *)(dyn + BS * (ctxb + (BIGSTACK ? 0 : sstride)));
  uint64_t *tenv = (uint64_t *)((uint8_t *)lcache + lcache_bytes(p.lcache));
  uint32_t *comb = (uint32_t *)((uint8_t *)tenv + kTenvBytes);
  uint8_t *const comb_d = (uint8_t *)(comb + p.comb_entries);  // delta rows (common.hpp comb_granule_off)
  // XDP images: the LDS tail-call frames of the first depths (common.hpp
  // kTailLdsMax), [depth][word][lane]
  uint64_t *const lfr = (uint64_t *)((uint8_t *)comb + comb_bytes(p.comb_entries));
  for (uint32_t i = tid; i < comb_bytes(p.comb_entries) / 4; i += BS) comb[i] = 0;
  for (uint32_t i = tid; i < lcache_bytes(p.lcache) / 4; i += BS) lcache[i] = 0;
  // ring-buffer staging (dev_helpers.hpp RbStage): LDS counters of the block
  __shared__ RbLds rb_lds;
  if (tid == 0) {
    rb_lds.used = rb_lds.nrec = 0;
    rb_lds.fd = -1;
  }
  RbStage rbs;
  if (p.rb_stage) {
    rbs.buf = p.rb_stage + (uint64_t)blockIdx.x * kRbStageBytes;
    rbs.lds = &rb_lds;
  }
  // counter v of the table (entry v / 4, counter v % 4 of its granule) as a
  // flush tag {address | (4-byte ? 1 : 0)} and delta
  auto comb_counter = [&](uint32_t v, uint64_t &tag, uint64_t &delta) {
    const uint32_t e = v >> 2, j = v & 3, t = comb[comb_tag_pos(e, p.comb_entries)];
    tag = delta = 0;
    if (!t) return;
    // 4-byte granules are 16-byte aligned; 8-byte ones 8-byte aligned (pairs)
    const uint64_t g = p.arena_lo + (t & ((t & 1) ? ~15u : ~7u));
    const uint8_t *gr = comb_d + comb_granule_off(e);
    if (t & 1) {
      delta = ((const uint32_t *)gr)[j];
      tag = (g + 4 * j) | 1;
    } else if (j < 2) {
      delta = ((const uint64_t *)gr)[j];
      tag = g + 8 * j;
    }
  };
  // tail-call launch constants for the asm tier (XDP images: the frames'
  // ctx copy is the lane's LDS ctx): frames (0: tail calls in C++), entry
  // table, word stride | depth stride << 32, stack / ctx save masks
  if (tid == 0) {
    const bool on = IMAGE && KIND == CTX_XDP && p.frames && p.tail_entry && !(p.dbg & 8);  // dbg 8: C++ frames
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 8;
    tenv[0] = on ? (uint64_t)(uintptr_t)p.frames : 0;
    // (other launches, BPFTIME_AMD_DBG 512: the lookup cache's hit / miss
    // counters, gen_fast.py lcache_count)
    tenv[1] = IMAGE ? (uint64_t)(uintptr_t)p.tail_entry : (uint64_t)(uintptr_t)p.dbg_counts;
    tenv[2] = stride | ((stride * p.frame_words) << 32);
    const uint32_t sw = p.stack_size / 8;  // (images in the asm tier: <= kLdsStackMax bytes)
    const uint32_t smask = p.tail_stack_mask & (sw >= 16 ? 0xffffu : (1u << sw) - 1);
    tenv[3] = (uint64_t)smask | ((uint64_t)p.stack_size << 16) | ((uint64_t)(p.tail_ctx_mask & 0x3f) << 32) |
              ((p.dbg & 16) ? 1ull << 63 : 0);  // dbg 16: frames popped in C++
    // G: the block's global r0 column minus the LDS address of the lane
    // columns (gen_fast.py rgb: v40 + r * 2048 + this addresses r's copy)
    tenv[4] = G ? (uint64_t)(uintptr_t)Rg - (uint32_t)(uintptr_t)&Rf[0] : 0;
    // the block's miss-log region (gen_fast.py comb_add) and its records
    // per partition
    tenv[5] = p.miss_log ? (uint64_t)(uintptr_t)(p.miss_log + (uint64_t)blockIdx.x * kMissParts * p.miss_cap * 2) : 0;
    tenv[6] = p.miss_cap;
    // images: the slot -> entry pc table of the asm tier's bpf_tail_call
    tenv[7] = (uint64_t)(uintptr_t)p.tail_slots;
    // the block's ring staging for the asm tier's bpf_ringbuf_output
    // (gen_fast.py call_rbout): its area and the LDS address of its counters
    tenv[kTenvRb / 8] = p.rb_stage ? (uint64_t)(uintptr_t)rbs.buf : 0;
    tenv[kTenvRb / 8 + 1] = (uint32_t)(uintptr_t)&rb_lds;
    // the LDS frames (gen_fast.py tail_env): their address relative to the
    // lane columns (v40 + this = the lane's word 0 at depth 0), depths | words << 8
    tenv[kTenvLf / 8] = IMAGE ? (uint64_t)(uint32_t)((uintptr_t)lfr - (uintptr_t)&Rf[0]) | ((uint64_t)p.tail_lds << 32) : 0;
  }
  uint32_t *const miss_cnt = (uint32_t *)((uint8_t *)tenv + 64);  // per partition: records claimed
  for (uint32_t i = tid; i < kMissParts; i += BS) miss_cnt[i] = 0;
  __syncthreads();
  uint64_t big_stack[BIGSTACK ? kStackSize / 8 : 1];
  const uint64_t stack_top = BIGSTACK ? (uint64_t)(uintptr_t)(big_stack + kStackSize / 8)
                                      : (uint64_t)(uintptr_t)(my_stack + p.stack_size);

  Ctx c;
  c.R = G ? &Rg[(tid & ~(kBlock - 1)) * 11 + (tid & (kBlock - 1))] : &Rg[tid];
  c.prog = (prog_ptr)p.prog;
  c.fast = p.fast;
  {
    const uint64_t sl = (uint64_t)(uintptr_t)p.lane_scratch;
    // (the lane scratch words, then the blocks' ring-buffer staging areas:
    // a program writes a record it reserved there; then the global ctxs)
    c.win = Win{p.data_lo, p.data_hi, p.arena_lo, p.arena_hi, sl,
                sl ? sl + 8ull * gridDim.x * BS + (p.rb_stage ? (uint64_t)gridDim.x * kRbStageBytes : 0) +
                         (p.gctx ? 48ull * gridDim.x * BS : 0)
                   : 0,
                p.checked != 0};
  }
  c.dummy = (uint64_t)(uintptr_t)&Rf[kDummy * BS + tid];
  c.verdicts = p.verdicts;
  c.rets = p.rets;
  c.step_limit = p.step_limit > 0xffffffffull ? 0xffffffffu : (uint32_t)p.step_limit;
  c.c0a = c.c0d = c.c1a = c.c1d = 0;
  c.c0s = c.c1s = 0;

  // fast-path operands, computed once into SGPRs (sreg: no per-entry rebuild)
  FastEnv fe;
  fe.fast = (const FInsn *)sreg((uint64_t)(uintptr_t)p.fast);
  fe.maps = p.maps;
  fe.comb = sreg((uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)comb));
  fe.combn = p.comb_entries;
  fe.head = p.head;
  // (bit 2, BPFTIME_AMD_DBG 128: counter adds that miss the combining table
  // are dropped -- a timing experiment, never a result)
  fe.oflags = sreg((uint32_t)__builtin_amdgcn_readfirstlane((p.verdicts ? 1u : 0u) | (p.rets ? 2u : 0u) |
                                                            ((p.dbg & 128) ? 4u : 0u) |
                                                            ((p.dbg & 512) && p.dbg_counts ? 8u : 0u)));
  fe.dlo = sreg((uint64_t)(p.checked ? p.data_lo : 0));
  fe.dhi = sreg((uint64_t)(p.checked ? p.data_hi : ~(uint64_t)0));
  fe.alo = p.arena_lo;
  fe.ahi = p.arena_hi;
  fe.shi = sreg((uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)(uintptr_t)&Rf[0] >> 32)));
  fe.phi = BIGSTACK ? sreg((uint32_t)__builtin_amdgcn_readfirstlane(
                          (uint32_t)((uint64_t)(uintptr_t)&big_stack[0] >> 32)))
                    : fe.shi;
  // (G: v40 + r * 2048 + tenv[4] addresses the lane's copy of r, gen_fast.py
  // rgb; v40 is no LDS address there)
  fe.rb = (uint32_t)(uintptr_t)&Rf[0] + 8 * (uint32_t)(G ? (c.R - Rg) : tid);

  // the host sized the staged window (gen_fast.py, unit staging) from the
  // program's static packet / slot accesses, 16-B aligned slots only
  fe.stage = p.stage;
  fe.ncpu = p.ncpu ? p.ncpu : 1;

  const bool ordered = p.ordered != 0;
  const uint64_t ustep = ordered ? 1 : (uint64_t)gridDim.x * BS;
  // Chained units (gen_fast.py chain_routine): while every lane of the wave
  // has a unit, the asm tier starts the wave's next unit itself.  Plain
  // strided batches only: no descriptors, no per-unit ctx in LDS or ctx
  // outputs, no syscall-number filter; dbg 64 turns it off.  (Images: only
  // from a unit no lane group is parked in, and the depth is reset.)
  const bool chain_ok = !ordered && !p.descs && p.stride && !p.out_data_off && !p.out_len &&
                        !(KIND == CTX_XDP && p.needs_ctx) &&
                        !(KIND == CTX_SYSCALL && (p.sys_nr >= 0 || p.sys_state)) &&
                        ustep * p.stride < (1ull << 32) && !(p.dbg & 64);
  uint64_t full = 0;  // iterations in which every lane of this wave has a unit
  if (chain_ok) {
    // (n - 64 - wb) / ustep + 1 for the wave's first unit wb < ustep, from
    // the host's quotient and remainder of (n - 64) / ustep
    const uint64_t wb = (uint64_t)blockIdx.x * BS + __builtin_amdgcn_readfirstlane(tid & ~63u);
    full = p.n >= wb + 64 ? p.full_q + (wb <= p.full_r ? 1 : 0) : 0;
  }
  fe.sstep = (uint32_t)(ustep * p.stride);
  fe.ustep = (uint32_t)ustep;
  const uint32_t ncpu = fe.ncpu;
  const bool ncpu_pow2 = (ncpu & (ncpu - 1)) == 0;
  const uint32_t chain_bits = (KIND != CTX_XDP ? 8u : 0u) | (KIND == CTX_RAW ? 16u : 0u) | (p.lens ? 32u : 0u) |
                              (KIND == CTX_SYSCALL ? 64u : 0u) | (IMAGE ? 128u : 0u) |
                              (p.step_cpu << 16);
  // the host linker's query (vm_api.cpp fast_xlat, one unit): the asm block
  // writes its handlers' offsets (u32 per handler id) at p.verdicts and the
  // kernel ends (through the one run_fast site, so the block is not inlined
  // twice)
  const bool xlat = (p.dbg & kDbgXlat) != 0;
  uint64_t it = 0;
  for (uint64_t u0 = ordered ? 0 : (uint64_t)blockIdx.x * BS; u0 < p.n; u0 += ustep, it++) {
    uint64_t unit, slot, chunk, vcpu;
    bool active, desc_ok;
    uint32_t len;
    int32_t miss_fd;
    uint64_t miss_hash;
    uint32_t lru_ops;
    bool ctx_ready;
    FastUnit fu;
    // the unit's addresses and per-unit helper state (also after the asm
    // tier chained into a later unit: `chained`)
    auto begin = [&](bool chained) {
      unit = ordered ? u0 : u0 + tid;
      active = ordered ? (tid == 0 && blockIdx.x == 0) : unit < p.n;
      slot = (uint64_t)(uintptr_t)p.data + unit * p.stride;
      chunk = slot;  // XDP ctx buffer_start
      len = p.fixed_len;
      desc_ok = true;
      if (p.descs) {
        // AF_XDP descriptor ring: the frame at umem + addr; its chunk bounds
        // the ctx buffer (aligned-chunk umem)
        uint64_t addr = 0;
        len = 0;
        if (active) {
          addr = p.descs[2 * unit];
          len = (uint32_t)p.descs[2 * unit + 1];
        }
        desc_ok = addr < p.umem_bytes && len <= p.umem_bytes - addr;
        if (!desc_ok) addr = len = 0;
        slot = (uint64_t)(uintptr_t)p.data + addr;
        chunk = (uint64_t)(uintptr_t)p.data + (p.stride ? addr - addr % p.stride : addr);
      } else if (active && p.lens) {
        len = p.lens[unit];
      }
      vcpu = (p.first_unit + unit) / 64;
      miss_fd = -1;
      miss_hash = 0;
      lru_ops = 0;
      fu.vm = ncpu_pow2 ? (uint32_t)vcpu & (ncpu - 1) : (uint32_t)(vcpu % ncpu);
      fu.slot = slot;
      fu.len = len;
      fu.vaddr = p.verdicts ? (uint64_t)(uintptr_t)(p.verdicts + unit) : 0;
      fu.raddr = p.rets ? (uint64_t)(uintptr_t)(p.rets + unit) : 0;
      fu.laddr = p.lens ? (uint64_t)(uintptr_t)(p.lens + unit) : 0;
      fu.chain = it + 1 < full ? (full - 1 - it > 0x7fffffffull ? 0x7fffffffu : (uint32_t)(full - 1 - it)) : 0;
      c.unit = unit;
      c.err = active && !desc_ok ? E_OOB : E_OK;
      ctx_ready = KIND != CTX_XDP || p.needs_ctx;
      (void)chained;
    };
    begin(false);
    // tail-call frames this lane has pushed (images: in LDS, the asm tier
    // pushes too)
    uint32_t tdepth_reg = 0;
    uint32_t *const tdep = IMAGE ? (uint32_t *)&Rf[(IMAGE ? kDepth : 0) * kBlock + tid] : &tdepth_reg;
    if (IMAGE) Rf[(IMAGE ? kDepth : 0) * kBlock + tid] = (uint64_t)(blockIdx.x * kBlock + tid) << 32;

    // ---- per-unit setup: r1, r2, r10 (other registers zero) are set by the
    // fast path's fresh entry, which every unit starts with ----
    fu.r10 = stack_top;
    fu.entry = 1u | (p.stage ? 2u : 0u) | (p.fast_div ? 4u : 0u) | chain_bits;
    if (p.descs && p.stage) {
      // staging needs every lane's window 16-B aligned inside the umem
      const bool bad = active && ((slot & 15) != 0 || slot + p.stage > (uint64_t)(uintptr_t)p.data + p.umem_bytes);
      if (__ballot(bad) != 0) fu.entry &= ~2u;
    }
    if (KIND == CTX_XDP) {
      // the ctx only exists in LDS when the program reads it generically
      // (loader: ctx uses other than the specialised data / data_end loads)
      XdpCtx *x = (XdpCtx *)my_ctx;
      if (p.needs_ctx) write_xdp_ctx(x, slot, len, chunk, p);
      fu.r1 = (uint64_t)(uintptr_t)x;
      fu.r2 = 48;
    } else {
      fu.r1 = slot;
      fu.r2 = len;  // (syscall kinds: the ctx size, 64 or 24, as fixed_len)
    }

    // syscall records this program does not run on: exit / exit_group
    // bypass every callback (syscall_trace_attach_impl.cpp:25), a per-syscall
    // program sees its nr only, and an exit program skips a record whose
    // enter programs overrode the return (:70-72; the dispatch's state)
    auto sys_skip = [&]() {
      const int64_t nr = *(const int64_t *)(slot + 8);
      return nr == 60 || nr == 231 || (p.sys_nr >= 0 && nr != p.sys_nr) ||
             (p.sys_state && p.sys_phase == 2 && (p.sys_state[unit] & 1));
    };
    bool alive = active;
    if (KIND == CTX_SYSCALL && active && sys_skip()) alive = false;
    c.alive = alive && desc_ok;
    c.pc = 0;
    c.lpc = 0;
    c.steps = 0;

    bool uni = true;
    // Divergent waves run one lane group at a time in the asm tier: the
    // group at the lowest pc runs as a uniform wave while the other lanes
    // are parked at their pcs (c.lpc), until the group exits, splits or
    // reaches a tail call / return; then the lowest group runs next, and
    // groups that meet at one pc run together again: tail-call images, and
    // the XDP launches with the register copy in global memory (G: hash
    // tables), where a hash insert's lanes run their insert path in asm
    // while the lanes that found their key wait (flow-hash's cold launch
    // 8.0 -> 5.0 ms; for the syscall kind the extra live state costs its
    // steady state 7 %, so it keeps the C++ divergent loop).
    // (BPFTIME_AMD_DBG bit 2: the C++ divergent loop instead.)
    const bool groups = (IMAGE || (G && KIND == CTX_XDP)) && p.fast_div && !(p.dbg & 4);
    bool parked = false;
    auto unpark = [&]() {
      c.alive = c.alive || parked;
      parked = false;
      uni = false;
    };
    // the asm tier computes specialised ctx->data / data_end loads from the
    // slot; the C++ tier reads the ctx, so it is written before the C++ tier
    // first runs an instruction of this unit (ctx_ready: begin)
    auto ctx_for_cpp = [&]() {
      if (KIND == CTX_XDP && !ctx_ready) {
        write_xdp_ctx((XdpCtx *)my_ctx, slot, len, chunk, p);
        ctx_ready = true;
      }
    };
    while (__ballot(c.alive || parked) != 0) {
      uint32_t r;
      if (groups && uni && __ballot(c.alive) == 0) {  // the running group died (a helper error): the parked lanes go on
        unpark();
        continue;
      }
      if (!uni && groups) {
        const uint32_t m = c.alive ? c.lpc : 0xffffffffu;
        const uint32_t cur = __builtin_amdgcn_readfirstlane(__reduce_min_sync(~0ull, m));
        parked = c.alive && c.lpc != cur;
        c.alive = c.alive && !parked;
        c.pc = cur;
        uni = true;
        continue;
      }
      if (uni) {
        // chain only from a unit every lane of the wave runs without a failure
        const bool whole = __ballot(c.alive) == ~0ull && __ballot(c.err != E_OK) == 0 && __ballot(parked) == 0;
        // entry bit 8: a lane's lookup just missed (the lookup-or-init race
        // rule of helper_update): its map updates stay in the C++ helper
        fu.entry = (fu.entry & ~256u) | (__ballot(miss_fd >= 0) != 0 ? 256u : 0u);
        uint32_t adv = 0;
        if (xlat) {
          fu.entry = ~0u;
          fu.vaddr = (uint64_t)(uintptr_t)p.verdicts;
        }
        const uint32_t why = run_fast<G>(c, fe, fu, whole ? fu.chain : 0u, adv);
        if (xlat) return;
        fu.entry &= ~1u;
        if (adv) {  // the asm tier finished `adv` units of this wave and is in the next
          it += adv;
          u0 += adv * ustep;
          begin(true);
        }
        if (why == FAST_EXIT) {  // every running lane ran exit; r0 already stored
          c.alive = false;
          if (__ballot(parked) == 0) break;
          unpark();
          continue;
        }
        if (why == FAST_SPLIT) {  // lane groups at different pcs (c.lpc)
          uni = false;
          unpark();
          continue;
        }
        if (why == FAST_STEPS) {
          c.err = c.alive || parked ? E_STEPS : c.err;
          c.alive = parked = false;
          break;
        }
        ctx_for_cpp();
        r = run_loop<true, true>(c);
      } else {
        ctx_for_cpp();
        r = run_loop<false>(c);
      }
      if (r == R_STEP) continue;
      if (r == R_DONE) {
        if (__ballot(parked) == 0) break;
        unpark();
        continue;
      }
      if (r == R_DIVERGE) {
        unpark();
        continue;
      }
      if (r == R_RECONV) {
        uni = true;
        continue;
      }
      // ---- R_CALL: helper call (bpf_helper.cpp helpers; csrc/dev_helpers.hpp) ----
      const bool csel = uni ? c.alive : (c.alive && c.lpc == c.call_pc);
      const uint32_t cid = __builtin_amdgcn_readfirstlane(c.call_id);  // uniform by construction
      if (p.tail_entry && (cid == kTailHelper || cid == (uint32_t)kRetHelper)) {
        // bpf_tail_call (bpf_helper.cpp:568-650) in a linked image
        // (common.hpp kTailHelper): push a frame and enter the target, or
        // pop one at a target's exit.  Lanes may go to different pcs.
        uint32_t next = c.lpc;
        if (csel) {
          ctx_for_cpp();
          uint64_t *R = c.R;
          // frames word-interleaved across the grid's lanes ([depth][word][lane]):
          // a wave's save of one word is one coalesced 512-B store
          uint64_t *const fbase = (uint64_t *)p.frames + (blockIdx.x * kBlock + tid);
          const uint64_t kLanes = (uint64_t)gridDim.x * kBlock;  // frames sized for this launch (vm_api.cpp)
          auto FW = [&](uint32_t d, uint32_t w) -> uint64_t & {
            return fbase[((uint64_t)d * p.frame_words + w) * kLanes];
          };
          // the LDS frames (depth < ldep): word w of the lane's frame at depth d
          const uint32_t ldep = p.tail_lds & 0xff, lwords = p.tail_lds >> 8;
          auto LF = [&](uint32_t d, uint32_t w) -> uint64_t & { return lfr[(d * lwords + w) * kBlock + tid]; };
          const uint32_t sbytes = BIGSTACK ? kStackSize : p.stack_size;
          if (cid == kTailHelper) {
            next = c.call_pc + 1;
            const uint64_t fd = R[2 * kBlock], a1 = R[1 * kBlock];
            const int32_t k = (int32_t)R[3 * kBlock];  // `int idx = index`
            int32_t entry = -1;
            if (fd < kMaxFds && p.maps[fd].type == MT_PROG_ARRAY && k >= 0 && (uint32_t)k < p.maps[fd].max_entries) {
              const int32_t t = *(const int32_t *)(p.maps[fd].data + 4ull * (uint32_t)k);
              if (t >= 0 && t < (int32_t)kMaxFds) entry = p.tail_entry[t];
            }
            // the 64-B ctx copy: the lane's LDS XDP ctx (48 B), else the
            // bytes of [a1, a1 + 64) the program may access (a unit shorter
            // than 64 B keeps to its window), outside its stack
            const bool lds_ctx = KIND == CTX_XDP && a1 == (uint64_t)(uintptr_t)my_ctx;
            uint32_t cb = 48;
            if (!lds_ctx)
              for (cb = 0; cb < kFrameCtx && c.win.ok(a1 + cb, 8); cb += 8) {
              }
            const bool in_stack = a1 + 64 > stack_top - sbytes && a1 < stack_top;
            if (entry >= 0 && tdep[0] < kTailDepth && a1 != 0 && !in_stack) {
              const uint32_t d = tdep[0];
              if (d < ldep) LF(d, 0) = 0;  // a full frame: in global memory
              for (int r = 1; r <= 10; r++) FW(d, r - 1) = R[r * kBlock];
              FW(d, 10) = a1;
              FW(d, 11) = (uint64_t)next | ((uint64_t)cb << 32);
              for (uint32_t i = 0; i < cb; i += 8) FW(d, kFrameHdr / 8 + i / 8) = mem_load(a1 + i, 8);
              const uint64_t sb = stack_top - sbytes;
              for (uint32_t i = 0; i < sbytes; i += 8)
                FW(d, (kFrameHdr + kFrameCtx) / 8 + i / 8) = *(const uint64_t *)(sb + i);
              for (int r = 0; r <= 10; r++) R[r * kBlock] = 0;
              R[1 * kBlock] = a1;
              R[2 * kBlock] = 64;  // bpftime_prog_exec(context, sizeof(context), ...)
              R[10 * kBlock] = stack_top;
              tdep[0] = d + 1;
              next = (uint32_t)entry;
            } else {
              R[0] = (uint64_t)-1;
            }
          } else if (tdep[0] == 0) {
            c.err = E_BADOP;
            c.alive = false;
          } else {
            const uint32_t d = tdep[0] - 1;
            tdep[0] = d;
            const uint64_t rv = R[0];
            const bool lds = d < ldep && (LF(d, 0) & kFrameMasked);
            const uint64_t w11 = lds ? LF(d, 0) : FW(d, 11);
            next = (uint32_t)w11;
            const uint64_t sb = stack_top - sbytes;
            if (lds) {  // an LDS frame (common.hpp kTailLdsMax): the words in order
              uint32_t w = 1;
              for (int r = 1; r <= 9; r++) {
                if ((w11 >> (kFrameLiveShift + r)) & 1) R[r * kBlock] = LF(d, w++);
                if ((w11 >> (kFrameRematShift + r)) & 1) R[r * kBlock] = (uint64_t)(uintptr_t)my_ctx;
              }
              R[10 * kBlock] = stack_top;
              for (uint32_t k = 0; k < 6; k++)
                if ((p.tail_ctx_mask >> k) & 1) mem_store((uint64_t)(uintptr_t)my_ctx + 8 * k, 8, LF(d, w++));
              for (uint32_t j = 0; 8 * j < sbytes && j < 16; j++)
                if ((p.tail_stack_mask >> j) & 1) *(uint64_t *)(sb + 8 * j) = LF(d, w++);
            } else if (w11 & kFrameMasked) {  // pushed by the asm tier (common.hpp kFrameMasked)
              for (int r = 1; r <= 9; r++) {
                if ((w11 >> (kFrameLiveShift + r)) & 1) R[r * kBlock] = FW(d, r - 1);
                if ((w11 >> (kFrameRematShift + r)) & 1) R[r * kBlock] = (uint64_t)(uintptr_t)my_ctx;
              }
              R[10 * kBlock] = stack_top;
              for (uint32_t k = 0; k < 6; k++)
                if ((p.tail_ctx_mask >> k) & 1) mem_store((uint64_t)(uintptr_t)my_ctx + 8 * k, 8, FW(d, kFrameHdr / 8 + k));
              for (uint32_t j = 0; 8 * j < sbytes; j++)
                if ((p.tail_stack_mask >> j) & 1) *(uint64_t *)(sb + 8 * j) = FW(d, (kFrameHdr + kFrameCtx) / 8 + j);
            } else {
              for (int r = 1; r <= 10; r++) R[r * kBlock] = FW(d, r - 1);
              const uint64_t a1 = FW(d, 10);
              const uint32_t cb = (uint32_t)(w11 >> 32) & 0xff;
              for (uint32_t i = 0; i < cb; i += 8) mem_store(a1 + i, 8, FW(d, kFrameHdr / 8 + i / 8));
              for (uint32_t i = 0; i < sbytes; i += 8)
                *(uint64_t *)(sb + i) = FW(d, (kFrameHdr + kFrameCtx) / 8 + i / 8);
            }
            R[0] = rv;
          }
        }
        c.lpc = csel ? next : c.lpc;
        unpark();
        continue;
      }
      if (csel) {
        LaneEnv env;
        env.vcpu = vcpu;
        env.scratch = p.lane_scratch ? (uint64_t)(uintptr_t)(p.lane_scratch + (uint64_t)blockIdx.x * BS + tid) : 0;
        env.miss_fd = miss_fd;
        env.miss_hash = miss_hash;
        env.lru_stamp = (p.lru_seq << kLruSeqShift) | ((unit & 0xffffffffull) << kLruUnitShift);
        env.lru_ops = lru_ops;
        env.exact = ordered;
        env.rb = rbs;
        env.ovr_state = p.sys_state ? p.sys_state + unit : nullptr;
        env.ovr_val = p.sys_ret ? p.sys_ret + unit : nullptr;
        env.ovr_bit = p.sys_phase;
        env.pid_tgid = p.pid_base ? *(const uint64_t *)(p.pid_base + unit * p.pid_stride) : p.pid_tgid;
        env.kt_on = p.kt_base != nullptr;
        env.ktime = p.kt_base ? *(const uint64_t *)(p.kt_base + unit * p.kt_stride) : 0;
        uint32_t cerr = E_OK;
        uint64_t *R = c.R;
        const uint64_t rv = call_helper(c.call_id, R[1 * kBlock], R[2 * kBlock], R[3 * kBlock], R[4 * kBlock],
                                        R[5 * kBlock], p.maps, p.ncpu,
                                        (p.first_unit + unit) ^ ((uint64_t)c.steps << 40), env, &cerr);
        R[0] = rv;
        miss_fd = env.miss_fd;
        miss_hash = env.miss_hash;
        lru_ops = env.lru_ops;
        if (cerr != E_OK) {
          c.err = cerr;
          c.alive = false;
        }
        // ebpf_set_unwind_function_index (ubpf unwind-on-success): the
        // helper's 0 return ends the unit with r0 = 0, as its exit would --
        // not inside a tail-call target, which the reference runs in a
        // program of its own without the index
        if (c.alive && (int32_t)c.call_id == p.unwind_idx && rv == 0 && tdep[0] == 0) {
          if (c.verdicts) c.verdicts[c.unit] = 0;
          if (c.rets) c.rets[c.unit] = 0;
          c.alive = false;
        }
      }
      if (uni)
        c.pc = c.call_pc + 1;
      else
        c.lpc = csel ? c.call_pc + 1 : c.lpc;
    }

    if (active) {
      if (c.err != E_OK) {
        // bpftime_prog.cpp:250-257: a failed exec reports 0
        if (p.verdicts) p.verdicts[unit] = 0;
        if (p.rets) p.rets[unit] = (p.dbg & 32) ? (0xE0000000ull | c.err | ((uint64_t)c.pc << 8) | ((uint64_t)c.lpc << 36)) : 0;
        atomicAdd(p.err_count, 1u);
      } else if (KIND == CTX_SYSCALL && sys_skip()) {
        if (p.verdicts) p.verdicts[unit] = 0;
        if (p.rets) p.rets[unit] = 0;
      }
      if (KIND == CTX_XDP) {
        const XdpCtx *x = (const XdpCtx *)my_ctx;
        if (p.out_data_off) p.out_data_off[unit] = p.needs_ctx ? (int32_t)(x->data - slot) : (int32_t)p.head;
        if (p.out_len) p.out_len[unit] = p.needs_ctx ? (uint32_t)(x->data_end - x->data) : len;
      }
    }
  }
  // the waves' fused-counter caches are combined per block before they
  // reach memory: every wave of the grid ends at about the same time, and
  // same-address device atomics serialize at the memory side (~12 ns each,
  // MI355X_MICROARCH.md 'fanin'), so one add per block instead of per wave
  // shortens the kernel's tail four-fold
  __shared__ uint64_t wdelta[BS / 64][2][2];  // {tag = address | (4-byte ? 1 : 0), delta}
  __shared__ uint32_t nlog;
  if ((tid & 63) == 0) {
    const uint32_t w = tid >> 6;
    wdelta[w][0][0] = c.c0a && c.c0d ? (c.c0a | (c.c0s == 4 ? 1 : 0)) : 0;
    wdelta[w][0][1] = c.c0d;
    wdelta[w][1][0] = c.c1a && c.c1d ? (c.c1a | (c.c1s == 4 ? 1 : 0)) : 0;
    wdelta[w][1][1] = c.c1d;
  }
  if (tid == 0) nlog = 0;
  __syncthreads();
  if (p.rb_stage) rb_publish(p.maps, rbs, tid, BS);
  if (p.miss_log)  // (records past the capacity were added directly)
    for (uint32_t i = tid; i < kMissParts; i += BS)
      p.miss_counts[(uint64_t)blockIdx.x * kMissParts + i] = min(miss_cnt[i], p.miss_cap);
  uint64_t *e = &wdelta[0][0][0];
  constexpr uint32_t NE = wave_cache_entries(BS);
  if (tid == 0) {
    for (uint32_t i = 0; i < NE; i++) {
      if (!e[2 * i]) continue;
      for (uint32_t j = i + 1; j < NE; j++)
        if (e[2 * j] == e[2 * i]) {
          e[2 * i + 1] += e[2 * j + 1];
          e[2 * j] = 0;
        }
      if (!p.flush_log) flush_delta_tag(e[2 * i], e[2 * i + 1]);
    }
  }
  if (!p.flush_log) {
    if (!(p.dbg & 1))
      for (uint32_t i = tid; i < 4 * p.comb_entries; i += BS) {
        uint64_t tag, delta;
        comb_counter(i, tag, delta);
        flush_delta_tag(tag, delta);
      }
    return;
  }
  // append the nonzero deltas (wave caches, then the table) to this block's
  // log region; k_comb_merge adds them.  A block holding many addresses adds
  // them itself: a map with that many hot values spans many memory channels,
  // so its atomics do not queue on a few words, and merging would not fold them
  __syncthreads();
  uint64_t *reg = p.flush_log + (uint64_t)blockIdx.x * p.log_words;
  const uint32_t total = NE + 4 * p.comb_entries;
  auto entry = [&](uint32_t i, uint64_t &tag, uint64_t &delta) {
    tag = delta = 0;
    if (i < NE) {
      tag = e[2 * i];
      delta = e[2 * i + 1];
    } else if (i < total) {
      comb_counter(i - NE, tag, delta);
    }
  };
  for (uint32_t r0 = 0; r0 < total; r0 += BS) {
    uint64_t tag, delta;
    entry(r0 + tid, tag, delta);
    const uint64_t m = __ballot(tag && delta);
    if ((tid & 63) == 0 && m) atomicAdd(&nlog, (uint32_t)__builtin_popcountll(m));
  }
  __syncthreads();
  const uint32_t used = nlog;
  __syncthreads();
  if (used > kMergeEntries / 8) {
    for (uint32_t i = tid; i < total && !(p.dbg & 1); i += BS) {
      uint64_t tag, delta;
      entry(i, tag, delta);
      flush_delta_tag(tag, delta);
    }
    if (tid == 0) reg[0] = 0;
    return;
  }
  if (tid == 0) nlog = 0;
  __syncthreads();
  for (uint32_t r0 = 0; r0 < total; r0 += BS) {
    uint64_t tag, delta;
    entry(r0 + tid, tag, delta);
    const bool nz = tag && delta;
    const uint64_t m = __ballot(nz);
    uint32_t base = 0;
    if ((tid & 63) == 0 && m) base = atomicAdd(&nlog, (uint32_t)__builtin_popcountll(m));
    base = __builtin_amdgcn_readfirstlane(base);
    if (nz) {
      const uint32_t k = base + (uint32_t)__builtin_popcountll(m & ((1ull << __lane_id()) - 1));
      reg[1 + 2 * k] = tag;
      reg[2 + 2 * k] = delta;
    }
  }
  __syncthreads();
  if (tid == 0) reg[0] = nlog;
}

// Second level of the block-end flush (common.hpp kMergeGroup): block m
// merges the logs of blocks [m * group, (m + 1) * group) in a 4-way LDS table
// and adds each address's sum with one device atomic; an entry whose set is
// full adds at once.
__global__ __launch_bounds__(kBlock) void k_comb_merge(const uint64_t *log, uint32_t log_words, uint32_t nblocks,
                                                       uint32_t group) {
  extern __shared__ __attribute__((aligned(16))) uint64_t mt[];  // tags[kMergeEntries], deltas[kMergeEntries]
  constexpr uint32_t E = kMergeEntries;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 2 * E; i += kBlock) mt[i] = 0;
  __syncthreads();
  const uint32_t b0 = blockIdx.x * group, b1 = min(nblocks, b0 + group);
  for (uint32_t b = b0; b < b1; b++) {
    const uint64_t *reg = log + (uint64_t)b * log_words;
    const uint32_t n = (uint32_t)reg[0];
    for (uint32_t i = tid; i < n; i += kBlock) {
      const uint64_t tag = reg[1 + 2 * i], d = reg[2 + 2 * i];
      const uint32_t set = ((uint32_t)((tag >> 3) * 0x9E3779B1u) >> (32 - 10)) * 4;  // E / 4 = 2^10 sets
      bool done = false;
      for (uint32_t w = 0; w < 4 && !done; w++) {
        uint64_t *t = &mt[set + w];
        uint64_t cur = __hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
          uint64_t z = 0;
          __hip_atomic_compare_exchange_strong(t, &z, tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          cur = z == 0 ? tag : z;
        }
        if (cur == tag) {
          __hip_atomic_fetch_add(&mt[E + set + w], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          done = true;
        }
      }
      if (!done) flush_delta_tag(tag, d);
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < E; i += kBlock) flush_delta_tag(mt[i], mt[E + i]);
}
static_assert(kMergeEntries == 4u << 10, "k_comb_merge hashes into 2^10 sets of 4");

// The miss log's second level (common.hpp kMissParts): block q combines
// partition q of every block's region in an open-addressing LDS table
// (linear probing, kMissProbes slots), then adds each address's sum with
// one device atomic; a record that finds no slot adds at once.
constexpr uint32_t kMissEntries = 4096, kMissProbes = 32;
__global__ __launch_bounds__(kBigBlock) void k_miss_merge(const uint64_t *log, const uint32_t *counts, uint32_t cap,
                                                          uint32_t nblocks, uint64_t lo1, uint64_t hi1, uint64_t lo2,
                                                          uint64_t hi2, uint32_t *bad) {
  __shared__ uint64_t mt[2 * kMissEntries];  // tags, then deltas
  const uint32_t tid = threadIdx.x, q = blockIdx.x;
  for (uint32_t i = tid; i < 2 * kMissEntries; i += kBigBlock) mt[i] = 0;
  __syncthreads();
  // wave w reads source blocks w, w + 16, ...; its lanes read a block's
  // records 64 at a time (coalesced)
  constexpr uint32_t kWaves = kBigBlock / 64;
  for (uint32_t b = tid / 64; b < nblocks; b += kWaves) {
    const uint32_t n = counts[(uint64_t)b * kMissParts + q];
    const uint64_t *rec = log + ((uint64_t)b * kMissParts + q) * cap * 2;
    for (uint32_t i = tid % 64; i < n; i += 64) {
      const uint64_t tag = rec[2 * i], d = rec[2 * i + 1];
      if (!tag || !d) continue;  // (a single add's empty second record)
      // (the windows the interpreter's counter adds may reach: a record
      // outside them is never added)
      const uint64_t a = tag & ~1ull, e = a + ((tag & 1) ? 4 : 8);
      if (!((a >= lo1 && e <= hi1) || (a >= lo2 && e <= hi2))) {
        atomicAdd(bad, 1u);
        continue;
      }
      uint32_t h = (uint32_t)((tag >> 2) * 0x9E3779B97F4A7C15ull >> 52);  // 12 bits
      bool done = false;
      for (uint32_t k = 0; k < kMissProbes && !done; k++, h = (h + 1) & (kMissEntries - 1)) {
        uint64_t cur = __hip_atomic_load(&mt[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
          uint64_t z = 0;
          __hip_atomic_compare_exchange_strong(&mt[h], &z, tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          cur = z == 0 ? tag : z;
        }
        if (cur == tag) {
          __hip_atomic_fetch_add(&mt[kMissEntries + h], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          done = true;
        }
      }
      if (!done) flush_delta_tag(tag, d);
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < kMissEntries; i += kBigBlock) flush_delta_tag(mt[i], mt[kMissEntries + i]);
}

// Thread-ordered syscall dispatch (common.hpp SeqParams; the host side is
// syscall_dispatch.cpp / vm_api.cpp seq_dispatch).  dispatch_syscall
// (attach/syscall_trace_attach_impl/src/syscall_trace_attach_impl.cpp:18-95)
// runs a call's callbacks on the calling thread, one call after another:
// here lane t walks thread t's records in record order and, per record, runs
// the attached programs as that function does -- exit / exit_group run
// nothing; the enter programs (per-syscall, then global) each on a fresh
// zeroed ctx {id, args}; if one overrode the return (58 / 187) the record
// returns it and no exit program runs; else the exit programs each on a
// fresh {id, ret}; the record returns ret or an exit override.  A wave runs
// one attached program at a time over the lanes it applies to, through the
// C++ tier (run_loop: uniform and divergent loops, helpers in between); every
// counter add reaches memory at once (the ORDERED links), so a thread's
// later callbacks see its earlier ones.  Threads are as independent as the
// reference's: different lanes, no order between them.
#ifdef BPFTIME_AMD_SEQ_PROF
// (experiment build only: per-region clock64 sums of k_sys_seq's waves,
// tools/experiments/seq_prof.py)
__device__ unsigned long long g_seqprof[32];
#define SP_NOW() ((uint64_t)clock64())
#define SP_ADD(i, v) sp_acc[i] += (v)
#else
#define SP_NOW() ((uint64_t)0)
#define SP_ADD(i, v) ((void)0)
#endif
__global__ __launch_bounds__(kBlock) void k_sys_seq(SeqParams p) {
#ifdef BPFTIME_AMD_SEQ_PROF
  uint64_t sp_acc[16] = {};
  const uint64_t sp_t0 = SP_NOW();
#endif
  __shared__ uint64_t Rf[12 * kBlock];   // r0..r10 columns, the dummy slot
  __shared__ uint64_t cx[kSeqCtxWords * kBlock];  // the lane's ctx copy (64 B), its caller and clock
  __shared__ uint32_t ovr_st[kBlock];    // override bits of the lane's record (1 enter, 2 exit)
  __shared__ int64_t ovr_v[kBlock];      // ... and the value
  const uint32_t tid = threadIdx.x;
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + tid;
  // the callbacks' stacks: private memory (512 B, the C++ tier), or (p.fast)
  // kLdsStackMax bytes of LDS per lane, which the asm tier addresses, followed
  // by the asm's launch constants (common.hpp seq_lds_bytes)
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  const bool fast = __builtin_amdgcn_readfirstlane(p.fast) != 0;
  uint64_t stk[kStackSize / 8];
  const uint64_t stack_top = fast ? (uint64_t)(uintptr_t)(dyn + (tid + 1) * kLdsStackMax)
                                  : (uint64_t)(uintptr_t)(stk + kStackSize / 8);
  uint64_t *const ctx = &cx[kSeqCtxWords * tid];
  FastEnv fe{};
  if (fast) {
    // tenv all zero (no tail-call frames, ring staging, lookup-cache
    // counters or miss log), no combining table: every asm path that would
    // read them leaves for the C++ tier, and the ORDERED links add to memory
    uint64_t *const tenv = (uint64_t *)(dyn + kBlock * kLdsStackMax);
    for (uint32_t i = tid; i < kTenvBytes / 8; i += kBlock) tenv[i] = 0;
    fe.maps = p.maps;
    fe.comb = sreg((uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(tenv + kTenvBytes / 8)));
    fe.combn = 0;
    fe.head = 0;
    fe.oflags = 0;  // callbacks' return values are not stored (the dispatch ignores them)
    fe.dlo = sreg((uint64_t)0);
    const uint32_t dh = __builtin_amdgcn_readfirstlane(p.checked ? 0u : ~0u);
    fe.dhi = sreg(((uint64_t)dh << 32) | dh);
    fe.alo = p.arena_lo;
    fe.ahi = p.arena_hi;
    fe.shi = sreg((uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)(uintptr_t)&Rf[0] >> 32)));
    fe.phi = fe.shi;
    fe.rb = (uint32_t)(uintptr_t)&Rf[0] + 8 * tid;
    fe.stage = 0;
    fe.ncpu = p.ncpu ? p.ncpu : 1;
    fe.sstep = fe.ustep = 0;
  }
  __syncthreads();
  Ctx c;
  c.R = &Rf[tid];
  // the programs see their ctx copy (LDS), their stack and the map arena
  c.win = Win{0, 0, p.arena_lo, p.arena_hi, 0, 0, p.checked != 0};
  c.dummy = (uint64_t)(uintptr_t)&Rf[11 * kBlock + tid];
  c.verdicts = nullptr;
  c.rets = nullptr;
  c.step_limit = p.step_limit > 0xffffffffull ? 0xffffffffu : (uint32_t)p.step_limit;
  c.c0a = c.c0d = c.c1a = c.c1d = 0;
  c.c0s = c.c1s = 0;
  uint64_t k = 0, end = 0;
  if (t < p.nseg) {
    k = p.seg ? p.seg[t] : 0;
    end = p.seg ? p.seg[t + 1] : p.n;
  }
  const uint32_t nprogs = __builtin_amdgcn_readfirstlane(p.nprogs);
  auto rfl64 = [](uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
  };
  // A record's fields, loaded one record ahead: a lane's records are a chain
  // of dependent memory round trips otherwise (its index, then the fields),
  // which nothing else on the CU hides when the threads are few.  The index
  // is loaded two records ahead.
  const SysLayout &L = p.lay;
  struct Rec {
    uint64_t idx, pid, kt_e, kt_x;
    int64_t nr, ret;
    uint64_t args[6];
  };
  auto perm_at = [&](uint64_t kk) -> uint64_t { return kk < end ? (p.perm ? (uint64_t)p.perm[kk] : kk) : 0; };
  auto fetch = [&](uint64_t kk, uint64_t idx) {
    Rec f;
    const bool h = kk < end;
    const uint8_t *en = L.enter ? L.enter + idx * L.estride : nullptr;
    const uint8_t *ex = L.exit ? L.exit + idx * L.xstride : nullptr;
    const uint8_t *ck = L.clock ? L.clock + idx * L.cstride : nullptr;
    f.idx = idx;
    f.nr = h ? *(const int64_t *)((en ? en : ex) + 8) : 0;
    f.ret = h && ex ? *(const int64_t *)(ex + 16) : 0;
    f.pid = h && L.pid ? *(const uint64_t *)(L.pid + idx * L.pstride) : p.pid_tgid;
    // (the recorded clocks at sys_enter and after the call)
    f.kt_e = h && ck ? *(const uint64_t *)ck : 0;
    f.kt_x = h && ck ? *(const uint64_t *)(ck + 8) : 0;
    for (int w = 0; w < 6; w++) f.args[w] = h && en ? *(const uint64_t *)(en + 16 + 8 * w) : 0;
    return f;
  };
  uint64_t idx_next = perm_at(k + 1);
  Rec cur = fetch(k, perm_at(k));
  while (__ballot(k < end) != 0) {
    uint64_t sp_r = SP_NOW();
    (void)sp_r;
    const bool has = k < end;
    // the next record's fields and the index after it, issued before this
    // record's callbacks run
    const uint64_t idx_next2 = perm_at(k + 2);
    const Rec nxt = fetch(k + 1, idx_next);
    const uint64_t idx = cur.idx;
    const int64_t nr = cur.nr, ret = cur.ret;
    const uint64_t pid = cur.pid, kt_e = cur.kt_e, kt_x = cur.kt_x;
    const bool clk = L.clock != nullptr;
    const bool live = has && nr != 60 && nr != 231;  // :23-26
    ovr_st[tid] = 0;
    ovr_v[tid] = 0;
    for (uint32_t a = 0; a < nprogs; a++) {
      const SeqProg *sp = &p.progs[a];
      const uint32_t enter = __builtin_amdgcn_readfirstlane(sp->enter);
      const int64_t snr = (int64_t)rfl64((uint64_t)sp->sys_nr);
      // an exit program skips a record whose enter programs overrode (:68-72)
      const bool run = live && (snr < 0 || snr == nr) && !(!enter && (ovr_st[tid] & 1));
      if (__ballot(run) == 0) continue;
      // each callback on its own copy of a zeroed ctx (:41-53, :57-66, :80-85)
      if (run) {
        ctx[0] = 0;
        ctx[1] = (uint64_t)nr;
        if (enter) {
          for (int w = 2; w < 8; w++) ctx[w] = cur.args[w - 2];
        } else {
          ctx[2] = (uint64_t)ret;
          for (int w = 3; w < 8; w++) ctx[w] = 0;
        }
        // the asm tier's bpf_get_current_pid_tgid / bpf_ktime_get_ns (CALL_REC)
        ctx[kSeqPidOff / 8] = pid;
        ctx[kSeqClockOff / 8] = clk ? (enter ? kt_e : kt_x) : (uint64_t)__builtin_amdgcn_s_memrealtime() * 10ull;
      }
      SP_ADD(1, SP_NOW() - sp_r);  // record fields + ctx build (first use waits on the loads)
      c.prog = (prog_ptr)rfl64((uint64_t)(uintptr_t)sp->prog);
      c.fast = (const FInsn *)rfl64((uint64_t)(uintptr_t)sp->fast);
      for (int r = 0; r <= 10; r++) c.R[r * kBlock] = 0;
      c.R[1 * kBlock] = (uint64_t)(uintptr_t)ctx;
      c.R[2 * kBlock] = enter ? 64 : 24;  // sizeof the ctx (:46)
      c.R[10 * kBlock] = stack_top;
      c.alive = run;
      c.err = E_OK;
      c.pc = 0;
      c.lpc = 0;
      c.steps = 0;
      c.unit = idx;
      int32_t miss_fd = -1;
      uint64_t miss_hash = 0;
      uint32_t lru_ops = 0;
      bool uni = true;
      // the asm tier's view of the callback: a fresh entry (r1 = the ctx
      // copy, r2 = its size, r10 = the LDS stack top), its ctx loads from the
      // copy through the generic path (no staging), no verdict / ret stores
      FastUnit fu{};
      if (fast) {
        fe.fast = (const FInsn *)rfl64((uint64_t)(uintptr_t)sp->fast);
        fu.r1 = fu.slot = (uint64_t)(uintptr_t)ctx;
        fu.r2 = fu.len = enter ? 64 : 24;
        fu.r10 = stack_top;
        fu.entry = 1u | 4u;  // fresh, lane groups scheduled in asm
        const uint64_t vcpu = idx / 64;
        fu.vm = (uint32_t)(vcpu % fe.ncpu);
      }
      SP_ADD(8, 1);
      while (__ballot(c.alive) != 0) {
        uint64_t sp_i = SP_NOW();
        (void)sp_i;
        uint32_t r;
        if (fast && uni) {
          uint32_t adv = 0;
          fu.entry = (fu.entry & ~256u) | (__ballot(miss_fd >= 0) != 0 ? 256u : 0u);  // (k_interp)
          const uint32_t why = run_fast<false>(c, fe, fu, 0u, adv);
          fu.entry &= ~1u;  // re-entries read the registers from their LDS columns
          if (why == FAST_EXIT) {  // every running lane ran exit
            c.alive = false;
            break;
          }
          if (why == FAST_SPLIT) {  // lane groups at different pcs (c.lpc): the C++ divergent loop
            uni = false;
            continue;
          }
          if (why == FAST_STEPS) {
            c.err = c.alive ? E_STEPS : c.err;
            c.alive = false;
            break;
          }
          r = run_loop<true, true>(c);  // the instruction the asm does not run
        } else {
          r = uni ? run_loop<true>(c) : run_loop<false>(c);
        }
        SP_ADD(2, SP_NOW() - sp_i);
        SP_ADD(uni ? 9 : 10, 1);
        sp_i = SP_NOW();
        if (r == R_STEP) continue;
        if (r == R_DONE) break;
        if (r == R_DIVERGE) {
          uni = false;
          continue;
        }
        if (r == R_RECONV) {
          uni = true;
          continue;
        }
        // R_CALL: the helper (dev_helpers.hpp) for the lanes at the call
        const bool csel = uni ? c.alive : (c.alive && c.lpc == c.call_pc);
        const uint32_t fid = __builtin_amdgcn_readfirstlane(c.call_id);
        if (fid == 5 || fid == 14) {
          // the replay's clock and caller: register values, no helper
          // dispatch (each pass through call_helper costs a lone wave
          // several microseconds of spill traffic: profiles/r06_seq_pmc.txt)
          if (csel) c.R[0] = fid == 14 ? pid : clk ? (enter ? kt_e : kt_x) : (uint64_t)__builtin_amdgcn_s_memrealtime() * 10ull;
        } else if (csel) {
          LaneEnv env;
          env.vcpu = idx / 64;
          env.scratch = 0;
          env.miss_fd = miss_fd;
          env.miss_hash = miss_hash;
          env.lru_stamp = (p.lru_seq << kLruSeqShift) | ((idx & 0xffffffffull) << kLruUnitShift);
          env.lru_ops = lru_ops;
          env.exact = p.exact != 0;
          env.ovr_state = &ovr_st[tid];
          env.ovr_val = &ovr_v[tid];
          env.ovr_bit = enter ? 1 : 2;
          env.pid_tgid = pid;
          env.kt_on = clk;
          env.ktime = enter ? kt_e : kt_x;
          uint32_t cerr = E_OK;
          uint64_t *R = c.R;
          const uint32_t cid = __builtin_amdgcn_readfirstlane(c.call_id);
          const uint64_t rv = cid == kTailHelper ? 0
                              : call_helper(cid, R[1 * kBlock], R[2 * kBlock], R[3 * kBlock], R[4 * kBlock],
                                            R[5 * kBlock], p.maps, p.ncpu, idx ^ ((uint64_t)c.steps << 40), env,
                                            &cerr);
          if (cid == kTailHelper) cerr = E_BADOP;  // (the host refuses such programs)
          R[0] = rv;
          miss_fd = env.miss_fd;
          miss_hash = env.miss_hash;
          lru_ops = env.lru_ops;
          if (cerr != E_OK) {
            c.err = cerr;
            c.alive = false;
          }
        }
        if (uni)
          c.pc = c.call_pc + 1;
        else
          c.lpc = csel ? c.call_pc + 1 : c.lpc;
        {
          const uint64_t sp_d = SP_NOW() - sp_i;
          (void)sp_d;
          SP_ADD(fid == 1 ? 3 : fid == 2 ? 4 : (fid == 5 || fid == 14) ? 5 : 6, sp_d);
          SP_ADD(fid == 1 ? 11 : fid == 2 ? 12 : (fid == 5 || fid == 14) ? 13 : 14, 1);
        }
      }
      // a failed callback is ignored by the dispatch (:47-52) and counted
      if (run && c.err != E_OK) atomicAdd(p.err_count, 1u);
      sp_r = SP_NOW();
    }
    SP_ADD(7, SP_NOW() - sp_r);  // the record's tail (out store, loop)
    if (has && p.out) p.out[idx] = ovr_st[tid] ? ovr_v[tid] : ret;
    if (has) {
      k++;
      cur = nxt;
      idx_next = idx_next2;
    }
  }
#ifdef BPFTIME_AMD_SEQ_PROF
  sp_acc[0] = SP_NOW() - sp_t0;
  sp_acc[15] = c.steps;
  if ((tid & 63) == 0 && __ballot(t < p.nseg) != 0) {
    for (int i = 0; i < 16; i++) atomicAdd(&g_seqprof[i], (unsigned long long)sp_acc[i]);
    atomicAdd(&g_seqprof[16], 1ull);
  }
#endif
}

#ifdef BPFTIME_AMD_SEQ_PROF
extern "C" int bpftime_amd_seq_prof(unsigned long long *out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seqprof), sizeof(g_seqprof)) != hipSuccess) return -1;
  if (reset) {
    static unsigned long long z[32];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_seqprof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// ---------------------------------------------------------------------------
// Host-side launch wrappers
// ---------------------------------------------------------------------------
// block: kBlock, or kBigBlock for G launches without a tail-call image
extern "C" hipError_t bpftime_amd_launch_interp(const KParams *p, uint32_t kind, bool big_stack, uint32_t grid,
                                                uint32_t ordered, uint32_t block, hipStream_t stream) {
  KParams q = *p;
  q.ordered = ordered;
  const bool image = q.tail_entry && !big_stack;
  const bool g_regs = q.gregs && !big_stack;
  if (block != kBlock && (block != kBigBlock || !g_regs || image || ordered)) return hipErrorInvalidValue;
  const size_t dyn = dyn_lds_for(kind, big_stack, p->stack_size, p->comb_entries, p->lcache, !p->gctx, block, p->tail_lds);
  dim3 g(grid), b(block);
#define L(K, B, I, G) hipLaunchKernelGGL((k_interp<K, B, I, G, kBlock>), g, b, dyn, stream, q)
#define LK(K)                                                          \
  if (big_stack) L(K, true, false, false);                             \
  else if (image) { if (g_regs) L(K, false, true, true); else L(K, false, true, false); } \
  else if (g_regs && block == kBigBlock) hipLaunchKernelGGL((k_interp<K, false, false, true, kBigBlock>), g, b, dyn, stream, q); \
  else { if (g_regs) L(K, false, false, true); else L(K, false, false, false); }
  if (kind == CTX_XDP) {
    LK(CTX_XDP)
  } else if (kind == CTX_SYSCALL) {
    LK(CTX_SYSCALL)
  } else {
    LK(CTX_RAW)
  }
#undef LK
#undef L
  return hipGetLastError();
}

// One block of the k_interp instance a launch of these parameters runs, in
// query mode: the asm tier's handler offsets (F_COUNT u32) into d_out
// (kind, big_stack, greg, image select the instance, as in a launch; the
// pointers that select it are never read)
extern "C" hipError_t bpftime_amd_launch_fast_xlat(uint32_t kind, bool big_stack, bool greg, bool image,
                                                   uint32_t *d_out, hipStream_t stream) {
  KParams q{};
  q.dbg = kDbgXlat;
  q.verdicts = d_out;
  q.n = 1;  // (one unit, over the output buffer: nothing reads it)
  q.data = (uint8_t *)d_out;
  q.data_lo = (uint64_t)(uintptr_t)d_out;
  q.data_hi = q.data_lo + 64;
  q.sys_nr = -1;
  q.unwind_idx = -1;
  q.pid_off = 0;
  q.step_limit = 1;
  q.gregs = greg ? (uint64_t *)d_out : nullptr;
  q.tail_entry = image ? (const int32_t *)d_out : nullptr;
  q.stack_size = 8;
  q.stack_stride = lane_stride(8);
  q.ctx_stride = lane_stride(kXdpCtxBytes);
  q.ncpu = 1;
  return bpftime_amd_launch_interp(&q, kind, big_stack, 1, 0, kBlock, stream);
}

extern "C" hipError_t bpftime_amd_launch_sys_seq(const SeqParams *p, hipStream_t stream) {
  const uint64_t grid = (p->nseg + kBlock - 1) / kBlock;
  if (grid == 0 || grid > 0x7fffffffull || p->nprogs > kSeqMaxProgs) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_sys_seq, dim3((uint32_t)grid), dim3(kBlock), seq_lds_bytes(kBlock, p->fast != 0), stream, *p);
  return hipGetLastError();
}

extern "C" hipError_t bpftime_amd_launch_merge(const uint64_t *log, uint32_t log_words, uint32_t nblocks,
                                                hipStream_t stream) {
  const uint32_t grid = (nblocks + kMergeGroup - 1) / kMergeGroup;
  hipLaunchKernelGGL(k_comb_merge, dim3(grid), dim3(kBlock), 2 * kMergeEntries * sizeof(uint64_t), stream, log,
                     log_words, nblocks, kMergeGroup);
  return hipGetLastError();
}

extern "C" hipError_t bpftime_amd_launch_miss_merge(const uint64_t *log, const uint32_t *counts, uint32_t cap,
                                                     uint32_t nblocks, const KParams *p, uint32_t *bad,
                                                     hipStream_t stream) {
  hipLaunchKernelGGL(k_miss_merge, dim3(kMissParts), dim3(kBigBlock), 0, stream, log, counts, cap, nblocks,
                     p->arena_lo, p->arena_hi, p->data_lo, p->data_hi, bad);
  return hipGetLastError();
}

// Static LDS of a k_interp instance (Rf, rb_lds, wdelta, nlog): the
// kernel's own attribute, or (no device) the same sum restated
template <uint32_t KIND, bool BIGSTACK, bool IMAGE, bool G, uint32_t BS>
static size_t static_lds_of() {
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, (const void *)k_interp<KIND, BIGSTACK, IMAGE, G, BS>) == hipSuccess)
    return a.sharedSizeBytes;
  (void)hipGetLastError();
  const size_t rf = (size_t)(IMAGE ? (G ? 2 : 13) : (G ? 1 : 12)) * BS * 8;
  return rf + sizeof(RbLds) + (BS / 64) * 2 * 2 * 8 + 16;
}

// (image: the kernel of a tail-call image, interp.hip bpftime_amd_launch_interp)
extern "C" size_t bpftime_amd_static_lds_image(uint32_t kind, bool big_stack, bool gregs, uint32_t block, bool image) {
#define S(K, B, G, BS) return static_lds_of<K, B, false, G, BS>()
#define SK(K)                                          \
  if (big_stack) S(K, true, false, kBlock);            \
  else if (image) { if (gregs) return static_lds_of<K, false, true, true, kBlock>(); else return static_lds_of<K, false, true, false, kBlock>(); } \
  else if (gregs && block == kBigBlock) S(K, false, true, kBigBlock); \
  else if (gregs) S(K, false, true, kBlock);           \
  else S(K, false, false, kBlock);
  if (kind == CTX_XDP) {
    SK(CTX_XDP)
  } else if (kind == CTX_SYSCALL) {
    SK(CTX_SYSCALL)
  } else {
    SK(CTX_RAW)
  }
#undef SK
#undef S
}

extern "C" size_t bpftime_amd_static_lds(uint32_t kind, bool big_stack, bool gregs, uint32_t block) {
  return bpftime_amd_static_lds_image(kind, big_stack, gregs, block, false);
}

extern "C" size_t bpftime_amd_lds_bytes(uint32_t kind, bool big_stack, uint32_t stack_size, uint32_t comb_entries,
                                        uint32_t lcache_sets, bool ctx_lds, bool gregs, uint32_t block) {
  return dyn_lds_for(kind, big_stack, stack_size, comb_entries, lcache_sets, ctx_lds, block) +
         bpftime_amd_static_lds(kind, big_stack, gregs, block);
}

extern "C" int bpftime_amd_occupancy(uint32_t kind, bool big_stack, size_t dyn_lds, bool gregs, uint32_t block,
                                    bool image) {
  // (a block asking for more LDS than a CU has never fits, whatever the
  // occupancy query answers for it: dynamic plus the kernel's static LDS)
  if (dyn_lds + bpftime_amd_static_lds_image(kind, big_stack, gregs, block, image) > kCuLds) return 0;
  int n = 0;
  hipError_t e;
#define O(K, B, G) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_interp<K, B, false, G, kBlock>, kBlock, dyn_lds)
#define OI(K, G) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_interp<K, false, true, G, kBlock>, kBlock, dyn_lds)
#define OK(K)                         \
  if (big_stack) O(K, true, false);   \
  else if (image) { if (gregs) OI(K, true); else OI(K, false); } \
  else if (gregs && block == kBigBlock) \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_interp<K, false, false, true, kBigBlock>, kBigBlock, dyn_lds); \
  else if (gregs) O(K, false, true);  \
  else O(K, false, false);
  if (kind == CTX_XDP) {
    OK(CTX_XDP)
  } else if (kind == CTX_SYSCALL) {
    OK(CTX_SYSCALL)
  } else {
    OK(CTX_RAW)
  }
#undef OK
#undef OI
#undef O
  return e == hipSuccess ? n : 1;
}

}  // namespace bpftime_amd

#ifdef BPFTIME_AMD_INSERT_STATS
extern "C" int bpftime_amd_insert_stats(uint64_t *out) {
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(out, HIP_SYMBOL(bpftime_amd::g_istats), 64) != hipSuccess)
    return -1;
  static const uint64_t z[8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(bpftime_amd::g_istats), z, 64) == hipSuccess ? 0 : -1;
}
#endif

