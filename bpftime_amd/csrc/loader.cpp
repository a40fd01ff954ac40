// bpftime_amd: program loader (patch -> validate -> pre-decode -> analyse).
//
// Load-time semantics follow bpftime_ubpf_vm::load_code
// (vm/compat/ubpf-vm/compat_ubpf.cpp:61-200): every opcode 0x85 is a helper
// call resolved through the registration map (:75-95, error strings kept),
// lddw src 1..6 are patched through the lddw helpers (:97-190).  Validation
// restates ubpf_load's checks (ubpf itself is absent from the reference).
// The device-specific steps -- decoding to DInsn, fusing ldx/add/stx
// read-modify-writes into one atomic add, sizing the per-lane stack -- are
// described in DESIGN.md §3.
#include "loader.hpp"
#include "runtime.hpp"

#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

namespace bpftime_amd {

bool device_helper_supported(uint32_t id) {
  switch (id) {
    case 1: case 2: case 3: case 5: case 7: case 8: case 28: case 44: case 65: case 189:
    case 130: case 131: case 132: case 133:
    case 58: case 187:  // bpf_override_return / bpf_set_retval (syscall dispatch state)
    case 14:            // bpf_get_current_pid_tgid (recorded caller / launching thread)
    case kTailHelper:
      return true;
  }
  return false;
}

static std::string fmt(const char *f, ...) __attribute__((format(printf, 1, 2)));
static std::string fmt(const char *f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

static inline uint8_t cls(uint8_t c) { return c & 7; }
enum { C_LD = 0, C_LDX, C_ST, C_STX, C_ALU, C_JMP, C_JMP32, C_ALU64 };

static bool opcode_known(uint8_t c) {
  uint8_t k = cls(c), op = c & 0xf0;
  switch (k) {
    case C_ALU:
    case C_ALU64:
      if (op > 0xd0) return false;
      if (op == 0xd0) return k == C_ALU;
      if (op == 0x80) return (c & 0x08) == 0;
      return true;
    case C_JMP:
    case C_JMP32:
      if (op > 0xd0) return false;
      if (k == C_JMP32 && (op == 0x00 || op == 0x80 || op == 0x90)) return false;
      if (op == 0x00 || op == 0x80 || op == 0x90) return (c & 0x08) == 0;
      return true;
    case C_LDX:
    case C_ST:
      return (c & 0xe0) == 0x60;
    case C_STX:
      return (c & 0xe0) == 0x60 ||
             ((c & 0xe0) == 0xc0 && ((c & 0x18) == 0x00 || (c & 0x18) == 0x18));
    case C_LD:
      return c == 0x18;
  }
  return false;
}

static bool writes_dst(uint8_t c) {
  uint8_t k = cls(c);
  return k == C_ALU || k == C_ALU64 || k == C_LDX || c == 0x18;
}

static bool atomic_imm_ok(int32_t imm) {
  switch (imm) {
    case 0x00: case 0x01: case 0x40: case 0x41: case 0x50: case 0x51: case 0xa0: case 0xa1:
    case 0xe1: case 0xf1:
      return true;
  }
  return false;
}

static int validate(const std::vector<RawInsn> &in, std::string &err) {
  const uint32_t n = (uint32_t)in.size();
  for (uint32_t i = 0; i < n; i++) {
    const RawInsn d = in[i];
    if (!opcode_known(d.code)) {
      err = fmt("unknown opcode 0x%02x at PC %u", d.code, i);
      return -1;
    }
    if (d.src > 10) {
      err = fmt("invalid source register at PC %u", i);
      return -1;
    }
    if (d.dst > 10 || (d.dst == 10 && writes_dst(d.code))) {
      err = fmt("invalid destination register at PC %u", i);
      return -1;
    }
    const uint8_t k = cls(d.code);
    if ((k == C_JMP || k == C_JMP32) && d.code != 0x85 && d.code != 0x95) {
      int64_t t = (int64_t)i + 1 + d.off;
      if (t < 0 || t >= (int64_t)n) {
        err = fmt("jump out of bounds at PC %u", i);
        return -1;
      }
      if (t > 0 && in[t - 1].code == 0x18 && in[t].code == 0) {
        err = fmt("jump to middle of lddw at PC %u", i);
        return -1;
      }
    }
    if (k == C_STX && (d.code & 0xe0) == 0xc0 && !atomic_imm_ok(d.imm)) {
      err = fmt("unknown atomic operation 0x%x at PC %u", (unsigned)d.imm, i);
      return -1;
    }
    if (d.code == 0x18) {
      if (i + 1 >= n || in[i + 1].code != 0) {
        err = fmt("incomplete lddw at PC %u", i);
        return -1;
      }
      i++;
    }
  }
  return 0;
}

// ---- pre-decoding ----------------------------------------------------------
static uint8_t size_code(uint8_t c) {
  switch (c & 0x18) {
    case 0x10: return 0;  // B
    case 0x08: return 1;  // H
    case 0x00: return 2;  // W
    default: return 3;    // DW
  }
}

static DInsn decode_one(const std::vector<RawInsn> &in, uint32_t i) {
  const RawInsn r = in[i];
  DInsn d{};
  d.dst = r.dst;
  d.src = r.src;
  d.off = r.off;
  d.imm = r.imm;
  d.tgt = 0;
  d.hi = 0;
  const uint8_t k = cls(r.code), op = r.code & 0xf0;
  const bool srcreg = (r.code & 0x08) != 0;
  if (k == C_ALU || k == C_ALU64) {
    const bool w32 = k == C_ALU;
    d.aux = (srcreg ? A_SRCREG : 0) | (w32 ? A_W32 : 0);
    switch (op) {
      case 0x00: d.op = X_ADD; break;
      case 0x10: d.op = X_SUB; break;
      case 0x20: d.op = X_MUL; break;
      case 0x40: d.op = X_OR; break;
      case 0x50: d.op = X_AND; break;
      case 0xa0: d.op = X_XOR; break;
      case 0xb0: d.op = X_MOV; break;
      case 0x30: d.op = w32 ? X_DIV32 : X_DIV64; break;
      case 0x90: d.op = w32 ? X_MOD32 : X_MOD64; break;
      case 0x60: d.op = w32 ? X_LSH32 : X_LSH64; break;
      case 0x70: d.op = w32 ? X_RSH32 : X_RSH64; break;
      case 0xc0: d.op = w32 ? X_ARSH32 : X_ARSH64; break;
      case 0x80: d.op = w32 ? X_NEG32 : X_NEG64; d.aux &= ~A_SRCREG; break;
      case 0xd0: d.op = srcreg ? X_BE : X_LE; d.aux = 0; break;
      default: d.op = X_BAD;
    }
    return d;
  }
  if (k == C_JMP || k == C_JMP32) {
    d.aux = (srcreg ? A_SRCREG : 0) | (k == C_JMP32 ? A_W32 : 0);
    d.tgt = (uint16_t)(i + 1 + r.off);
    switch (op) {
      case 0x00: d.op = X_JA; d.aux = 0; break;
      case 0x10: d.op = X_JEQ; break;
      case 0x20: d.op = X_JGT; break;
      case 0x30: d.op = X_JGE; break;
      case 0x40: d.op = X_JSET; break;
      case 0x50: d.op = X_JNE; break;
      case 0x60: d.op = X_JSGT; break;
      case 0x70: d.op = X_JSGE; break;
      case 0xa0: d.op = X_JLT; break;
      case 0xb0: d.op = X_JLE; break;
      case 0xc0: d.op = X_JSLT; break;
      case 0xd0: d.op = X_JSLE; break;
      case 0x80: d.op = X_CALL; d.hi = r.imm; d.aux = 0; d.tgt = 0; break;
      case 0x90: d.op = X_EXIT; d.aux = 0; d.tgt = 0; break;
      default: d.op = X_BAD;
    }
    return d;
  }
  const uint8_t sz = (uint8_t)(size_code(r.code) << A_SIZE_SHIFT);
  if (k == C_LDX) {
    d.op = X_LDX;
    d.aux = sz;
    return d;
  }
  if (k == C_ST) {
    d.op = X_ST;
    d.aux = sz;
    return d;
  }
  if (k == C_STX) {
    if ((r.code & 0xe0) == 0xc0) {
      d.op = X_ATOMIC;
      d.aux = sz;
      d.hi = r.imm;
    } else {
      d.op = X_STX;
      d.aux = sz;
    }
    return d;
  }
  if (r.code == 0x18) {
    d.op = X_LDDW;
    d.imm = r.imm;
    d.hi = in[i + 1].imm;
    return d;
  }
  d.op = X_BAD;
  return d;
}

// ---- analysis --------------------------------------------------------------
// Argument count of each device helper (linux/bpf.h prototypes).
static int helper_arity(uint32_t id) {
  switch (id) {
    case 5: case 7: case 8: return 0;          // ktime_get_ns, get_prandom_u32, get_smp_processor_id
    case 1: case 3: case 44: case 65: return 2;  // map_lookup/delete_elem, xdp_adjust_head/tail
    case 2: case 189: return 4;                // map_update_elem, xdp_load_bytes
    case kTailHelper: return 3;                // tail_call(ctx, prog_array, index)
    case (uint32_t)kRetHelper: return 0;       // a linked tail-call target's exit
    default: return 5;                         // csum_diff and anything else
  }
}

typedef uint16_t RegSet;  // bit per register r0..r10

static void use_def(const DInsn &d, RegSet &use, RegSet &def) {
  use = def = 0;
  auto U = [&](int r) { use |= (RegSet)(1u << r); };
  auto D = [&](int r) { def |= (RegSet)(1u << r); };
  switch (d.op) {
    case X_MOV:
      if (d.aux & A_SRCREG) U(d.src);
      D(d.dst);
      break;
    case X_ADD: case X_SUB: case X_MUL: case X_OR: case X_AND: case X_XOR: case X_DIV64:
    case X_MOD64: case X_LSH64: case X_RSH64: case X_ARSH64: case X_DIV32: case X_MOD32:
    case X_LSH32: case X_RSH32: case X_ARSH32:
      U(d.dst);
      if (d.aux & A_SRCREG) U(d.src);
      D(d.dst);
      break;
    case X_NEG64: case X_NEG32: case X_LE: case X_BE:
      U(d.dst);
      D(d.dst);
      break;
    case X_LDX: U(d.src); D(d.dst); break;
    case X_ST: U(d.dst); break;
    case X_STX: U(d.dst); U(d.src); break;
    case X_ATOMIC:
      U(d.dst);
      U(d.src);
      if (d.hi == 0xf1) {
        U(0);
        D(0);
      } else if (d.hi & 1) {
        D(d.src);
      }
      break;
    case X_LDDW: D(d.dst); break;
    case X_JA: break;
    case X_JEQ: case X_JGT: case X_JGE: case X_JSET: case X_JNE: case X_JSGT: case X_JSGE:
    case X_JLT: case X_JLE: case X_JSLT: case X_JSLE:
      U(d.dst);
      if (d.aux & A_SRCREG) U(d.src);
      break;
    case X_CALL:
      // a helper reads only its declared arguments; r1-r5 survive the call
      // (ubpf semantics, restated by oracle/interp.c: helpers get copies)
      for (int r = 1; r <= helper_arity((uint32_t)d.hi); r++) U(r);
      if (d.hi == kRetHelper) U(0);
      D(0);
      break;
    case X_EXIT: U(0); break;
    case X_RMW_ADD:
      U(d.dst);
      if (d.aux & A_SRCREG) U(d.src);
      if (d.aux & A_FETCH) D(d.hi);
      break;
    default: break;
  }
}

static void successors(const std::vector<DInsn> &p, uint32_t i, uint32_t s[2], int &ns) {
  const DInsn &d = p[i];
  ns = 0;
  switch (d.op) {
    case X_EXIT: return;
    case X_CALL:
      if (d.hi == kRetHelper) return;  // a linked target's exit
      if (i + 1 < p.size()) s[ns++] = i + 1;
      return;
    case X_JA: s[ns++] = d.tgt; return;
    case X_RMW_ADD: if (d.tgt < p.size()) s[ns++] = d.tgt; return;
    case X_LDDW: if (i + 2 < p.size()) s[ns++] = i + 2; return;
    case X_JEQ: case X_JGT: case X_JGE: case X_JSET: case X_JNE: case X_JSGT: case X_JSGE:
    case X_JLT: case X_JLE: case X_JSLT: case X_JSLE:
      if (i + 1 < p.size()) s[ns++] = i + 1;
      s[ns++] = d.tgt;
      return;
    default:
      if (i + 1 < p.size()) s[ns++] = i + 1;
  }
}

// Stack lattice per register: UNDEF, FP+k, OTHER, TOP
struct SVal {
  uint8_t kind;  // 0 undef, 1 fp, 2 other, 3 top
  int32_t k;
  bool operator==(const SVal &o) const { return kind == o.kind && (kind != 1 || k == o.k); }
};
static SVal join(SVal a, SVal b) {
  if (a.kind == 0) return b;
  if (b.kind == 0) return a;
  if (a == b) return a;
  if (a.kind == 2 && b.kind == 2) return a;
  return SVal{3, 0};
}

// Returns per-lane stack bytes needed, or -1 if accesses cannot be bounded.
static int stack_depth(const std::vector<DInsn> &p, const std::vector<bool> &reach) {
  const uint32_t n = (uint32_t)p.size();
  std::vector<std::vector<SVal>> in(n, std::vector<SVal>(11, SVal{0, 0}));
  std::vector<bool> queued(n, false);
  std::vector<uint32_t> work;
  for (int r = 0; r < 11; r++) in[0][r] = SVal{2, 0};
  in[0][10] = SVal{1, 0};
  work.push_back(0);
  queued[0] = true;
  int64_t lowest = 0;  // most negative byte offset from fp touched
  bool escape = false;
  auto touch = [&](int64_t lo) { lowest = std::min(lowest, lo); };
  while (!work.empty()) {
    uint32_t i = work.back();
    work.pop_back();
    queued[i] = false;
    std::vector<SVal> st = in[i];
    const DInsn &d = p[i];
    auto base_access = [&](int reg, int sz) {
      SVal b = st[reg];
      if (b.kind == 1) touch((int64_t)b.k + d.off);
      else if (b.kind == 3) escape = true;
      (void)sz;
    };
    switch (d.op) {
      case X_MOV:
        st[d.dst] = (d.aux & A_SRCREG) ? ((d.aux & A_W32) ? SVal{2, 0} : st[d.src]) : SVal{2, 0};
        break;
      case X_ADD:
      case X_SUB:
        if (st[d.dst].kind == 1 && !(d.aux & A_SRCREG) && !(d.aux & A_W32)) {
          int64_t k = (int64_t)st[d.dst].k + (d.op == X_ADD ? (int64_t)d.imm : -(int64_t)d.imm);
          if (k < -65536 || k > 65536) escape = true;
          st[d.dst] = SVal{1, (int32_t)k};
          touch(k);
        } else {
          if (st[d.dst].kind == 1 || st[d.dst].kind == 3) escape = true;
          if ((d.aux & A_SRCREG) && (st[d.src].kind == 1 || st[d.src].kind == 3)) escape = true;
          st[d.dst] = SVal{2, 0};
        }
        break;
      case X_LDX:
        base_access(d.src, 0);
        st[d.dst] = SVal{2, 0};
        break;
      case X_ST:
        base_access(d.dst, 0);
        break;
      case X_RMW_ADD:
        base_access(d.dst, 0);
        if ((d.aux & A_SRCREG) && (st[d.src].kind == 1 || st[d.src].kind == 3)) escape = true;
        if (d.aux & A_FETCH) st[d.hi] = SVal{2, 0};
        break;
      case X_STX:
        base_access(d.dst, 0);
        if (st[d.src].kind == 1 || st[d.src].kind == 3) escape = true;  // fp value spilled
        break;
      case X_ATOMIC:
        base_access(d.dst, 0);
        if (st[d.src].kind == 1 || st[d.src].kind == 3) escape = true;
        if (d.hi == 0xf1) st[0] = SVal{2, 0};
        else if (d.hi & 1) st[d.src] = SVal{2, 0};
        break;
      case X_CALL:
        for (int r = 1; r <= 5; r++)
          if (st[r].kind == 1) touch(st[r].k);
          else if (st[r].kind == 3) escape = true;
        st[0] = SVal{2, 0};
        break;
      case X_EXIT:
      case X_JA:
        break;
      case X_JEQ: case X_JGT: case X_JGE: case X_JSET: case X_JNE: case X_JSGT: case X_JSGE:
      case X_JLT: case X_JLE: case X_JSLT: case X_JSLE:
        break;
      default: {
        RegSet u, df;
        use_def(d, u, df);
        for (int r = 0; r < 11; r++)
          if (df & (1u << r)) {
            if (st[r].kind == 1 || st[r].kind == 3) {
              // an fp-derived value transformed by other arithmetic
              if (u & (1u << r)) escape = true;
            }
            st[r] = SVal{2, 0};
          }
        break;
      }
    }
    uint32_t s[2];
    int ns;
    successors(p, i, s, ns);
    for (int j = 0; j < ns; j++) {
      uint32_t t = s[j];
      bool changed = false;
      for (int r = 0; r < 11; r++) {
        SVal nv = join(in[t][r], st[r]);
        if (!(nv == in[t][r])) {
          in[t][r] = nv;
          changed = true;
        }
      }
      if (changed && !queued[t]) {
        queued[t] = true;
        work.push_back(t);
      }
    }
  }
  (void)reach;
  if (escape) return -1;
  int64_t depth = -lowest;
  if (depth > kStackSize) return -1;
  return (int)depth;
}

int load_program(const RawInsn *code, size_t n, const std::map<size_t, size_t> &helper_id_map,
                 const std::map<size_t, std::string> &helper_names, const LddwHelpers &lddw,
                 LoadOut &out, std::string &err, const std::vector<uint32_t> &entries) {
  if (n > kMaxInsts) {
    err = fmt("too many instructions (max %u)", kMaxInsts);
    return -1;
  }
  std::vector<RawInsn> in(code, code + n);
  out.lddw_src.assign(n, 0);
  // compat_ubpf.cpp:72-190
  for (size_t i = 0; i < n; i++) {
    RawInsn &cur = in[i];
    if (cur.code == 0x85 && cur.imm == kRetHelper && !entries.empty()) {
      // linked image (vm_api.cpp link_tail_image): a target's exit
    } else if (cur.code == 0x85) {
      if (cur.imm == (int32_t)kTailHelper) out.tail_call = true;
      if (helper_id_map.find((size_t)(uint32_t)cur.imm) == helper_id_map.end() || cur.imm < 0) {
        if (cur.imm >= 64) {
          err = "invalid call immediate at PC " + std::to_string(i);
        } else {
          err = "call to nonexistent function " + std::to_string(cur.imm) + " at PC " + std::to_string(i);
        }
        return -EINVAL;
      }
      if (!device_helper_supported((uint32_t)cur.imm)) {
        auto it = helper_names.find((size_t)cur.imm);
        err = "helper " + std::to_string(cur.imm) + " (" + (it != helper_names.end() ? it->second : "?") +
              ") has no device implementation at PC " + std::to_string(i);
        return -EINVAL;
      }
      if (cur.imm == 3) out.may_delete = true;
      if (cur.imm == 58 || cur.imm == 187) out.sets_retval = true;
    } else if (cur.code == 0x18) {
      if (i + 1 == n) {
        err = "Unable to patch lddw instructions at " + std::to_string(i) + ", it's the last instruction";
        return -EINVAL;
      }
      RawInsn &nx = in[i + 1];
      uint64_t imm;
      const std::string at = "Unable to patch lddw instruction at " + std::to_string(i);
      switch (cur.src) {
        case 0:
          imm = (uint64_t)(uint32_t)cur.imm | ((uint64_t)(uint32_t)nx.imm << 32);
          break;
        case 1:
          if (!lddw.map_by_fd) { err = at + ", map_by_fd not defined"; return -EINVAL; }
          imm = lddw.map_by_fd((uint32_t)cur.imm);
          break;
        case 2:
          if (!lddw.map_by_fd || !lddw.map_val) { err = at + ", map_by_fd or map_val not defined"; return -EINVAL; }
          imm = lddw.map_val(lddw.map_by_fd((uint32_t)cur.imm)) + (uint64_t)(int64_t)nx.imm;
          break;
        case 3:
          if (!lddw.var_addr) { err = at + ", var_addr not defined"; return -EINVAL; }
          imm = lddw.var_addr((uint32_t)cur.imm);
          break;
        case 4:
          if (!lddw.code_addr) { err = at + ", code_addr not defined"; return -EINVAL; }
          imm = lddw.code_addr((uint32_t)cur.imm);
          break;
        case 5:
          if (!lddw.map_by_idx) { err = at + ", map_by_idx not defined"; return -EINVAL; }
          imm = lddw.map_by_idx((uint32_t)cur.imm);
          break;
        case 6:
          if (!lddw.map_by_idx || !lddw.map_val) { err = at + ", map_by_idx or map_val not defined"; return -EINVAL; }
          imm = lddw.map_val(lddw.map_by_idx((uint32_t)cur.imm)) + (uint64_t)(int64_t)nx.imm;
          break;
        default:
          err = at + ", unsupported src_reg " + std::to_string(cur.src);
          return -EINVAL;
      }
      cur.imm = (int32_t)(uint32_t)(imm & 0xffffffffu);
      nx.imm = (int32_t)(uint32_t)(imm >> 32);
      out.lddw_src[i] = cur.src;
      cur.src = 0;
      i++;
    }
  }
  if (validate(in, err) < 0) return -1;
  if (n == 0) {
    err = "no instructions";
    return -1;
  }

  // pre-decode
  std::vector<DInsn> p(n);
  for (uint32_t i = 0; i < n; i++) {
    if (in[i].code == 0x18) {
      p[i] = decode_one(in, i);
      p[i + 1] = DInsn{};
      p[i + 1].op = X_NOP;
      i++;
    } else {
      p[i] = decode_one(in, i);
    }
  }

  // reachability + jump-target marks
  std::vector<bool> reach(n, false), is_target(n, false);
  {
    std::vector<uint32_t> st{0};
    reach[0] = true;
    for (uint32_t e : entries)  // linked tail-call targets
      if (e < n && !reach[e]) {
        reach[e] = true;
        st.push_back(e);
      }
    while (!st.empty()) {
      uint32_t i = st.back();
      st.pop_back();
      uint32_t s[2];
      int ns;
      successors(p, i, s, ns);
      for (int j = 0; j < ns; j++) {
        if (s[j] != i + 1 && !(p[i].op == X_LDDW && s[j] == i + 2)) is_target[s[j]] = true;
        if (!reach[s[j]]) {
          reach[s[j]] = true;
          st.push_back(s[j]);
        }
      }
    }
  }

  // liveness (backward, to fixpoint)
  std::vector<RegSet> live_in(n, 0), live_out(n, 0);
  for (bool changed = true; changed;) {
    changed = false;
    for (int64_t i = (int64_t)n - 1; i >= 0; i--) {
      if (!reach[i]) continue;
      uint32_t s[2];
      int ns;
      successors(p, (uint32_t)i, s, ns);
      RegSet o = 0;
      for (int j = 0; j < ns; j++) o |= live_in[s[j]];
      RegSet u, d;
      use_def(p[i], u, d);
      RegSet li = (RegSet)(u | (o & ~d));
      if (li != live_in[i] || o != live_out[i]) {
        live_in[i] = li;
        live_out[i] = o;
        changed = true;
      }
    }
  }

  // what a tail-call frame must keep of its caller's registers
  out.tail_live.assign(n, 0);
  for (uint32_t i = 0; i + 1 < n; i++)
    if (reach[i] && p[i].op == X_CALL && p[i].hi == (int32_t)kTailHelper)
      out.tail_live[i] = (uint16_t)(live_in[i + 1] & 0x3fe);

  // RMW fusion: ldx r,[b+o]; add r,v; stx [b+o],r is one atomic add (the
  // reference's ld/add/st is not atomic, but it runs one unit at a time: a
  // parallel batch needs the add to be indivisible to give the same total).
  // r dead after the stx: a plain add; r live: a fetch-add that also leaves
  // old + v in r (A_FETCH), which is what the three instructions compute.
  uint32_t fused = 0;
  for (uint32_t i = 0; i + 2 < n; i++) {
    const DInsn &a = p[i], &b = p[i + 1], &c = p[i + 2];
    if (a.op != X_LDX || b.op != X_ADD || c.op != X_STX) continue;
    const uint32_t sz = (a.aux >> A_SIZE_SHIFT) & 3;
    if (sz < 2) continue;                                   // 4 / 8 byte counters
    if (sz == 3 && (b.aux & A_W32)) continue;               // 32-bit add on a u64 value
    if (((c.aux >> A_SIZE_SHIFT) & 3) != sz) continue;
    const uint8_t r = a.dst, base = a.src;
    if (r == base || b.dst != r || c.src != r || c.dst != base || c.off != a.off) continue;
    if ((b.aux & A_SRCREG) && b.src == r) continue;
    if (is_target[i + 1] || is_target[i + 2]) continue;
    const bool fetch = (live_out[i + 2] & (1u << r)) != 0;
    DInsn f{};
    f.op = X_RMW_ADD;
    f.dst = base;
    f.off = a.off;
    f.aux = (uint8_t)((sz << A_SIZE_SHIFT) | (b.aux & A_SRCREG) | (fetch ? (A_FETCH | (b.aux & A_W32)) : 0));
    f.src = b.src;
    f.imm = b.imm;
    f.hi = r;
    f.tgt = (uint16_t)(i + 3);
    p[i] = f;
    fused++;
    i += 2;
  }

  int depth = entries.empty() ? stack_depth(p, reach) : -1;  // an image: every program on a 512-B stack
  out.multi_entry = !entries.empty();
  out.entries = entries;
  if (depth < 0 || depth > (int)kLdsStackMax) {
    out.big_stack = true;
    out.stack_size = kStackSize;
  } else {
    out.big_stack = false;
    out.stack_size = (uint32_t)std::max(8, (depth + 7) & ~7);
  }
  out.fused_rmw = fused;
  // sentinel: a program that falls off its end fails its lanes on the device
  // instead of fetching past the allocation
  // (two of them: the device prefetches pc + 1)
  DInsn sentinel{};
  sentinel.op = X_BAD;
  p.push_back(sentinel);
  p.push_back(sentinel);
  out.prog = std::move(p);
  return 0;
}

}  // namespace bpftime_amd

namespace bpftime_amd {

static uint32_t fast_id(const DInsn &d) {
  const bool r = (d.aux & A_SRCREG) != 0;
  const bool w32 = (d.aux & A_W32) != 0;
  const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
  auto alu = [&](uint32_t r64, uint32_t i64, uint32_t r32, uint32_t i32) {
    return w32 ? (r ? r32 : i32) : (r ? r64 : i64);
  };
  auto by_size = [&](uint32_t s1, uint32_t s2, uint32_t s4, uint32_t s8) {
    return sz == 1 ? s1 : sz == 2 ? s2 : sz == 4 ? s4 : s8;
  };
#define ALU4(OP) alu(F_A64_##OP##_R, F_A64_##OP##_I, F_A32_##OP##_R, F_A32_##OP##_I)
#define JCC(CC) alu(F_J64_##CC##_R, F_J64_##CC##_I, F_J32_##CC##_R, F_J32_##CC##_I)
  switch (d.op) {
    case X_ADD: return ALU4(ADD);
    case X_SUB: return ALU4(SUB);
    case X_MUL: return ALU4(MUL);
    case X_OR: return ALU4(OR);
    case X_AND: return ALU4(AND);
    case X_XOR: return ALU4(XOR);
    case X_MOV: return ALU4(MOV);
    case X_LSH64: return r ? F_A64_LSH_R : F_A64_LSH_I;
    case X_RSH64: return r ? F_A64_RSH_R : F_A64_RSH_I;
    case X_ARSH64: return r ? F_A64_ARSH_R : F_A64_ARSH_I;
    case X_LSH32: return r ? F_A32_LSH_R : F_A32_LSH_I;
    case X_RSH32: return r ? F_A32_RSH_R : F_A32_RSH_I;
    case X_ARSH32: return r ? F_A32_ARSH_R : F_A32_ARSH_I;
    case X_NEG64: return F_A64_NEG;
    case X_NEG32: return F_A32_NEG;
    case X_LE: return d.imm == 16 ? F_LE16 : d.imm == 32 ? F_LE32 : d.imm == 64 ? F_NOP : F_SLOW;
    case X_BE: return d.imm == 16 ? F_BE16 : d.imm == 32 ? F_BE32 : d.imm == 64 ? F_BE64 : F_SLOW;
    case X_LDX: return by_size(F_LDX1, F_LDX2, F_LDX4, F_LDX8);
    case X_STX: return by_size(F_STX1, F_STX2, F_STX4, F_STX8);
    case X_ST: return by_size(F_ST1, F_ST2, F_ST4, F_ST8);
    case X_LDDW: return F_LDDW;
    case X_JA: return F_JA;
    case X_JEQ: return JCC(EQ);
    case X_JGT: return JCC(GT);
    case X_JGE: return JCC(GE);
    case X_JSET: return JCC(SET);
    case X_JNE: return JCC(NE);
    case X_JSGT: return JCC(SGT);
    case X_JSGE: return JCC(SGE);
    case X_JLT: return JCC(LT);
    case X_JLE: return JCC(LE);
    case X_JSLT: return JCC(SLT);
    case X_JSLE: return JCC(SLE);
    case X_CALL: return d.hi == 1 ? F_CALL_LOOKUP : F_SLOW;  // map_lookup_elem; other helpers in C++
    case X_EXIT: return F_EXIT;
    case X_ATOMIC: {
      const uint32_t aop = (uint32_t)d.hi & ~1u, fetch = (uint32_t)d.hi & 1u;
      if (sz != 4 && sz != 8) return F_SLOW;
      static const uint32_t t4[4][2] = {{F_ATOM4_ADD, F_ATOM4_ADD_F}, {F_ATOM4_OR, F_ATOM4_OR_F},
                                        {F_ATOM4_AND, F_ATOM4_AND_F}, {F_ATOM4_XOR, F_ATOM4_XOR_F}};
      static const uint32_t t8[4][2] = {{F_ATOM8_ADD, F_ATOM8_ADD_F}, {F_ATOM8_OR, F_ATOM8_OR_F},
                                        {F_ATOM8_AND, F_ATOM8_AND_F}, {F_ATOM8_XOR, F_ATOM8_XOR_F}};
      const int k = aop == 0x00 ? 0 : aop == 0x40 ? 1 : aop == 0x50 ? 2 : aop == 0xa0 ? 3 : -1;
      if (k < 0) return F_SLOW;  // xchg / cmpxchg
      return sz == 8 ? t8[k][fetch] : t4[k][fetch];
    }
    case X_RMW_ADD:
      return sz == 8 ? (r ? F_RMW8_R : F_RMW8_I) : sz == 4 ? (r ? F_RMW4_R : F_RMW4_I) : F_SLOW;
    default: return F_SLOW;  // div/mod, atomics
  }
#undef ALU4
#undef JCC
}


// ---------------------------------------------------------------------------
// Pointer kinds for the fast path (a small slice of what the kernel verifier
// tracks): which registers hold the unit's slot, its packet data, its XDP
// ctx, its stack, a map or a map value, at a constant offset.  A load/store
// whose base has such a kind gets a handler that needs no per-lane window
// check: packet / slot bytes come from the staged VGPRs (link_fast), ctx
// fields are computed from the unit's slot / length, stack bytes are plain
// LDS accesses, map values are plain global accesses.
// ---------------------------------------------------------------------------
// P_CONST: an lddw immediate (id = its pc) plus a constant offset k: a
// wave-uniform constant, counters behind it need no combining.  P_MAPFD: lddw
// of a map fd (id = the fd, as map_ptr_by_fd yields it).  P_MVNULL: the
// result of map_lookup_elem before its null check; P_MAPVAL after it (id =
// fd, k = offset into the value).  Map fds are bound at load time, as the
// kernel binds BPF_PSEUDO_MAP_FD.
enum PKind : uint8_t { P_UNDEF = 0, P_CTX, P_PKT, P_SLOT, P_STK, P_CONST, P_MAPFD, P_MVNULL, P_MAPVAL, P_OTHER };
struct PVal {
  uint8_t kind;
  int32_t k;
  int32_t id;
  bool operator==(const PVal &o) const { return kind == o.kind && k == o.k && id == o.id; }
};
static const PVal kOther{P_OTHER, 0, 0};
static PVal pjoin(PVal a, PVal b) {
  if (a.kind == P_UNDEF) return b;
  if (b.kind == P_UNDEF) return a;
  return a == b ? a : kOther;
}

static const MapRec *map_rec(int64_t fd) {
  Runtime &r = rt();
  if (fd < 0 || fd >= (int64_t)kMaxFds || r.kind[fd] != HKind::MAP) return nullptr;
  return &r.maps[fd];
}

// the array map whose storage holds [a, a+sz) (map_val addresses), or -1
static int32_t array_fd_of(uint64_t a, uint32_t sz) {
  Runtime &r = rt();
  for (uint32_t fd = 0; fd < kMaxFds; fd++) {
    if (r.kind[fd] != HKind::MAP) continue;
    const MapRec &m = r.maps[fd];
    if (m.type != MT_ARRAY && m.type != MT_PERCPU_ARRAY) continue;
    if (a >= m.d.data && a + sz <= m.d.data + m.bytes) return (int32_t)fd;
  }
  return -1;
}

// [a, a+sz) inside the storage of an array map (map_val addresses)
static bool in_array_storage(uint64_t a, uint32_t sz) {
  Runtime &r = rt();
  for (uint32_t fd = 0; fd < kMaxFds; fd++) {
    if (r.kind[fd] != HKind::MAP) continue;
    const MapRec &m = r.maps[fd];
    if (m.type != MT_ARRAY && m.type != MT_PERCPU_ARRAY) continue;
    if (a >= m.d.data && a + sz <= m.d.data + m.bytes) return true;
  }
  return false;
}

static bool is_cond_jump(uint8_t op) { return op >= X_JEQ && op <= X_JSLE; }

// in[i][r]: kind of register r before instruction i; returns false when the
// program may rewrite its ctx (then no ctx / packet kinds are trusted).
//
// A linked tail-call image (vm_api.cpp) also enters at every target: with r1
// = the ctx the caller passed (`ctx_entries`: the caller's own ctx / slot at
// every tail-call site, checked by the caller of this function), r2 = 64, r10
// = the same stack top.  Only stores that can move the packet pointers (ctx
// data / data_end / buffer_start / buffer_end) make the ctx untrusted; a
// target that rewrites other fields of its ctx copy gets them back restored.
static bool pointer_kinds(const std::vector<DInsn> &p, const std::vector<uint8_t> &lddw_src, bool xdp,
                          bool pkt_ok, std::vector<std::vector<PVal>> &in,
                          const std::vector<uint32_t> &entries = {}, bool ctx_entries = false) {
  const uint32_t n = (uint32_t)p.size();
  in.assign(n, std::vector<PVal>(11, PVal{P_UNDEF, 0, 0}));
  std::vector<bool> queued(n, false);
  std::vector<uint32_t> work;
  const PVal ctx0 = xdp ? PVal{P_CTX, 0, 0} : PVal{P_SLOT, 0, 0};
  auto seed = [&](uint32_t e, bool ctx) {
    for (int r = 0; r < 11; r++) in[e][r] = kOther;
    in[e][1] = ctx ? ctx0 : kOther;
    in[e][10] = PVal{P_STK, 0, 0};
    work.push_back(e);
    queued[e] = true;
  };
  seed(0, true);
  for (uint32_t e : entries)
    if (e < n && !queued[e]) seed(e, ctx_entries);
  bool ctx_written = false;
  // a store to [at, at + sz) of the ctx: does it reach a packet pointer field?
  auto moves_pkt = [&](const PVal &b, int64_t off, uint32_t sz) {
    if (b.kind != P_CTX) return false;
    const int64_t at = (int64_t)b.k + off;
    auto hit = [&](int64_t lo, int64_t hi) { return at < hi && lo < at + (int64_t)sz; };
    return hit(0, 16) || hit(32, 48);
  };
  auto ptr = [](uint8_t k) {
    return k == P_CTX || k == P_PKT || k == P_SLOT || k == P_STK || k == P_CONST || k == P_MAPVAL;
  };
  while (!work.empty()) {
    const uint32_t i = work.back();
    work.pop_back();
    queued[i] = false;
    std::vector<PVal> st = in[i];
    const DInsn &d = p[i];
    const bool w32 = (d.aux & A_W32) != 0, sreg = (d.aux & A_SRCREG) != 0;
    switch (d.op) {
      case X_MOV:
        st[d.dst] = (sreg && !w32) ? st[d.src] : kOther;
        break;
      case X_ADD:
      case X_SUB:
        if (ptr(st[d.dst].kind) && !sreg && !w32) {
          const int64_t k = (int64_t)st[d.dst].k + (d.op == X_ADD ? (int64_t)d.imm : -(int64_t)d.imm);
          st[d.dst] = (k > -(1 << 20) && k < (1 << 20)) ? PVal{st[d.dst].kind, (int32_t)k, st[d.dst].id} : kOther;
        } else {
          st[d.dst] = kOther;
        }
        break;
      case X_LDX: {
        const PVal b = st[d.src];
        const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
        PVal v = kOther;
        if (b.kind == P_CTX && sz == 8) {
          const int64_t at = (int64_t)b.k + d.off;
          if (at == 0 && pkt_ok) v = PVal{P_PKT, 0, 0};        // ctx->data
          else if (at == 32) v = PVal{P_SLOT, 0, 0};           // ctx->buffer_start
        }
        st[d.dst] = v;
        break;
      }
      case X_ST:
      case X_STX:
        if (moves_pkt(st[d.dst], d.off, 1u << ((d.aux >> A_SIZE_SHIFT) & 3))) ctx_written = true;
        break;
      case X_RMW_ADD:
        if (moves_pkt(st[d.dst], d.off, 1u << ((d.aux >> A_SIZE_SHIFT) & 3))) ctx_written = true;
        if (d.aux & A_FETCH) st[d.hi] = kOther;
        break;
      case X_ATOMIC:
        if (moves_pkt(st[d.dst], d.off, 1u << ((d.aux >> A_SIZE_SHIFT) & 3))) ctx_written = true;
        if (d.hi == 0xf1) st[0] = kOther;
        else if (d.hi & 1) st[d.src] = kOther;
        break;
      case X_CALL: {
        // r1-r5 survive (ubpf); a lookup on a bound map yields a nullable value pointer
        const PVal m = st[1];
        st[0] = (d.hi == 1 && m.kind == P_MAPFD && map_rec(m.id)) ? PVal{P_MVNULL, 0, m.id} : kOther;
        break;
      }
      case X_LDDW: {
        const uint64_t v = (uint64_t)(uint32_t)d.imm | ((uint64_t)(uint32_t)d.hi << 32);
        const bool fd = i < lddw_src.size() && lddw_src[i] == 1 && v < kMaxFds;
        st[d.dst] = fd ? PVal{P_MAPFD, 0, (int32_t)v} : PVal{P_CONST, 0, (int32_t)i};
        break;
      }
      case X_EXIT: case X_JA: case X_JEQ: case X_JGT: case X_JGE: case X_JSET: case X_JNE:
      case X_JSGT: case X_JSGE: case X_JLT: case X_JLE: case X_JSLT: case X_JSLE:
        break;
      default: {
        RegSet u, df;
        use_def(d, u, df);
        for (int r = 0; r < 11; r++)
          if (df & (1u << r)) st[r] = kOther;
        break;
      }
    }
    uint32_t sx[2];
    int ns;
    successors(p, i, sx, ns);
    // null check of a lookup result: `if (r == 0)` / `if (r != 0)` refines r
    // to a map-value pointer on the non-null edge
    const bool nullchk = (d.op == X_JEQ || d.op == X_JNE) && !sreg && !w32 && d.imm == 0 &&
                         st[d.dst].kind == P_MVNULL && d.tgt != i + 1;
    for (int j = 0; j < ns; j++) {
      const uint32_t t = sx[j];
      std::vector<PVal> edge;
      const std::vector<PVal> *src = &st;
      if (nullchk) {
        edge = st;
        const bool taken = t == d.tgt;
        const bool nonnull = d.op == X_JEQ ? !taken : taken;
        edge[d.dst] = nonnull ? PVal{P_MAPVAL, 0, st[d.dst].id} : kOther;
        src = &edge;
      }
      bool changed = false;
      for (int r = 0; r < 11; r++) {
        const PVal nv = pjoin(in[t][r], (*src)[r]);
        if (!(nv == in[t][r])) {
          in[t][r] = nv;
          changed = true;
        }
      }
      if (changed && !queued[t]) {
        queued[t] = true;
        work.push_back(t);
      }
    }
  }
  return !ctx_written;
}

// ---------------------------------------------------------------------------
// Counter deferral.  Counter adds (fused ldx/add/stx and BPF_ATOMIC add
// without fetch) may be summed per wave or per block and reach memory when
// the wave / block ends (interp.hip delta cache, gen_fast.py comb_add) only
// while nothing the same unit executes afterwards can observe the location:
// a unit must see its own increments (bpftime_prog.cpp:231-260 runs ld/add/st
// one unit at a time).  Locations are abstracted from the pointer kinds: a
// constant address (lddw), a map value range (map fd, offset range), the
// unit's own memory (stack, ctx, packet, slot: never a map) or anything.
// ---------------------------------------------------------------------------
namespace {
struct Loc {
  enum : uint8_t { LOCAL, CONST, MAPVAL, ANY } cls;
  int32_t fd;
  int64_t lo, hi;  // byte range (CONST: absolute addresses; MAPVAL: offsets in the value)
};
constexpr int64_t kUnknownLen = 1 << 16;
}  // namespace

static Loc loc_of(const std::vector<DInsn> &p, const PVal &b, int64_t off, int64_t len) {
  switch (b.kind) {
    case P_CTX: case P_PKT: case P_SLOT: case P_STK:
      return Loc{Loc::LOCAL, -1, 0, 0};
    case P_CONST: {
      const DInsn &l = p[b.id];
      const int64_t a = (int64_t)((uint64_t)(uint32_t)l.imm | ((uint64_t)(uint32_t)l.hi << 32)) + b.k + off;
      return Loc{Loc::CONST, -1, a, a + len};
    }
    case P_MAPVAL: case P_MVNULL:
      return Loc{Loc::MAPVAL, b.id, (int64_t)b.k + off, (int64_t)b.k + off + len};
    default:
      return Loc{Loc::ANY, -1, 0, 0};
  }
}

static bool may_alias(const Loc &a, const Loc &b) {
  if (a.cls == Loc::ANY || b.cls == Loc::ANY) return true;
  if (a.cls == Loc::LOCAL || b.cls == Loc::LOCAL) return a.cls == b.cls;
  if (a.cls == Loc::CONST && b.cls == Loc::CONST) return a.lo < b.hi && b.lo < a.hi;
  if (a.cls == Loc::MAPVAL && b.cls == Loc::MAPVAL) return a.fd == b.fd && a.lo < b.hi && b.lo < a.hi;
  const Loc &c = a.cls == Loc::CONST ? a : b, &m = a.cls == Loc::CONST ? b : a;
  const MapRec *r = map_rec(m.fd);
  if (!r) return true;
  return c.lo < (int64_t)(r->d.data + r->bytes) && (int64_t)r->d.data < c.hi;
}

// Memory the instruction at i reads or writes, other than as a counter add.
static void accesses(const std::vector<DInsn> &p, uint32_t i, const std::vector<PVal> &st, std::vector<Loc> &out) {
  out.clear();
  const DInsn &d = p[i];
  const int64_t sz = 1 << ((d.aux >> A_SIZE_SHIFT) & 3);
  switch (d.op) {
    case X_LDX: out.push_back(loc_of(p, st[d.src], d.off, sz)); return;
    case X_ST: case X_STX: out.push_back(loc_of(p, st[d.dst], d.off, sz)); return;
    case X_ATOMIC:
      if (d.hi != 0x00) out.push_back(loc_of(p, st[d.dst], d.off, sz));
      return;
    case X_RMW_ADD:
      if (d.aux & A_FETCH) out.push_back(loc_of(p, st[d.dst], d.off, sz));
      return;
    case X_CALL: break;
    default: return;
  }
  const uint32_t id = (uint32_t)d.hi;
  auto arg = [&](int r) { out.push_back(loc_of(p, st[r], 0, kUnknownLen)); };
  auto map_values = [&]() {  // the values of the map in r1
    if (st[1].kind == P_MAPFD) out.push_back(Loc{Loc::MAPVAL, st[1].id, 0, kUnknownLen});
    else out.push_back(Loc{Loc::ANY, -1, 0, 0});
  };
  switch (id) {
    case 5: case 7: case 8: case 131: case 44: case 65: return;  // no memory (ctx helpers: unit-local)
    case 1: arg(2); return;
    case 2: arg(2); arg(3); map_values(); return;
    case 3: arg(2); map_values(); return;
    case 28: arg(1); arg(3); return;
    case 130: arg(2); return;
    case 132: case 133: arg(1); return;
    case 189: arg(3); return;
    default:
      if ((int32_t)id == kRetHelper) return;
      out.push_back(Loc{Loc::ANY, -1, 0, 0});  // tail calls and anything else
  }
}

// nodefer[i] for every counter-add site i: an access that may alias it is
// reachable from it (loops included).
static std::vector<bool> counter_nodefer(const std::vector<DInsn> &p, const std::vector<std::vector<PVal>> &in) {
  const uint32_t n = (uint32_t)p.size();
  auto reached = [&](uint32_t i) { return !(in[i][0].kind == P_UNDEF && in[i][1].kind == P_UNDEF); };
  std::vector<std::vector<Loc>> acc(n);
  for (uint32_t i = 0; i < n; i++)
    if (reached(i)) accesses(p, i, in[i], acc[i]);
  std::vector<bool> nodefer(n, false);
  std::vector<uint32_t> seen(n, UINT32_MAX), work;
  // a linked target's exit continues after every tail-call site
  std::vector<uint32_t> ret_points;
  for (uint32_t i = 0; i + 1 < n; i++)
    if (p[i].op == X_CALL && p[i].hi == (int32_t)kTailHelper && reached(i)) ret_points.push_back(i + 1);
  auto next_of = [&](uint32_t k, std::vector<uint32_t> &w) {
    if (p[k].op == X_CALL && p[k].hi == kRetHelper) {
      for (uint32_t r : ret_points) w.push_back(r);
      return;
    }
    uint32_t s[2];
    int ns;
    successors(p, k, s, ns);
    for (int j = 0; j < ns; j++) w.push_back(s[j]);
  };
  for (uint32_t i = 0; i < n; i++) {
    const DInsn &d = p[i];
    const bool add = (d.op == X_RMW_ADD && !(d.aux & A_FETCH)) || (d.op == X_ATOMIC && d.hi == 0x00);
    if (!add || !reached(i)) continue;
    const int64_t sz = 1 << ((d.aux >> A_SIZE_SHIFT) & 3);
    const Loc me = loc_of(p, in[i][d.dst], d.off, sz);
    if (me.cls == Loc::LOCAL || me.cls == Loc::ANY) {  // the unit's own memory / unknown: nothing to gain
      nodefer[i] = true;
      continue;
    }
    bool hit = false;
    work.clear();
    next_of(i, work);
    while (!work.empty() && !hit) {
      const uint32_t k = work.back();
      work.pop_back();
      if (seen[k] == i) continue;
      seen[k] = i;
      for (const Loc &l : acc[k])
        if (may_alias(me, l)) hit = true;
      next_of(k, work);
    }
    nodefer[i] = hit;
  }
  return nodefer;
}

// Loads at a constant address (an lddw map_val immediate + offsets) inside
// an ARRAY / PER-CPU ARRAY map's storage that nothing in the program may
// write -- no store, atomic or counter add that may alias it, no helper that
// writes that map -- are the same for every unit of a launch (host writes
// reach the device between launches, and the kernel starts with a fresh
// scalar cache): they read through the scalar cache (F_KLDX).  A .rodata
// value (libbpf's const volatile globals) is the common case: syscount's
// filters.  kimm[i] = the 4-aligned address, kaux[i] = 0 (8 bytes) or
// width << 16 | bit offset.
static void const_loads(const std::vector<DInsn> &p, const std::vector<uint8_t> &lddw_src,
                        const std::vector<std::vector<PVal>> &in, std::vector<int64_t> &kimm,
                        std::vector<int32_t> &kaux) {
  const uint32_t n = (uint32_t)p.size();
  kimm.assign(n, 0);
  kaux.assign(n, -1);
  auto reached = [&](uint32_t i) { return !(in[i][0].kind == P_UNDEF && in[i][1].kind == P_UNDEF); };
  std::vector<Loc> writes;
  for (uint32_t i = 0; i < n; i++) {
    if (!reached(i)) continue;
    const DInsn &d = p[i];
    const int64_t sz = 1 << ((d.aux >> A_SIZE_SHIFT) & 3);
    const std::vector<PVal> &st = in[i];
    switch (d.op) {
      case X_ST: case X_STX: case X_ATOMIC: case X_RMW_ADD:
        writes.push_back(loc_of(p, st[d.dst], d.off, sz));
        break;
      case X_CALL:
        switch (d.hi) {
          case 1: case 5: case 7: case 8: case 14: case 28: case 58: case 187: case 130:
          case 131: case 132: case 133: case 44: case 65:
            break;  // no array-map writes (ring memory, the unit's ctx, dispatch state)
          case 2: case 3:  // the values of the map in r1
            if (st[1].kind == P_MAPFD) writes.push_back(Loc{Loc::MAPVAL, st[1].id, 0, kUnknownLen});
            else writes.push_back(Loc{Loc::ANY, -1, 0, 0});
            break;
          case 189:
            writes.push_back(loc_of(p, st[3], 0, kUnknownLen));
            break;
          default:
            if (d.hi != kRetHelper) writes.push_back(Loc{Loc::ANY, -1, 0, 0});
        }
        break;
      default:
        break;
    }
  }
  for (uint32_t i = 0; i < n; i++) {
    const DInsn &d = p[i];
    if (d.op != X_LDX || !reached(i)) continue;
    const PVal b = in[i][d.src];
    if (b.kind != P_CONST || b.id < 0 || (size_t)b.id >= lddw_src.size() || lddw_src[b.id] != 2) continue;
    const int64_t sz = 1 << ((d.aux >> A_SIZE_SHIFT) & 3);
    const Loc me = loc_of(p, b, d.off, sz);
    const uint64_t a = (uint64_t)me.lo;
    if (a % sz != 0 || (sz == 8 && a % 4 != 0) || !in_array_storage(a, (uint32_t)sz)) continue;
    bool hit = false;
    for (const Loc &w : writes) hit = hit || may_alias(me, w);
    if (hit) continue;
    kimm[i] = (int64_t)(a & ~3ull);
    kaux[i] = sz == 8 ? 0 : (int32_t)(((8 * sz) << 16) | (8 * (a & 3)));
  }
}

// A hash element's bucket can change owner while a launch runs: LRU inserts
// evict, and a deleted key's bucket is reused.  A counter add held until its
// block ends could then land in another key's value, so adds into such maps
// go to memory at once.
static bool rebinds(const std::vector<DInsn> &p, const PVal &b, bool may_delete) {
  auto moves = [&](const MapRec *m) {
    return m && (m->type == MT_LRU_HASH || (may_delete && (m->type == MT_HASH || m->type == MT_PERCPU_HASH)));
  };
  if (b.kind == P_MAPVAL) return moves(map_rec(b.id));
  if (b.kind != P_CONST) return false;
  const Loc l = loc_of(p, b, 0, 8);
  Runtime &r = rt();
  for (uint32_t fd = 0; fd < kMaxFds; fd++) {
    if (r.kind[fd] != HKind::MAP || !moves(&r.maps[fd])) continue;
    const MapRec &m = r.maps[fd];
    if (l.lo < (int64_t)(m.d.data + m.bytes) && (int64_t)m.d.data < l.hi) return true;
  }
  return false;
}

// map_update_elem / map_delete_elem calls that may change an LPM trie
// (FastForm::lpm_writes): the call's map when the pointer kinds bind r1 to
// an lddw map fd, else every LPM trie the program names in an lddw.
static void lpm_write_sites(const std::vector<DInsn> &p, const std::vector<uint8_t> &lddw_src,
                            const std::vector<std::vector<PVal>> *in, FastForm &out) {
  std::vector<int32_t> named;
  for (size_t i = 0; i < p.size(); i++) {
    if (p[i].op != X_LDDW || i >= lddw_src.size() || lddw_src[i] != 1) continue;
    const uint64_t v = (uint64_t)(uint32_t)p[i].imm | ((uint64_t)(uint32_t)p[i].hi << 32);
    const MapRec *m = v < kMaxFds ? map_rec((int64_t)v) : nullptr;
    if (m && m->type == MT_LPM_TRIE) named.push_back((int32_t)v);
  }
  out.names_lpm = !named.empty();
  auto add = [&](uint32_t h, int32_t fd) {
    if (std::find(out.lpm_writes.begin(), out.lpm_writes.end(), std::make_pair(h, fd)) == out.lpm_writes.end())
      out.lpm_writes.emplace_back(h, fd);
  };
  for (size_t i = 0; i < p.size(); i++) {
    if (p[i].op != X_CALL || (p[i].hi != 2 && p[i].hi != 3)) continue;
    const uint32_t h = (uint32_t)p[i].hi;
    if (in) {
      const PVal &r1 = (*in)[i][1];
      if (r1.kind == P_UNDEF && (*in)[i][0].kind == P_UNDEF) continue;  // unreachable
      if (r1.kind == P_MAPFD) {
        const MapRec *m = map_rec(r1.id);
        if (m && m->type == MT_LPM_TRIE) add(h, r1.id);
        continue;
      }
    }
    for (const int32_t fd : named) add(h, fd);
  }
}

// The ctx and stack words a linked target may write (FastForm
// tail_ctx_mask / tail_stack_mask): its stores through ctx / stack pointers
// of known offset, and the helpers that write ctx fields or stack buffers.
// Targets are the pcs before the loaded program (vm_api.cpp links them first,
// behind a jump at pc 0); anything not understood saves everything.
static void tail_save_masks(const std::vector<DInsn> &p, const std::vector<std::vector<PVal>> &in,
                            uint32_t stack_size, FastForm &out) {
  uint32_t cm = 0, sm = 0;
  const uint32_t all_s = stack_size >= 256 ? 0xffffffffu : (1u << ((stack_size + 7) / 8)) - 1;
  auto ctx_bytes = [&](int64_t at, int64_t len) {
    for (int64_t k = 0; k < 6; k++)
      if (at < 8 * k + 8 && 8 * k < at + len) cm |= 1u << k;
  };
  auto stk_bytes = [&](int64_t at, int64_t len) {  // at: offset from the stack top (< 0)
    const int64_t lo = (int64_t)stack_size + at, hi = lo + len;
    if (lo < 0 || hi > (int64_t)stack_size) {
      sm = all_s;
      return;
    }
    for (int64_t j = 0; 8 * j < (int64_t)stack_size; j++)
      if (lo < 8 * j + 8 && 8 * j < hi) sm |= 1u << j;
  };
  auto write = [&](const PVal &b, int64_t off, int64_t len) {
    switch (b.kind) {
      case P_CTX: ctx_bytes((int64_t)b.k + off, len); break;
      case P_STK: stk_bytes((int64_t)b.k + off, len); break;
      case P_PKT: case P_SLOT: case P_MAPVAL: case P_CONST: break;
      default: cm = 0x3f; sm = all_s;
    }
  };
  uint32_t end = (uint32_t)p.size();
  if (!p.empty() && p[0].op == X_JA) end = p[0].tgt;  // the loaded program starts there
  for (uint32_t i = 1; i < end; i++) {
    const std::vector<PVal> &st = in[i];
    if (st[0].kind == P_UNDEF && st[1].kind == P_UNDEF) continue;  // unreached
    const DInsn &d = p[i];
    const int64_t sz = 1 << ((d.aux >> A_SIZE_SHIFT) & 3);
    if (d.op == X_ST || d.op == X_STX || d.op == X_ATOMIC || d.op == X_RMW_ADD) write(st[d.dst], d.off, sz);
    if (d.op != X_CALL) continue;
    switch ((uint32_t)d.hi) {
      case 1: case 2: case 3: case 5: case 7: case 8: case 12: case 28: case 130: case 131: case 132: case 133:
        break;
      case 44: case 65: ctx_bytes(0, 16); break;  // adjust_head / adjust_tail: data, data_end
      case 189: write(st[3], 0, 1 << 16); break;  // xdp_load_bytes(ctx, off, to, len)
      default:
        if (d.hi != kRetHelper) {
          cm = 0x3f;
          sm = all_s;
        }
    }
  }
  out.tail_ctx_mask = cm;
  out.tail_stack_mask = sm & all_s;
}

static uint32_t direct_add_handler(const DInsn &d) {
  const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
  if (sz != 4 && sz != 8) return F_SLOW;
  if (d.op == X_ATOMIC) return sz == 8 ? F_ATOMD8 : F_ATOMD4;
  if (d.aux & A_FETCH) return F_SLOW;
  const bool r = (d.aux & A_SRCREG) != 0;
  return sz == 8 ? (r ? F_RMWD8_R : F_RMWD8_I) : (r ? F_RMWD4_R : F_RMWD4_I);
}

static bool is_counter_add(const DInsn &d) {
  return d.op == X_RMW_ADD || (d.op == X_ATOMIC && d.hi == 0x00);
}

uint32_t lcache_sets() {
  static const uint32_t sets = [] {
    uint32_t s = kLcacheSets;
    if (const char *e = getenv("BPFTIME_AMD_LCACHE_SETS")) {
      const uint32_t v = (uint32_t)atoi(e);
      if (v >= 256 && v <= 4096 && (v & (v - 1)) == 0) s = v;
    }
    return s;
  }();
  return sets;
}

// FastForm::map_fx from the pointer kinds: which maps each load, store,
// atomic and map helper call reaches.  Accesses of the unit's own memory (its
// stack, its ctx copy, packet / slot bytes) are not map effects; an access
// whose base the kinds cannot place, or a helper that is not modelled, may
// reach any map (any_fx).
static void map_effects(const std::vector<DInsn> &prog, const std::vector<std::vector<PVal>> &in, FastForm &out) {
  out.map_fx.clear();
  out.any_fx = 0;
  auto mark = [&](int32_t fd, uint8_t bits) {
    if (fd >= 0) out.map_fx[fd] |= bits;
    else out.any_fx |= bits;
  };
  // the map a memory access through base kind b (+ off) reaches: fd, -1 any
  // map, -2 the unit's own memory
  auto target = [&](size_t i, const PVal &b, int64_t off, uint32_t sz) -> int32_t {
    switch (b.kind) {
      case P_STK: case P_CTX: case P_PKT: case P_SLOT:
        return -2;
      case P_MAPVAL: case P_MVNULL:
        return b.id;
      case P_CONST: {
        const DInsn &l = prog[(size_t)b.id];
        const uint64_t a = ((uint64_t)(uint32_t)l.imm | ((uint64_t)(uint32_t)l.hi << 32)) + (int64_t)b.k + off;
        return array_fd_of(a, sz);
      }
      default:
        (void)i;
        return -1;
    }
  };
  for (size_t i = 0; i < prog.size(); i++) {
    const DInsn &d = prog[i];
    const std::vector<PVal> &st = in[i];
    if (st[10].kind == P_UNDEF) continue;  // unreachable
    const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
    switch (d.op) {
      case X_LDX: {
        const int32_t t = target(i, st[d.src], d.off, sz);
        if (t != -2) mark(t, FX_READ);
        break;
      }
      case X_ST: case X_STX: {
        const int32_t t = target(i, st[d.dst], d.off, sz);
        if (t != -2) mark(t, FX_WRITE);
        break;
      }
      case X_RMW_ADD: case X_ATOMIC: {
        const uint32_t asz = d.op == X_ATOMIC ? (((d.aux >> A_SIZE_SHIFT) & 3) == 3 ? 8 : 4) : sz;
        const int32_t t = target(i, st[d.dst], d.off, asz);
        const bool add = d.op == X_RMW_ADD ? !(d.aux & A_FETCH) : d.hi == 0x00;
        if (t != -2) mark(t, add ? FX_ADD : FX_WRITE);
        break;
      }
      case X_CALL: {
        const PVal &m = st[1];
        const int32_t fd = m.kind == P_MAPFD ? m.id : -1;
        switch (d.hi) {
          case 1: mark(fd, FX_READ); break;                             // map_lookup_elem
          case 2: case 3: case 130: case 131: mark(fd, FX_WRITE); break;  // update, delete, ringbuf output / reserve
          case 5: case 7: case 8: case 14: case 28: case 44: case 58: case 65: case 132: case 133: case 187: case 189:
            break;  // no map effects (132 / 133 finish a reservation 131 marked)
          default: mark(-1, FX_READ | FX_WRITE); break;                 // bpf_tail_call, anything else
        }
        break;
      }
      default:
        break;
    }
  }
}

void build_fast(const LoadOut &lo, bool xdp, FastForm &out) {
  const std::vector<DInsn> &prog = lo.prog;
  out.fast.assign(prog.size(), FInsn{});
  out.stat.assign(prog.size(), FStatic{});
  out.add_site.assign(prog.size(), 0);
  for (size_t i = 0; i < prog.size(); i++) out.add_site[i] = is_counter_add(prog[i]) ? 1 : 0;
  out.specialized = 0;
  out.needs_comb = true;
  out.needs_ctx = xdp;
  out.tail_max_live = 0;
  out.join.assign(prog.size(), 1);  // (filled in below when the pointer kinds hold)
  for (size_t i = 0; i < prog.size(); i++) {
    const DInsn &d = prog[i];
    FInsn &f = out.fast[i];
    const bool mem = d.op == X_LDX || d.op == X_ST || d.op == X_STX || d.op == X_ATOMIC || d.op == X_RMW_ADD;
    f.hoff = 4 + 4 * fast_id(d);
    f.w1 = 0;
    f.dst_x2 = (uint32_t)d.dst * 2;
    f.src_x2 = (uint32_t)d.src * 2;
    f.imm = d.op == X_LDDW ? (int64_t)((uint64_t)(uint32_t)d.imm | ((uint64_t)(uint32_t)d.hi << 32))
            : mem          ? (int64_t)d.off
                           : (int64_t)d.imm;
    f.target = (uint32_t)d.tgt * kFastInsnBytes;
    f.aux = d.imm;
    // tail calls / a linked target's exit: asm frames in the XDP form
    // (gen_fast.py tail_call; the raw form's ctx copy is left to C++)
    if (xdp && d.op == X_CALL && d.hi == (int32_t)kTailHelper) {
      f.hoff = 4 + 4 * F_TAIL;
      f.imm = i < lo.tail_live.size() ? lo.tail_live[i] : 0x3fe;  // registers the frame keeps
      out.tail_max_live = std::max<uint32_t>(out.tail_max_live, (uint32_t)__builtin_popcount((uint32_t)f.imm & 0x3fe));
    }
    if (xdp && d.op == X_CALL && d.hi == kRetHelper) f.hoff = 4 + 4 * F_TRET;
  }
  // helpers that move ctx->data / data_end invalidate packet pointers
  bool pkt_ok = true;
  for (const DInsn &d : prog)
    if (d.op == X_CALL && (d.hi == 44 || d.hi == 65)) pkt_ok = false;
  std::vector<std::vector<PVal>> in;
  auto make_direct = [&](size_t i) {
    out.fast[i].hoff = 4 + 4 * direct_add_handler(prog[i]);
    out.fast[i].w1 |= FW_NODEFER;
  };
  bool kinds_ok;
  if (lo.multi_entry) {
    // targets enter with the caller's ctx when every tail-call site passes it
    kinds_ok = pointer_kinds(prog, lo.lddw_src, xdp, pkt_ok, in, lo.entries, true);
    const PVal ctx0 = xdp ? PVal{P_CTX, 0, 0} : PVal{P_SLOT, 0, 0};
    bool passes = true;
    for (size_t i = 0; i < prog.size(); i++)
      if (prog[i].op == X_CALL && prog[i].hi == (int32_t)kTailHelper && in[i][1].kind != P_UNDEF &&
          !(in[i][1] == ctx0))
        passes = false;
    if (kinds_ok && !passes) kinds_ok = pointer_kinds(prog, lo.lddw_src, xdp, pkt_ok, in, lo.entries, false);
  } else {
    kinds_ok = pointer_kinds(prog, lo.lddw_src, xdp, pkt_ok, in);
  }
  lpm_write_sites(prog, lo.lddw_src, kinds_ok ? &in : nullptr, out);
  // may a store reach the memory r1 points to at entry (the unit: the
  // syscall dispatch runs such a program on a copy of its records, as each
  // reference callback gets its own ctx copy)
  out.stores_unit = !kinds_ok;
  if (kinds_ok) map_effects(prog, in, out);  // (else any_fx stays: every map, read and written)
  for (size_t i = 0; kinds_ok && i < prog.size(); i++) {
    const DInsn &d = prog[i];
    if (d.op != X_ST && d.op != X_STX && d.op != X_RMW_ADD && d.op != X_ATOMIC) continue;
    const uint8_t k = in[i][d.dst].kind;
    if (k != P_UNDEF && k != P_STK && k != P_MAPVAL && k != P_CONST) out.stores_unit = true;
  }
  if (!kinds_ok) {
    // ctx rewritten: generic handlers only, no pointer kinds to prove a
    // counter unobserved
    for (size_t i = 0; i < prog.size(); i++)
      if (out.add_site[i]) make_direct(i);
    out.needs_comb = false;
    return;
  }
  const std::vector<bool> nodefer = counter_nodefer(prog, in);
  for (size_t i = 0; i < prog.size(); i++)
    if (out.add_site[i] && (nodefer[i] || (prog[i].aux & A_FETCH) || rebinds(prog, in[i][prog[i].dst], lo.may_delete)))
      make_direct(i);
  // per-lane counter adds (fused counters, atomic adds without fetch) whose
  // target is not a wave-uniform constant use the LDS combining table
  bool comb = false;
  for (size_t i = 0; i < prog.size(); i++) {
    const DInsn &d = prog[i];
    if (out.add_site[i] && !(out.fast[i].w1 & FW_NODEFER) && in[i][d.dst].kind != P_CONST &&
        in[i][d.dst].kind != P_UNDEF)
      comb = true;
  }
  out.needs_comb = comb;
  // how many counter granules the table can be asked to hold per block: the
  // elements of every map a deferred add reaches (the sites adding to one
  // value share its granules) -- per-CPU elements for the few virtual CPUs a
  // block's consecutive units span (kBlock / 64 waves)
  {
    uint64_t hint = 0;
    std::vector<uint32_t> seen;
    for (size_t i = 0; i < prog.size() && hint < ~0u; i++) {
      const DInsn &d = prog[i];
      if (!out.add_site[i] || (out.fast[i].w1 & FW_NODEFER)) continue;
      const PVal b = in[i][d.dst];
      if (b.kind == P_CONST || b.kind == P_UNDEF) continue;
      const MapRec *m = b.kind == P_MAPVAL ? map_rec(b.id) : nullptr;
      if (!m) {
        hint = ~0u;
        break;
      }
      if (std::find(seen.begin(), seen.end(), (uint32_t)b.id) != seen.end()) continue;
      seen.push_back((uint32_t)b.id);
      const bool percpu = m->type == MT_PERCPU_ARRAY || m->type == MT_PERCPU_HASH;
      hint += (uint64_t)m->max_entries * (percpu ? kBlock / 64 : 1);
    }
    out.comb_hint = hint >= ~0u ? ~0u : (uint32_t)hint;
  }
  if (lo.multi_entry && xdp) {
    tail_save_masks(prog, in, lo.stack_size, out);
    // a live register holding the lane's own ctx pointer at a tail call is
    // not saved: the return sets it again (FInsn imm bit 10 + r, header bit
    // kFrameRematShift + r; gen_fast.py tail_call / tail_ret)
    const PVal ctx0{P_CTX, 0, 0};
    out.tail_max_live = 0;
    for (size_t i = 0; i < prog.size(); i++) {
      FInsn &f = out.fast[i];
      if (f.hoff != 4 + 4 * F_TAIL) continue;
      for (int r = 1; r <= 9; r++)
        if (((uint64_t)f.imm >> r) & 1 && in[i][r] == ctx0) f.imm = (int64_t)(((uint64_t)f.imm & ~(1ull << r)) | (1ull << (10 + r)));
      out.tail_max_live = std::max<uint32_t>(out.tail_max_live, (uint32_t)__builtin_popcountll((uint64_t)f.imm & 0x3fe));
    }
  }
  std::vector<int64_t> kimm;
  std::vector<int32_t> kaux;
  if (!getenv("BPFTIME_AMD_NO_KLDX")) const_loads(prog, lo.lddw_src, in, kimm, kaux);
  uint32_t nspec = 0;
  bool ctx_escapes = false;
  const bool big_stack = lo.big_stack;
  const int64_t stack_size = lo.stack_size;
  for (size_t i = 0; i < prog.size(); i++) {
    const DInsn &d = prog[i];
    const std::vector<PVal> &st = in[i];
    if (st[0].kind == P_UNDEF && st[1].kind == P_UNDEF) continue;  // unreachable
    const uint32_t sz = 1u << ((d.aux >> A_SIZE_SHIFT) & 3);
    const uint32_t si = sz == 1 ? 0 : sz == 2 ? 1 : sz == 4 ? 2 : 3;
    const bool sreg = (d.aux & A_SRCREG) != 0;
    FInsn &f = out.fast[i];
    if (xdp) {
      // the LDS ctx is needed unless the ctx pointer is only copied, offset
      // by constants, compared, or read through the specialised data /
      // data_end loads
      RegSet u, df;
      use_def(d, u, df);
      for (int r = 0; r < 11; r++) {
        if (!(u & (1u << r)) || st[r].kind != P_CTX) continue;
        bool ok = false;
        if (d.op == X_MOV) ok = sreg && r == d.src;
        else if (d.op == X_ADD || d.op == X_SUB) ok = r == d.dst && !sreg && !(d.aux & A_W32);
        else if (d.op == X_LDX) {
          const int64_t at = (int64_t)st[r].k + d.off;
          ok = r == d.src && pkt_ok && sz == 8 && (at == 0 || at == 8);
        } else if (is_cond_jump(d.op) || d.op == X_EXIT) {
          ok = true;
        }
        if (!ok) ctx_escapes = true;
      }
    }
    if (d.op == X_CALL) {
      // bpf_ringbuf_output of packet bytes at a constant offset into a ring
      // bound at load: the asm tier writes the record from the staged
      // window when the launch stages the ring (link_staged, gen_fast.py
      // call_rbout; op 3 with the ring's fd in imm)
      if (d.hi == 130) {
        const MapRec *m = st[1].kind == P_MAPFD ? map_rec(st[1].id) : nullptr;
        if (m && m->type == MT_RINGBUF && st[2].kind == P_PKT && st[2].k >= 0 &&
            st[2].k + 16 <= (int64_t)kFastStageBytes && !getenv("BPFTIME_AMD_NO_ASM_RINGBUF")) {
          FStatic &s = out.stat[i];
          s.kind = 1;
          s.op = 3;
          s.sz = 16;  // (the window must hold the largest record the asm writes)
          s.at = st[2].k;
          s.imm = st[1].id;
        }
        continue;
      }
      if (d.hi == 2) {
        // update of a HASH map with key and value on the stack (gen_fast.py
        // call_update_stk): an element every lane finds is overwritten in
        // asm; anything else (a new key, a lane whose lookup of the key just
        // missed: the lookup-or-init race rule) runs the C++ helper
        const PVal key = st[2], val = st[3];
        const MapRec *m = st[1].kind == P_MAPFD ? map_rec(st[1].id) : nullptr;
        const int64_t ka = (int64_t)key.k, va = (int64_t)val.k;
        if (m && m->type == MT_HASH && !big_stack && m->key_size % 4 == 0 && m->key_size <= 16 &&
            m->value_size % 4 == 0 && m->value_size > 0 && m->value_size <= 64 && key.kind == P_STK &&
            ka >= -stack_size && ka + m->key_size <= 0 && ka % 4 == 0 && val.kind == P_STK &&
            va >= -stack_size && va + m->value_size <= 0 && va % 4 == 0 && !getenv("BPFTIME_AMD_NO_ASM_UPDATE")) {
          f.hoff = 4 + 4 * F_CALL_UPDATE_STK;
          f.target = (uint32_t)(int32_t)ka;  // (w6: the key's offset from the stack top)
          f.imm = va;                         // (w2: the value's)
          f.aux = (int32_t)(m->value_size / 4);
          nspec++;
        }
        continue;
      }
      if (d.hi != 1) continue;
      // lookup with its key on the stack: key read straight from LDS; an
      // ARRAY map bound at load needs no map-table read at all
      const PVal key = st[2];
      const int64_t at = (int64_t)key.k;
      if (key.kind == P_STK && !big_stack && at >= -stack_size && at + 4 <= 0 && at % 4 == 0) {
        const MapRec *m = st[1].kind == P_MAPFD ? map_rec(st[1].id) : nullptr;
        if (m && m->type == MT_ARRAY) {
          f.hoff = 4 + 4 * F_CALL_LOOKUP_AK;
          f.imm = (int64_t)m->d.data;
          f.dst_x2 = m->max_entries;
          f.src_x2 = m->value_size;
        } else {
          f.hoff = 4 + 4 * F_CALL_LOOKUP_STK;
          // a HASH map nothing deletes from during the launch: found slots
          // can be remembered in the block's LDS lookup cache
          if (m && m->type == MT_HASH && !lo.may_delete && m->key_size % 4 == 0 && m->key_size <= 16 &&
              !getenv("BPFTIME_AMD_NO_LCACHE")) {
            f.w1 |= FW_LCACHE;
            f.dst_x2 = lcache_sets();  // (gen_fast.py lcache_probe: the cache's set count)
            out.needs_lcache = true;
          }
        }
        f.target = (uint32_t)(int32_t)at;
        nspec++;
      }
      continue;
    }
    if (d.op == X_RMW_ADD || (d.op == X_ATOMIC && d.hi == 0x00)) {
      if (sz != 4 && sz != 8) continue;
      if (f.w1 & FW_NODEFER) continue;  // direct handler chosen above
      const PVal b = st[d.dst];
      const int64_t at = (int64_t)b.k + d.off;
      const MapRec *m = b.kind == P_MAPVAL ? map_rec(b.id) : nullptr;
      const bool in_value = m && at >= 0 && at + sz <= m->value_size;
      if (d.op == X_ATOMIC) {
        if (in_value) {
          f.hoff = 4 + 4 * (sz == 8 ? F_ATOMMV8_ADD : F_ATOMMV4_ADD);
          nspec++;
        }
        continue;
      }
      if (b.kind == P_CONST && lo.lddw_src[b.id] == 2) {
        const DInsn &l = prog[b.id];
        const uint64_t a = ((uint64_t)(uint32_t)l.imm | ((uint64_t)(uint32_t)l.hi << 32)) + (uint64_t)at;
        if (a % sz == 0 && in_array_storage(a, sz)) {
          f.hoff = 4 + 4 * (sz == 8 ? (sreg ? F_RMWK8_R : F_RMWK8_I) : (sreg ? F_RMWK4_R : F_RMWK4_I));
          f.imm = (int64_t)a;
          nspec++;
        }
      } else if (in_value) {
        f.hoff = 4 + 4 * (sz == 8 ? (sreg ? F_RMWMV8_R : F_RMWMV8_I) : (sreg ? F_RMWMV4_R : F_RMWMV4_I));
        nspec++;
      }
      continue;
    }
    if (d.op != X_LDX && d.op != X_STX && d.op != X_ST) continue;
    const PVal b = st[d.op == X_LDX ? d.src : d.dst];
    const int64_t at = (int64_t)b.k + d.off;
    static const uint32_t ldk[4] = {F_LDX1_STK, F_LDX2_STK, F_LDX4_STK, F_LDX8_STK};
    static const uint32_t stxk[4] = {F_STX1_STK, F_STX2_STK, F_STX4_STK, F_STX8_STK};
    static const uint32_t stk[4] = {F_ST1_STK, F_ST2_STK, F_ST4_STK, F_ST8_STK};
    static const uint32_t ldm[4] = {F_LDX1_MV, F_LDX2_MV, F_LDX4_MV, F_LDX8_MV};
    static const uint32_t stxm[4] = {F_STX1_MV, F_STX2_MV, F_STX4_MV, F_STX8_MV};
    if ((b.kind == P_PKT || b.kind == P_SLOT) && at >= 0 && at + sz <= kFastStageBytes) {
      // packet bytes: data = slot + head, resolved with the batch head
      FStatic &s = out.stat[i];
      s.kind = b.kind == P_PKT ? 1 : 2;
      s.op = d.op == X_LDX ? 0 : d.op == X_STX ? 1 : 2;
      s.sz = (uint8_t)sz;
      s.at = (int32_t)at;
      s.imm = d.imm;
      nspec++;
    } else if (b.kind == P_STK && !big_stack && at >= -stack_size && at + sz <= 0 && at % sz == 0) {
      const uint32_t *tab = d.op == X_LDX ? ldk : d.op == X_STX ? stxk : stk;
      f.hoff = 4 + 4 * tab[si];
      f.target = (uint32_t)(int32_t)at;  // static byte offset from the stack top
      nspec++;
    } else if (pkt_ok && b.kind == P_CTX && d.op == X_LDX && sz == 8 && (at == 0 || at == 8)) {
      // ctx->data = slot + head, ctx->data_end = data + len (interp.hip setup)
      f.hoff = 4 + 4 * (at == 0 ? F_LDX_CTXDATA : F_LDX_CTXEND);
      nspec++;
    } else if (xdp && b.kind == P_CTX && at >= 0 && at + sz <= 48 && at % sz == 0) {
      // another field of the lane's own XDP ctx (userspace_xdp.h:6-17): in
      // LDS whenever the program reads or writes it this way (the escape
      // analysis below sets needs_ctx), at a static offset from r1
      static const uint32_t ldc[4] = {F_LDX1_CTX, F_LDX2_CTX, F_LDX4_CTX, F_LDX8_CTX};
      static const uint32_t stxc[4] = {F_STX1_CTX, F_STX2_CTX, F_STX4_CTX, F_STX8_CTX};
      static const uint32_t stc[4] = {F_ST1_CTX, F_ST2_CTX, F_ST4_CTX, F_ST8_CTX};
      f.hoff = 4 + 4 * (d.op == X_LDX ? ldc : d.op == X_STX ? stxc : stc)[si];
      f.target = (uint32_t)at;
      nspec++;
    } else if (b.kind == P_MAPVAL && d.op != X_ST) {
      const MapRec *m = map_rec(b.id);
      if (m && at >= 0 && at + sz <= m->value_size) {
        f.hoff = 4 + 4 * (d.op == X_LDX ? ldm[si] : stxm[si]);
        nspec++;
      }
    } else if (d.op == X_LDX && i < kaux.size() && kaux[i] >= 0) {
      f.hoff = 4 + 4 * F_KLDX;
      f.imm = kimm[i];
      f.aux = kaux[i];
      nspec++;
    }
  }
  // adjacent 8-byte atomic adds through one map-value base at off / off + 8
  // (the {packets, bytes} idiom) share one combining-table probe
  // (gen_fast.py atomic_pair); the second must not be a jump target or entry
  {
    std::vector<uint8_t> target(prog.size() + 1, 0);
    for (const DInsn &d : prog)
      if ((d.op == X_JA || is_cond_jump(d.op)) && d.tgt >= 0 && (size_t)d.tgt < prog.size()) target[d.tgt] = 1;
    for (uint32_t e : lo.entries)
      if (e < prog.size()) target[e] = 1;
    out.join.assign(target.begin(), target.begin() + prog.size());
    for (size_t i = 0; i + 1 < prog.size() && !getenv("BPFTIME_AMD_NO_PAIR"); i++) {
      const DInsn &a = prog[i], &b = prog[i + 1];
      if (out.fast[i].hoff != 4 + 4 * F_ATOMMV8_ADD || out.fast[i + 1].hoff != 4 + 4 * F_ATOMMV8_ADD) continue;
      if (target[i + 1] || a.dst != b.dst || b.off != a.off + 8 || !(in[i][a.dst] == in[i + 1][b.dst])) continue;
      out.fast[i].hoff = 4 + 4 * F_ATOMMV8_ADD2;
      out.fast[i].aux = (int32_t)b.src * 2;
      i++;
    }
  }
  out.specialized = nspec;
  out.needs_ctx = xdp && ctx_escapes;
}

static int64_t static_slot_offset(const FStatic &s, uint32_t head) {
  return (int64_t)s.at + (s.kind == 1 ? (int64_t)head : 0);
}

uint32_t stage_need(const FastForm &f, uint32_t head) {
  int64_t ext = 0;
  for (const FStatic &s : f.stat) {
    if (!s.kind) continue;
    const int64_t so = static_slot_offset(s, head);
    if (so >= 0 && so + s.sz <= (int64_t)kFastStageBytes) ext = std::max<int64_t>(ext, so + s.sz);
  }
  return (uint32_t)((ext + 15) & ~15);
}

// FInsn slots an entry covers: lddw, and the pairs run as one dispatch;
// a fused lookup (its lddw, lea and call) five
static size_t fspan(const std::vector<DInsn> &prog, const std::vector<FInsn> &out, size_t i) {
  if (out[i].hoff == 4 + 4 * F_CALL_LOOKUP_STK3 || out[i].hoff == 4 + 4 * F_CALL_LOOKUP_AK3) return 5;
  return (i < prog.size() && prog[i].op == X_LDDW) || out[i].hoff == 4 + 4 * F_ATOMMV8_ADD2 ||
                 out[i].hoff == 4 + 4 * F_LEA || (out[i].w1 & FW_MOVI)
             ? 2
             : 1;
}

// Superinstructions: pairs of adjacent instructions that compilers emit
// together run as one dispatch (gen_fast.py lea, movi_prefix): `mov64 rA,
// rB; add64 rA, imm` (pointer + offset: stack key arguments, packet bounds)
// and `mov64 r, imm32` in front of a conditional jump or exit (the verdict
// set before a bounds check or a return).  The pair's second instruction
// must not be a jump target or an entry, and keeps its own FInsn: the C++
// tier, which runs one instruction at a time, re-enters the asm there.
// BPFTIME_AMD_NO_FUSE turns it off.
static void fuse_pairs(const std::vector<DInsn> &prog, const std::vector<uint8_t> &join,
                       std::vector<FInsn> &out) {
  if (getenv("BPFTIME_AMD_NO_FUSE") || join.size() != prog.size()) return;
  auto is = [&](size_t i, uint32_t id) { return out[i].hoff == 4 + 4 * id; };
  auto jcc_or_exit = [&](size_t i) {
    const uint32_t id = (out[i].hoff - 4) / 4;
    return id == F_EXIT || (id >= F_J64_EQ_R && id <= F_J32_SLE_I);
  };
  for (size_t i = 0; i + 1 < prog.size(); i++) {
    if (join[i + 1] || prog[i].op == X_LDDW) continue;
    const DInsn &a = prog[i], &b = prog[i + 1];
    if (is(i, F_A64_MOV_R) && (is(i + 1, F_A64_ADD_I) || is(i + 1, F_A64_SUB_I)) && a.dst == b.dst) {
      FInsn g = out[i];
      g.hoff = 4 + 4 * F_LEA;
      g.imm = b.op == X_ADD ? (int64_t)b.imm : -(int64_t)b.imm;
      out[i] = g;
      i++;
    } else if (is(i, F_A64_MOV_I) && jcc_or_exit(i + 1) && !(out[i + 1].w1 & FW_MOVI)) {
      FInsn g = out[i + 1];
      g.w1 |= FW_MOVI | ((uint32_t)a.dst << FW_MOVI_REG_SHIFT);
      g.aux = a.imm;
      out[i] = g;
      i++;
    }
  }
  // a map lookup's argument set-up and call, `lddw r1, map; r2 = r10 + k;
  // call 1` in either order of the first two, as one dispatch at the first
  // (the call's FInsn with the map fd in w7: gen_fast.py CALL_LOOKUP_*3); the
  // other two keep their FInsns for jumps into the sequence and the C++
  // tier's re-entry
  for (size_t i = 0; i + 4 < prog.size(); i++) {
    const size_t c = i + 4;
    if (!is(c, F_CALL_LOOKUP_STK) && !is(c, F_CALL_LOOKUP_AK)) continue;
    size_t ld = i, le = i + 2;
    if (is(i, F_LEA)) std::swap(ld, le);
    if (!is(ld, F_LDDW) || prog[ld].op != X_LDDW || out[ld].dst_x2 != 2 || (uint64_t)out[ld].imm >= kMaxFds) continue;
    if (!is(le, F_LEA) || out[le].dst_x2 != 4 || out[le].src_x2 != 20 ||
        out[le].imm != (int64_t)(int32_t)out[c].target)
      continue;
    if (join[i + 2] || join[c]) continue;  // (sequential flow only: a jump into the middle runs the originals)
    FInsn g = out[c];
    g.hoff = 4 + 4 * (is(c, F_CALL_LOOKUP_STK) ? F_CALL_LOOKUP_STK3 : F_CALL_LOOKUP_AK3);
    g.aux = (int32_t)out[ld].imm;
    out[i] = g;
  }
}

// w1 bits 8+: the handler offset of the FInsn sequential flow reaches next
// (gen_fast.py next_seq jumps on it before the fetch lands); the SLOW handler
// past the end
static void link_next(const std::vector<DInsn> &prog, std::vector<FInsn> &out) {
  for (size_t i = 0; i < out.size(); i++) {
    const size_t nx = i + fspan(prog, out, i);
    const uint32_t h = nx < out.size() ? out[nx].hoff : 4 + 4 * F_SLOW;
    out[i].w1 = (out[i].w1 & 0xffu) | (h << 8);
  }
}

static void link_staged(const FastForm &f, uint32_t head, uint32_t stage, bool ordered,
                        const std::vector<DInsn> &prog, std::vector<FInsn> &out);

void link_fast(const FastForm &f, uint32_t head, uint32_t stage, bool ordered, const std::vector<DInsn> &prog,
               std::vector<FInsn> &out, int32_t unwind_idx, uint32_t lc_sets, uint32_t pid_off, bool no_kldx,
               bool rec_helpers) {
  link_staged(f, head, stage, ordered, prog, out);
  // rec_helpers (the thread-ordered kernel): bpf_get_current_pid_tgid and
  // bpf_ktime_get_ns read the caller / clock the kernel keeps beside the
  // lane's ctx copy (interp.hip k_sys_seq: ctx + kSeqPidOff / kSeqClockOff)
  if (rec_helpers)
    for (size_t i = 0; i < prog.size() && i < out.size(); i++)
      if (prog[i].op == X_CALL && (prog[i].hi == 14 || prog[i].hi == 5) && unwind_idx != prog[i].hi) {
        out[i].hoff = 4 + 4 * F_CALL_REC;
        out[i].aux = (int32_t)(prog[i].hi == 14 ? kSeqPidOff : kSeqClockOff);
      }
  // no_kldx: the launch runs other programs that may write the array
  // storage this one reads at constant addresses (the thread-ordered
  // kernel: const_loads proves the absence of writes per program only), so
  // those loads go through the vector memory path again, as unspecialised
  if (no_kldx)
    for (size_t i = 0; i < prog.size() && i < out.size(); i++)
      if (out[i].hoff == 4 + 4 * F_KLDX) {
        out[i].hoff = 4 + 4 * fast_id(prog[i]);
        out[i].imm = (int64_t)prog[i].off;
        out[i].aux = prog[i].imm;
      }
  // bpf_get_current_pid_tgid of a recorded syscall: a load from the unit
  if (pid_off && pid_off < 256)
    for (size_t i = 0; i < prog.size() && i < out.size(); i++)
      if (prog[i].op == X_CALL && prog[i].hi == 14 && unwind_idx != 14) {
        out[i].hoff = 4 + 4 * F_CALL_PID;
        out[i].aux = (int32_t)pid_off;
        // (inside the staged window: its dword index, and a flag)
        const bool staged = pid_off % 4 == 0 && pid_off + 8 <= stage;
        out[i].imm = staged ? (int64_t)(pid_off / 4) | (1ll << 32) : 0;
      }
  // the launch's lookup-cache set count (vm_api.cpp) into the lookups that
  // use it; a launch without a cache (0: the thread-ordered kernel) turns it off
  for (FInsn &x : out)
    if (x.w1 & FW_LCACHE) {
      if (lc_sets)
        x.dst_x2 = lc_sets;
      else
        x.w1 &= ~(uint32_t)FW_LCACHE;
    }
  // an unwind helper (ebpf_set_unwind_function_index) is called from the
  // C++ tier, which ends the unit when it returns 0: map_lookup_elem leaves
  // its asm handlers then
  if (unwind_idx == 2)
    for (size_t i = 0; i < prog.size() && i < out.size(); i++)
      if (prog[i].op == X_CALL && prog[i].hi == 2) out[i].hoff = 4 + 4 * F_SLOW;
  if (unwind_idx == 1)
    for (size_t i = 0; i < prog.size() && i < out.size(); i++)
      if (prog[i].op == X_CALL && prog[i].hi == 1) {
        out[i].hoff = 4 + 4 * F_SLOW;
        out[i].w1 &= ~(uint32_t)FW_LCACHE;
      }
  fuse_pairs(prog, f.join, out);
  link_next(prog, out);
}

static void link_staged(const FastForm &f, uint32_t head, uint32_t stage, bool ordered,
                        const std::vector<DInsn> &prog, std::vector<FInsn> &out) {
  out = f.fast;
  if (ordered)  // the reference's sequential order: every counter add reaches memory at once
    for (size_t i = 0; i < out.size(); i++)
      if (i < f.add_site.size() && f.add_site[i]) {
        out[i].hoff = 4 + 4 * direct_add_handler(prog[i]);
        out[i].w1 |= FW_NODEFER;
      }
  if (!stage) return;
  for (size_t i = 0; i < f.stat.size(); i++) {
    const FStatic &s = f.stat[i];
    if (!s.kind) continue;
    const int64_t so = static_slot_offset(s, head);
    if (so < 0 || so + s.sz > (int64_t)stage) continue;
    const uint32_t o = (uint32_t)so, sz = s.sz, sh = 8 * (o & 3);
    FInsn g = out[i];
    g.imm = (int64_t)((uint64_t)(o >> 2) | ((uint64_t)sh << 32));  // w2 dword index, w3 bit shift
    g.target = o;                                                // fallback: slot + o
    if (s.op == 3) {  // bpf_ringbuf_output's source: dword-aligned in the window
      if (o & 3) continue;
      g.hoff = 4 + 4 * F_CALL_RBOUT;
      g.imm = (int64_t)(o >> 2);
      g.target = (uint32_t)s.imm;  // the ring's fd
      out[i] = g;
      continue;
    }
    if (s.op == 0) {
      uint32_t id;
      if (sz == 8) id = (o & 3) ? F_LDXS8U : F_LDXS8A;
      else if ((o & 3) + sz <= 4) id = sz == 1 ? F_LDXS1 : sz == 2 ? F_LDXS2 : F_LDXS4;
      else id = sz == 2 ? F_LDXS2X : F_LDXS4X;
      g.hoff = 4 + 4 * id;
    } else {
      const bool fits = sz <= 2 ? (o & 3) + sz <= 4 : (o & 3) == 0;
      if (!fits) continue;  // straddles dwords: the generic handler ends staging
      static const uint32_t stx[4] = {F_STXS1, F_STXS2, F_STXS4, F_STXS8};
      static const uint32_t sti[4] = {F_STS1, F_STS2, F_STS4, F_STS8};
      const uint32_t si = sz == 1 ? 0 : sz == 2 ? 1 : sz == 4 ? 2 : 3;
      g.hoff = 4 + 4 * (s.op == 1 ? stx[si] : sti[si]);
      g.dst_x2 = (1u << (o >> 4)) | (1u << ((o + sz - 1) >> 4));     // dirty chunks
      g.aux = sz <= 2 ? (int32_t)((((1u << (8 * sz)) - 1)) << sh) : 0;  // byte mask
      if (s.op == 2) g.src_x2 = (uint32_t)s.imm;
    }
    out[i] = g;
  }
}

}  // namespace bpftime_amd
