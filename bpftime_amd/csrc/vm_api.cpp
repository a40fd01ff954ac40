// bpftime_amd: the drop-in VM C ABI (include/ebpf-vm.h).
//
// Mirrors vm/vm-core/src/ebpf-vm.cpp:6-98 over a single backend class that
// plays the role of a bpftime::vm::compat::bpftime_vm_impl
// (vm/compat/include/bpftime_vm_compat.hpp:27-198) registered under the name
// "mi355x" (the reference registers "ubpf" the same way,
// vm/compat/ubpf-vm/compat_ubpf.cpp:253-257).
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "loader.hpp"
#include "runtime.hpp"

namespace bpftime_amd {
extern "C" hipError_t bpftime_amd_launch_interp(const KParams *p, uint32_t kind, bool big_stack, uint32_t grid,
                                                uint32_t ordered, uint32_t block, hipStream_t stream);
extern "C" int bpftime_amd_occupancy(uint32_t kind, bool big_stack, size_t dyn_lds, bool gregs, uint32_t block,
                                    bool image);
extern "C" size_t bpftime_amd_static_lds_image(uint32_t kind, bool big_stack, bool gregs, uint32_t block, bool image);
extern "C" hipError_t bpftime_amd_launch_merge(const uint64_t *log, uint32_t log_words, uint32_t nblocks,
                                                hipStream_t stream);
extern "C" hipError_t bpftime_amd_launch_miss_merge(const uint64_t *log, const uint32_t *counts, uint32_t cap,
                                                     uint32_t nblocks, const KParams *p, uint32_t *bad,
                                                     hipStream_t stream);

// Off by default: measured on one box (profiles/r06_ab_lane_pad.txt) the
// padding halves flow-hash's LDS bank conflicts but costs the lines LDS
// (residency, table reach, LDS tail-call frames): tail-call 1.186 -> 1.277
// ms, lpm-route 0.454 -> 0.471, flow-hash 0.670 -> 0.682, syscount equal
bool lane_pad() {
  static const bool on = getenv("BPFTIME_AMD_LANE_PAD") && atoi(getenv("BPFTIME_AMD_LANE_PAD")) != 0;
  return on;
}

extern "C" hipError_t bpftime_amd_launch_fast_xlat(uint32_t kind, bool big_stack, bool greg, bool image,
                                                   uint32_t *d_out, hipStream_t stream);

// The asm tier dispatches straight into its handlers (gen_fast.py: direct
// dispatch): an FInsn names its handler by the handler's offset from the
// asm's handler base, not by its id.  The offsets are assembly-time
// constants of each of the two asm variants (the C++ tier's register copy in
// LDS or in global memory, k_interp G); the kernel reports them once per
// process (its query entry), and every linked program is translated from
// handler ids to them.  Handlers are laid out in id order, so the offsets
// must rise: anything else fails the link.
static std::mutex g_xlat_mu;
static std::vector<uint32_t> g_xlat[2];
static const std::vector<uint32_t> *fast_xlat(bool greg) {
  std::lock_guard<std::mutex> g(g_xlat_mu);
  std::vector<uint32_t> &t = g_xlat[greg ? 1 : 0];
  if (!t.empty()) return &t;
  uint32_t *d = nullptr;
  std::vector<uint32_t> h(F_COUNT, ~0u);
  bool ok = hipMalloc((void **)&d, 4 * F_COUNT) == hipSuccess &&
            hipMemset(d, 0xff, 4 * F_COUNT) == hipSuccess &&
            bpftime_amd_launch_fast_xlat(CTX_RAW, false, greg, false, d, nullptr) == hipSuccess &&
            hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(h.data(), d, 4 * F_COUNT, hipMemcpyDeviceToHost) == hipSuccess;
  if (d) hipFree(d);
  for (uint32_t i = 1; ok && i < F_COUNT; i++) ok = h[i] > h[i - 1] && h[i] < (1u << 24);
  if (!ok) return nullptr;
  t = std::move(h);
  return &t;
}

// experiment counters (BPFTIME_AMD_DBG 512), a device buffer made on first use
static std::mutex g_dbg_mu;
static uint64_t *g_dbg = nullptr;  // lookup-cache hit / miss lanes (gen_fast.py lcache_count)
static constexpr int kDbgCounts = 4;
uint64_t *dbg_counts() {
  std::lock_guard<std::mutex> g(g_dbg_mu);
  if (!g_dbg && (hipMalloc((void **)&g_dbg, 8 * kDbgCounts) != hipSuccess ||
                 hipMemset(g_dbg, 0, 8 * kDbgCounts) != hipSuccess))
    g_dbg = nullptr;
  return g_dbg;
}


struct HelperReg {
  std::string name;
  void *fn;
};

// A loaded program in device form.  Tail-call images (common.hpp
// kTailHelper) are rebuilt when a prog array changes; a batch holds a
// reference to the image it launches, so a relink by another thread never
// frees what an exec_batch in flight is reading (hipFree waits for the
// device, so launches already queued are safe too).
struct Image {
  LoadOut prog;
  DInsn *d_prog = nullptr;
  // threaded-code forms: XDP entry (r1 = ctx) and raw/syscall entry (r1 = the
  // unit's slot) differ in the loader's pointer kinds
  FastForm fx, fr;
  int32_t *d_tail_entry = nullptr;  // prog fd -> entry pc (tail-call images)
  // the asm tier's one-load form of the same: [kMaxFds] offsets of each
  // reachable PROG_ARRAY's slots (-1: not in the image), then per slot the
  // entry pc of the program it held at link time (-1: none / not linked)
  int32_t *d_tail_slots = nullptr;
  uint32_t frame_words = 0;         // tail-call frame: header + ctx + the image's stack bytes, / 8
  uint64_t gen = 0;                 // rt().prog_gen it was linked at
  // linked FInsn arrays per launch configuration (entry form, ORDERED,
  // staged bytes, batch head): a few per program, built on first use
  std::mutex link_mu;
  std::map<std::pair<uint64_t, uint32_t>, FInsn *> links;

  ~Image() {
    if (d_prog) hipFree(d_prog);
    if (d_tail_entry) hipFree(d_tail_entry);
    if (d_tail_slots) hipFree(d_tail_slots);
    for (auto &kv : links) hipFree(kv.second);
  }
  // greg: the asm variant of the launch (k_interp G), whose handler offsets
  // the form is translated to
  const FInsn *linked(bool greg, bool xdp, uint32_t head, uint32_t stage, bool ordered, int32_t unwind_idx,
                      uint32_t lc_sets, int32_t pid_off, bool no_kldx = false, bool rec_helpers = false) {
    std::lock_guard<std::mutex> g(link_mu);
    // (the helpers with asm handlers an unwind index changes: lookup, pid_tgid)
    const bool uw = unwind_idx == 1, uwp = unwind_idx == 14;
    const uint32_t po = pid_off > 0 && pid_off < 256 && !uwp ? (uint32_t)pid_off : 0;
    const uint64_t key = ((uint64_t)xdp << 63) | ((uint64_t)ordered << 62) | ((uint64_t)uw << 61) |
                         ((uint64_t)(lc_sets & 0x1fff) << 47) | ((uint64_t)stage << 40) | ((uint64_t)po << 32) |
                         (stage ? head : 0);
    const bool uwu = unwind_idx == 2;  // (map_update_elem's asm handler)
    const auto lk = std::make_pair(key, (uint32_t)no_kldx | ((uint32_t)rec_helpers << 1) | ((uint32_t)uwu << 2) |
                                            ((uint32_t)greg << 3));
    auto it = links.find(lk);
    if (it != links.end()) return it->second;
    std::vector<FInsn> out;
    link_fast(xdp ? fx : fr, head, stage, ordered, prog.prog, out, uw ? 1 : uwu ? 2 : -1, lc_sets, po, no_kldx,
              rec_helpers);
    if (getenv("BPFTIME_AMD_DUMP_FAST"))  // the linked threaded form, one FInsn a line
      for (size_t i = 0; i < out.size(); i++)
        fprintf(stderr, "bpftime_amd: fast %3zu %-18s w1 %08x imm %llx dst %u src %u tgt %u aux %x\n", i,
                fop_name((out[i].hoff - 4) / 4), out[i].w1, (unsigned long long)out[i].imm, out[i].dst_x2 / 2,
                out[i].src_x2 / 2, out[i].target / kFastInsnBytes, (unsigned)out[i].aux);
    // handler ids -> the variant's handler offsets (this FInsn's and, in
    // w1 bits 8.., the next one's)
    const std::vector<uint32_t> *xl = fast_xlat(greg);
    if (!xl) return nullptr;
    // jumps also carry their target's handler offset (gen_fast.py
    // jump_taken): w2 for JA and register compares (their imm is unused),
    // w5 for immediate compares (their src is unused)
    std::vector<uint32_t> jt(out.size(), ~0u);
    for (size_t i = 0; i < out.size(); i++) {
      const uint32_t id = (out[i].hoff - 4) / 4;
      if (id != F_JA && (id < F_J64_EQ_R || id > F_J32_SLE_I)) continue;
      const size_t t = out[i].target / kFastInsnBytes;
      jt[i] = t < out.size() ? (out[t].hoff - 4) / 4 : (uint32_t)F_SLOW;
      if (jt[i] >= F_COUNT) return nullptr;
    }
    for (FInsn &x : out) {
      const uint32_t id = (x.hoff - 4) / 4, nid = ((x.w1 >> 8) - 4) / 4;
      if (x.hoff < 4 || id >= F_COUNT || (x.w1 >> 8) < 4 || nid >= F_COUNT) return nullptr;
      x.hoff = (*xl)[id];
      x.w1 = (x.w1 & 0xffu) | ((*xl)[nid] << 8);
      const size_t i = &x - out.data();
      if (jt[i] == ~0u) continue;
      static_assert((F_J64_EQ_I - F_J64_EQ_R) == 1 && (F_J32_SLE_I - F_J64_EQ_R) % 2 == 1,
                    "jump handlers alternate register / immediate forms");
      if (id != F_JA && (id - F_J64_EQ_R) % 2 == 1)
        x.src_x2 = (*xl)[jt[i]];
      else
        x.imm = (int64_t)(*xl)[jt[i]];
    }
    FInsn *d = nullptr;
    const size_t bytes = out.size() * sizeof(FInsn);
    if (hipMalloc((void **)&d, bytes) != hipSuccess) return nullptr;
    if (hipMemcpy(d, out.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
      hipFree(d);
      return nullptr;
    }
    links[lk] = d;
    return d;
  }
  // device copy of the decoded program + both threaded forms
  int upload(LoadOut &&out, std::string &err) {
    build_fast(out, true, fx);
    build_fast(out, false, fr);
    out.comb_entries = (fx.needs_comb || fr.needs_comb) ? kComb : 0;
    const size_t bytes = out.prog.size() * sizeof(DInsn);
    if (hipMalloc((void **)&d_prog, bytes) != hipSuccess ||
        hipMemcpy(d_prog, out.prog.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
      err = "device upload failed";
      return -1;
    }
    prog = std::move(out);
    return 0;
  }
};

// device buffers kept per stream: a batch's launches use them in stream
// order, batches on other streams have their own
struct StreamBufs {
  struct Buf {
    void *p = nullptr;
    uint64_t bytes = 0;
  };
  std::mutex mu;
  std::map<hipStream_t, Buf> bufs;
  ~StreamBufs() {
    for (auto &kv : bufs)
      if (kv.second.p) hipFree(kv.second.p);
  }
  void *get(hipStream_t s, uint64_t bytes) {
    std::lock_guard<std::mutex> g(mu);
    Buf &b = bufs[s];
    if (b.bytes < bytes) {
      // the stream may still run a batch that uses the old buffer
      if (b.p && (hipStreamSynchronize(s) != hipSuccess || hipFree(b.p) != hipSuccess)) return nullptr;
      b.p = nullptr;
      b.bytes = 0;
      if (hipMalloc(&b.p, bytes) != hipSuccess) return nullptr;
      b.bytes = bytes;
    }
    return b.p;
  }
};

class Mi355xVm {
 public:
  std::string error;
  // compat_ubpf.hpp:42-44 (bpftime id -> ubpf-style id)
  std::map<size_t, size_t> helper_id_map;
  std::map<size_t, std::string> helper_names;
  size_t next_helper_id = 1;
  LddwHelpers lddw;
  bool bounds_check = true;
  int (*error_print)(FILE *, const char *, ...) = nullptr;
  int unwind_idx = -1;
  uint32_t ctx_kind = CTX_RAW;
  uint64_t step_limit = 1ull << 22;

  bool loaded = false;
  std::mutex img_mu;                 // guards img (replaced by tail-call relinks)
  std::shared_ptr<Image> img;
  std::shared_ptr<Image> image() {
    std::lock_guard<std::mutex> g(img_mu);
    return img;
  }
  // failed-unit counters, one per in-flight batch: concurrent batches on
  // different streams must not share (and re-zero) one counter
  static constexpr uint32_t kErrSlots = 64;
  uint32_t *d_err = nullptr;
  std::atomic<uint32_t> err_slot{0};
  // staging for ebpf_exec
  std::mutex stage_mu;
  uint8_t *d_stage = nullptr;
  size_t stage_size = 0;
  // bpf_tail_call: the loaded code, relinked with the prog arrays' targets
  // when rt().prog_gen moves
  std::vector<RawInsn> raw;
  bool has_tail = false;
  uint32_t base_stack = 0;  // the loaded program's own stack need (kStackSize + 1: unknown)
  std::string link_note;    // targets left out of the last image, and why
  // block-end flush logs (common.hpp kMergeGroup) and tail-call frames
  StreamBufs logs, frames, scratch, regs, misses;
  // the kernels of the last EBPF_BATCH_TIMED batch
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;

  Mi355xVm() {
    // bpftime_prog.cpp:126-127 defaults, pointed at the device registry
    lddw.map_by_fd = bpftime_amd_map_ptr_by_fd;
    lddw.map_val = bpftime_amd_map_val;
    const char *sl = getenv("BPFTIME_AMD_STEP_LIMIT");
    if (sl) step_limit = strtoull(sl, nullptr, 0);
  }
  ~Mi355xVm() {
    if (ev_t0) hipEventDestroy(ev_t0);
    if (ev_t1) hipEventDestroy(ev_t1);
    unload();
    if (d_err) hipFree(d_err);
    if (d_stage) hipFree(d_stage);
  }
  void unload() {
    std::lock_guard<std::mutex> g(img_mu);
    img.reset();
    loaded = false;
    raw.clear();
    has_tail = false;
  }
  int register_external_function(size_t index, const std::string &name, void *fn) {
    // compat_ubpf.cpp:50-59: allocate the next id; ubpf caps helpers at 64
    size_t next_id = next_helper_id++;
    if (next_id >= 64) {
      error = "too many helpers (ubpf supports 64)";
      return -1;
    }
    helper_id_map[index] = next_id;
    helper_names[index] = name;
    (void)fn;
    return 0;
  }
  int load_code(const void *code, size_t code_len) {
    if (code_len % 8 != 0) {
      error = "Length of code must be a multiple of 8";
      return -1;
    }
    if (loaded) {
      error = "code has already been loaded into this VM. Use ebpf_unload_code() if you need to reuse this VM";
      return -1;
    }
    LoadOut out;
    std::string err;
    int rc = load_program((const RawInsn *)code, code_len / 8, helper_id_map, helper_names, lddw, out, err);
    if (rc < 0) {
      error = err;
      return rc;
    }
    if (rt().ensure_device() < 0) {
      error = "no HIP device: " + rt().last_error;
      return -1;
    }
    if (!d_err && hipMalloc((void **)&d_err, 4 * kErrSlots) != hipSuccess) {
      error = "device alloc failed";
      return -1;
    }
    has_tail = out.tail_call;
    base_stack = out.big_stack ? kStackSize + 1 : out.stack_size;
    auto im = std::make_shared<Image>();
    if (im->upload(std::move(out), error) < 0) return -1;
    raw.assign((const RawInsn *)code, (const RawInsn *)code + code_len / 8);
    {
      std::lock_guard<std::mutex> g(img_mu);
      img = std::move(im);
    }
    loaded = true;
    return 0;
  }

  // Link the loaded program with the programs its prog arrays can reach:
  // the arrays it loads by fd (lddw src 1), the targets they name, and
  // transitively the arrays those targets load.  One image, the targets
  // appended (raw jumps are relative, so they need no relocation) with their
  // exits turned into kRetHelper calls, plus a prog fd -> entry pc table.  A
  // target that does not load alone is left out, so tail calls to it return
  // -1 like a failed bpftime_prog_load (bpf_helper.cpp:623-628); the reason
  // is kept in link_note.  Called with img_mu held.
  int link_tail_image_locked() {
    Runtime &r = rt();
    if (img && img->gen == r.prog_gen && img->d_tail_entry) return 0;
    std::map<size_t, size_t> hm = helper_id_map;
    std::map<size_t, std::string> names = helper_names;
    for (uint32_t id : {1u, 2u, 3u, 5u, 7u, 8u, 12u, 28u, 44u, 65u, 130u, 131u, 132u, 133u, 189u})
      if (!hm.count(id)) hm[id] = 63;  // the runtime's helper groups (bpf_helper.cpp:606-620)
    // prog arrays named by lddw src 1 in `code`
    auto arrays_of = [&](const RawInsn *code, size_t n, std::set<int32_t> &out) {
      // (the fd as BPF_PSEUDO_MAP_FD, or as a plain 64-bit immediate the way
      // runtime/unit-test/tailcall/test_user_to_user_tailcall.cpp loads it)
      for (size_t i = 0; i + 1 < n; i++)
        if (code[i].code == 0x18) {
          const uint64_t v = (uint64_t)(uint32_t)code[i].imm | ((uint64_t)(uint32_t)code[i + 1].imm << 32);
          const bool as_fd = code[i].src == 1 || (code[i].src == 0 && v < kMaxFds);
          const int32_t fd = code[i].imm;
          if (as_fd && fd >= 0 && fd < (int32_t)kMaxFds && r.kind[fd] == HKind::MAP &&
              r.maps[fd].type == MT_PROG_ARRAY)
            out.insert(fd);
          i++;
        }
    };
    // the prog arrays each program loads, and the targets each array names
    std::map<int32_t, std::set<int32_t>> arrays_of_prog;  // target prog fd -> arrays
    std::map<int32_t, std::vector<int32_t>> slots_of;     // array fd -> target prog fds
    std::map<int32_t, std::vector<int32_t>> slot_fds;     // array fd -> its slots (prog fds) at link time
    std::set<int32_t> root_arrays, pending;
    arrays_of(raw.data(), raw.size(), root_arrays);
    pending = root_arrays;
    link_note.clear();
    while (!pending.empty()) {
      const int32_t fd = *pending.begin();
      pending.erase(pending.begin());
      if (slots_of.count(fd)) continue;
      std::vector<int32_t> slots(r.maps[fd].max_entries);
      if (!slots.empty() &&
          hipMemcpy(slots.data(), (const void *)r.maps[fd].d.data, 4 * slots.size(), hipMemcpyDeviceToHost) != hipSuccess) {
        error = "prog array read failed";
        return -1;
      }
      slot_fds[fd] = slots;
      std::vector<int32_t> &ts = slots_of[fd];
      for (int32_t v : slots)
        if (v >= 0 && v < (int32_t)kMaxFds && r.kind[v] == HKind::PROG) {
          ts.push_back(v);
          if (!arrays_of_prog.count(v)) {
            const std::vector<uint8_t> &b = r.progs[v].insns;
            arrays_of((const RawInsn *)b.data(), b.size() / 8, arrays_of_prog[v]);
            for (int32_t a : arrays_of_prog[v]) pending.insert(a);
          }
        }
    }
    // Targets before the loaded program (which goes last behind a jump at
    // pc 0), callers before callees among them (reverse post-order): lane
    // groups run lowest pc first, so every target runs before the loaded
    // program's code it returns to -- lanes returning from different targets
    // (or failing the call) meet at the return point -- and a target that
    // other targets call runs after them, so the lanes that reach it from a
    // nested call join the lanes that called it directly (one group, one
    // pass over its code: tail-call line 1.30 -> 1.1x ms).  Lanes whose
    // nested call fails continue in their caller before the callee runs.
    std::vector<int32_t> order;
    std::set<int32_t> visited;
    std::function<void(int32_t)> visit = [&](int32_t t) {
      if (!visited.insert(t).second) return;
      for (int32_t a : arrays_of_prog[t])
        for (int32_t u : slots_of[a]) visit(u);
      order.push_back(t);
    };
    for (int32_t a : root_arrays)
      for (int32_t u : slots_of[a]) visit(u);
    std::reverse(order.begin(), order.end());
    std::vector<RawInsn> code;
    std::vector<uint32_t> entries;
    std::vector<int32_t> entry(kMaxFds, -1);
    uint32_t stack_need = base_stack;  // the deepest program of the image
    if (!order.empty()) code.push_back(RawInsn{});  // pc 0: ja to the loaded program
    for (int32_t t : order) {
      const std::vector<uint8_t> &bytes = r.progs[t].insns;
      const size_t n = bytes.size() / 8;
      if (code.size() + n + raw.size() + 1 > kMaxInsts || code.size() + n > 0x7fff) {
        link_note += "prog " + std::to_string(t) + ": image would exceed " + std::to_string(kMaxInsts) + " insns; ";
        continue;
      }
      LoadOut alone;
      std::string err;
      if (load_program((const RawInsn *)bytes.data(), n, hm, names, lddw, alone, err) < 0) {
        link_note += "prog " + std::to_string(t) + ": " + err + "; ";
        continue;
      }
      stack_need = std::max(stack_need, alone.big_stack ? kStackSize + 1 : alone.stack_size);
      entry[t] = (int32_t)code.size();
      entries.push_back((uint32_t)code.size());
      const RawInsn *c = (const RawInsn *)bytes.data();
      for (size_t i = 0; i < n; i++) {
        RawInsn x = c[i];
        if (x.code == 0x95) {  // exit -> return to the caller's frame
          x = RawInsn{};
          x.code = 0x85;
          x.imm = kRetHelper;
        }
        code.push_back(x);
        if (c[i].code == 0x18 && i + 1 < n) code.push_back(c[++i]);
      }
    }
    if (entries.empty()) {
      code.clear();  // nothing linked: the program alone
    } else {
      code[0].code = 0x05;  // ja +off
      code[0].off = (int16_t)(code.size() - 1);
    }
    code.insert(code.end(), raw.begin(), raw.end());
    if (!entries.empty()) {
      RawInsn ex{};
      ex.code = 0x95;
      code.push_back(ex);
    }
    LoadOut out;
    std::string err;
    if (load_program(code.data(), code.size(), hm, names, lddw, out, err, entries) < 0) {
      error = "tail-call image: " + err;
      return -1;
    }
    if (stack_need <= kLdsStackMax) {
      // every program's stack fits the LDS stack: the frames save that many bytes
      out.big_stack = false;
      out.stack_size = std::max<uint32_t>(8, stack_need);
    }
    auto im = std::make_shared<Image>();
    im->frame_words = (kFrameHdr + kFrameCtx + (out.big_stack ? kStackSize : out.stack_size)) / 8;
    im->gen = r.prog_gen;
    if (im->upload(std::move(out), error) < 0) return -1;
    // slot -> entry pc per reachable prog array (the image is relinked when
    // a prog, an array or a slot changes: Runtime::prog_gen)
    std::vector<int32_t> tslots(kMaxFds, -1);
    for (const auto &kv : slot_fds) {
      tslots[kv.first] = (int32_t)tslots.size();
      for (const int32_t v : kv.second)
        tslots.push_back(v >= 0 && v < (int32_t)kMaxFds && r.kind[v] == HKind::PROG ? entry[v] : -1);
    }
    if (hipMalloc((void **)&im->d_tail_entry, 4 * kMaxFds) != hipSuccess ||
        hipMemcpy(im->d_tail_entry, entry.data(), 4 * kMaxFds, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc((void **)&im->d_tail_slots, 4 * tslots.size()) != hipSuccess ||
        hipMemcpy(im->d_tail_slots, tslots.data(), 4 * tslots.size(), hipMemcpyHostToDevice) != hipSuccess) {
      error = "device upload failed";
      return -1;
    }
    img = std::move(im);
    return 0;
  }

  int exec_batch(const ebpf_batch *b);
  int exec_one(void *mem, size_t mem_len, uint64_t *ret);
};

// The message of a launch whose block does not fit the CU's LDS: the parts
// of its dynamic LDS (common.hpp dyn_lds_for) and the kernel's static LDS
std::string lds_fit_error(uint32_t kind, bool big_stack, uint32_t stack_size, uint32_t comb_entries,
                          uint32_t lcache, bool ctx_lds, bool greg, uint32_t block, bool image, uint32_t tail_lds) {
  const size_t lanes = (size_t)block * ((kind == CTX_XDP && ctx_lds ? lane_stride(kXdpCtxBytes) : 0) +
                                        (big_stack ? 0 : lane_stride(stack_size)) +
                                        tail_lds_lane_bytes(tail_lds));
  const size_t dyn = dyn_lds_for(kind, big_stack, stack_size, comb_entries, lcache, ctx_lds, block, tail_lds);
  const size_t stat = bpftime_amd_static_lds_image(kind, big_stack, greg, block, image);
  return "launch does not fit the CU's LDS: " + std::to_string(dyn + stat) + " bytes per " +
         std::to_string(block) + "-lane block (lanes' ctx, stacks and tail-call frames " + std::to_string(lanes) +
         ", lookup cache " + std::to_string(lcache) + " sets " + std::to_string(lcache_bytes(lcache)) +
         ", launch constants " + std::to_string(kTenvBytes) + ", combining table " + std::to_string(comb_entries) +
         " entries " + std::to_string(comb_bytes(comb_entries)) + ", static " + std::to_string(stat) + ") > " +
         std::to_string(kCuLds) + " (check BPFTIME_AMD_COMB_ENTRIES / BPFTIME_AMD_LCACHE_SETS)";
}

int Mi355xVm::exec_batch(const ebpf_batch *b) {
  if (!loaded) {
    error = "no program loaded";
    return -1;
  }
  if (!b || b->ctx_kind > EBPF_CTX_SYSCALL_EXIT || (b->count && !b->data) || (b->count && !b->stride && !b->descs)) {
    error = "invalid batch";
    return -1;
  }
  // the sys_exit ctx runs on the syscall kernel: only r2 (the ctx size) and
  // the window differ (EBPF_CTX_SYSCALL_EXIT, include/ebpf-vm.h)
  const bool sys_exit = b->ctx_kind == EBPF_CTX_SYSCALL_EXIT;
  const uint32_t kind = sys_exit ? CTX_SYSCALL : b->ctx_kind;
  if (b->sys_state && (kind != CTX_SYSCALL || (b->sys_phase != 1 && b->sys_phase != 2))) {
    error = "sys_state needs a syscall batch with sys_phase 1 (enter) or 2 (exit)";
    return -1;
  }
  if (b->descs && (kind == CTX_SYSCALL || !b->umem_bytes)) {
    error = "descriptor batches need an XDP / raw ctx and umem_bytes";
    return -1;
  }
  // the recorded caller / clock (include/ebpf-vm.h): syscall kinds only; an
  // offset 8-aligned with the u64 inside the unit (the kernel
  // reads it for any nonzero value, in both tiers), or an array with an
  // 8-aligned stride, not both
  {
    const uint64_t extent = sys_exit && b->stride >= 96 ? b->stride - 64 : b->stride;
    struct R {
      const char *name;
      int32_t off;
      const void *arr;
      uint64_t stride;
    };
    for (const R &o : {R{"pid_tgid", b->pid_tgid_off, b->pid_tgid_arr, b->pid_tgid_stride},
                       R{"ktime", b->ktime_off, b->ktime_arr, b->ktime_stride}}) {
      if (!o.off && !o.arr) continue;
      std::string bad;
      if (kind != CTX_SYSCALL || b->descs)
        bad = "a syscall batch only";
      else if (o.off && o.arr)
        bad = "an offset or an array, not both";
      else if (o.off && (o.off < 0 || o.off % 8 != 0 || (uint64_t)o.off + 8 > extent))
        bad = "the u64 inside the unit (8-aligned, off + 8 <= " + std::to_string(extent) + ")";
      else if (o.arr && (o.stride == 0 || o.stride % 8 != 0 || (uintptr_t)o.arr % 8 != 0))
        bad = "an 8-aligned array with a nonzero stride that is a multiple of 8";
      if (!bad.empty()) {
        error = std::string(o.name) + (o.arr ? "_arr" : "_off " + std::to_string(o.off)) + ": " + bad;
        return -1;
      }
    }
  }
  hipStream_t s = (hipStream_t)b->stream;
  if (b->count == 0) return 0;
  Runtime &r = rt();
  std::shared_ptr<Image> imp;
  {
    std::lock_guard<std::mutex> g(img_mu);
    if (has_tail && link_tail_image_locked() < 0) return -1;
    imp = img;
  }
  if (!imp) {
    error = "no program loaded";
    return -1;
  }
  Image &im = *imp;
  // the unwind helper as the device knows helpers (bpftime ids): the
  // registration that was given ubpf id unwind_idx
  int32_t unwind_helper = -1;
  for (const auto &kv : helper_id_map)
    if ((int)kv.second == unwind_idx) unwind_helper = (int32_t)kv.first;
  if (unwind_helper == (int)kTailHelper && im.d_tail_entry) {
    error = "an unwind index on bpf_tail_call is not supported on the device";
    return -1;
  }
  const LoadOut &prog = im.prog;
  KParams p{};
  p.prog = im.d_prog;
  {
    // staged window: what the static packet / slot accesses need, when every
    // slot is 16-B aligned and at least that long (a window never reaches
    // into the next unit)
    const bool xdp = kind == CTX_XDP;
    const uint32_t head = xdp ? b->head : 0;
    const uint32_t need = stage_need(xdp ? im.fx : im.fr, head);
    // (descriptor batches: the kernel checks each wave's frames)
    const bool aligned = ((uint64_t)(uintptr_t)b->data % 16) == 0 &&
                         (b->descs ? true : (b->stride % 16) == 0 && b->stride >= need);
    p.stage = (need && aligned && !getenv("BPFTIME_AMD_NO_STAGING")) ? need : 0;
    p.needs_ctx = xdp && im.fx.needs_ctx ? 1 : 0;
    p.lcache = (xdp ? im.fx : im.fr).needs_lcache ? lcache_sets() : 0;  // (sized below)
    p.fast_div = getenv("BPFTIME_AMD_NO_ASM_DIVERGENCE") ? 0 : 1;
  }
  p.maps = r.d_maptab;
  p.data = (uint8_t *)b->data;
  p.lens = kind == CTX_SYSCALL ? nullptr : b->lens;
  p.verdicts = b->verdicts;
  p.rets = b->rets;
  p.out_data_off = b->data_off_out;
  p.out_len = b->len_out;
  uint32_t *err = d_err + (err_slot.fetch_add(1) % kErrSlots);
  p.err_count = err;
  p.n = b->count;
  p.stride = b->stride;
  p.first_unit = b->first_unit;
  p.data_lo = (uint64_t)(uintptr_t)b->data;
  // (a sys_exit unit is 24 B inside its record: the window ends with the
  // last record's exit half, 32 B of a 96-B record)
  p.data_hi = p.data_lo + (b->descs  ? b->umem_bytes
                           : sys_exit ? (b->count - 1) * b->stride + (b->stride < 32 ? b->stride : 32)
                                      : b->count * b->stride);
  p.descs = (const uint64_t *)b->descs;
  p.umem_bytes = b->umem_bytes;
  p.sys_nr = (b->flags & EBPF_BATCH_SYS_NR) && kind == CTX_SYSCALL ? b->sys_nr : -1;
  p.sys_state = b->sys_state;
  p.sys_ret = b->sys_ret;
  p.sys_phase = b->sys_phase;
  p.pid_off = b->pid_tgid_off;
  if (b->pid_tgid_off) {
    p.pid_base = (const uint8_t *)b->data + b->pid_tgid_off;
    p.pid_stride = b->stride;
  } else if (b->pid_tgid_arr) {
    p.pid_base = (const uint8_t *)b->pid_tgid_arr;
    p.pid_stride = b->pid_tgid_stride;
  }
  if (b->ktime_off) {
    p.kt_base = (const uint8_t *)b->data + b->ktime_off;
    p.kt_stride = b->stride;
  } else if (b->ktime_arr) {
    p.kt_base = (const uint8_t *)b->ktime_arr;
    p.kt_stride = b->ktime_stride;
  }
  p.pid_tgid = ((uint64_t)(uint32_t)getpid() << 32) | (uint32_t)syscall(SYS_gettid);
  p.arena_lo = (uint64_t)(uintptr_t)r.arena;
  p.arena_hi = p.arena_lo + r.arena_size;
  p.step_limit = step_limit;
  // (syscall kinds: r2 = sizeof the ctx, syscall_trace_attach_impl.cpp:46)
  p.fixed_len = kind != CTX_SYSCALL ? b->fixed_len : sys_exit ? 24 : 64;
  p.stack_size = prog.stack_size;
  p.stack_stride = lane_stride(prog.stack_size);
  p.ctx_stride = lane_stride(kXdpCtxBytes);
  // ORDERED: every counter add goes straight to memory (link_fast), no table
  p.comb_entries = (b->flags & EBPF_BATCH_ORDERED) ? 0 : prog.comb_entries;
  // launches holding a combining table or lookup cache keep the C++ tier's
  // register copy in global memory (k_interp G): their units stay in the asm
  // tier, and the LDS goes to resident blocks (latency-bound: more waves
  // hide the packet and probe loads)
  const bool greg = !(b->flags & EBPF_BATCH_ORDERED) && !prog.big_stack && (p.comb_entries || p.lcache) &&
                    !getenv("BPFTIME_AMD_LDS_REGS");
  // ... and an XDP program that reads its ctx only through the specialised
  // data / data_end loads (the loader's escape analysis) keeps the ctx there
  // too: only the C++ tier reads it (48 B of LDS per lane)
  const bool gctx = greg && kind == CTX_XDP && !p.needs_ctx && !im.d_tail_entry &&
                    !getenv("BPFTIME_AMD_LDS_CTX");
  bool prog_arrays = false, rings = false;
  for (uint32_t fd = 0; fd < kMaxFds; fd++)
    if (r.kind[fd] == HKind::MAP) {
      prog_arrays |= r.maps[fd].type == MT_PROG_ARRAY;
      rings |= r.maps[fd].type == MT_RINGBUF;
    }
  const bool ordered = (b->flags & EBPF_BATCH_ORDERED) != 0;
  const bool stage = rings && !ordered && !getenv("BPFTIME_AMD_NO_RB_STAGE");
  // G launches without a tail-call image or ring staging run kBigBlock-lane
  // blocks (common.hpp): one table and lookup cache per 16 waves
  // (BPFTIME_AMD_BLOCK=256 keeps 4-wave blocks)
  uint32_t block = greg && !im.d_tail_entry && !stage ? kBigBlock : kBlock;
  const bool image = im.d_tail_entry != nullptr && !prog.big_stack;  // (bpftime_amd_launch_interp)
  if (const char *bs = getenv("BPFTIME_AMD_BLOCK"))
    if (atoi(bs) == (int)kBlock) block = kBlock;
  // the lookup cache: 1024 sets, or 2048 in a 1024-lane block whose
  // combining table would stay below 2048 entries (the LDS is there:
  // syscall-agg 0.645 -> 0.61 ms; flow-hash, whose table fills the CU, is
  // best at 1024: 2048 sets 1.08 ms, 512 0.93, 1024 0.89)
  {
    const FastForm &ff = kind == CTX_XDP ? im.fx : im.fr;
    uint32_t want = 0;
    if (prog.comb_entries) {
      want = 2 * kComb;
      if (ff.comb_hint == ~0u)
        want = 1024;
      else
        while (want < kCombMax && 32ull * want < ff.comb_hint) want *= 2;
    }
    if (p.lcache && block == kBigBlock && want < 2048 && !getenv("BPFTIME_AMD_LCACHE_SETS")) p.lcache = 2 * kLcacheSets;
    // a 1024-lane block must fit the CU with the smallest table it may get
    // (lanes' ctx and stacks, lookup cache, launch constants): drop the
    // doubled lookup cache first, then fall back to 256-lane blocks
    if (block == kBigBlock) {
      const uint32_t e_min = prog.comb_entries ? kComb : 0;
      auto fits = [&](uint32_t lc) {
        return bpftime_amd_occupancy(kind, prog.big_stack,
                                     dyn_lds_for(kind, prog.big_stack, prog.stack_size, e_min, lc, !gctx,
                                                 kBigBlock),
                                     greg, kBigBlock, image) >= 1;
      };
      if (!fits(p.lcache) && p.lcache > kLcacheSets && !getenv("BPFTIME_AMD_LCACHE_SETS")) p.lcache = kLcacheSets;
      if (!fits(p.lcache)) {
        block = kBlock;
        if (!getenv("BPFTIME_AMD_LCACHE_SETS")) p.lcache = p.lcache ? lcache_sets() : 0;
      }
    }
    p.fast = im.linked(greg, kind == CTX_XDP, kind == CTX_XDP ? b->head : 0, p.stage, ordered, unwind_helper,
                       p.lcache, b->pid_tgid_off);
    if (!p.fast) {
      error = "device upload failed";
      return -1;
    }
  }
  auto dyn_of = [&](uint32_t e) {
    return dyn_lds_for(kind, prog.big_stack, prog.stack_size, e, p.lcache, !gctx, block, p.tail_lds);
  };
  if (p.comb_entries) {
    // the table's reach: a counter that finds no entry is a device atomic
    // (memory-side, ~10 G/s chip-wide for scattered 8-byte adds), so the
    // table should hold the hot part of the counter granules a block's adds
    // can reach (the loader's hint), even at a block fewer per CU.  Measured
    // with the register copy in global memory (k_interp G, one MI355X):
    // flow-hash (65536 flows) 512 entries at 3 blocks / CU 2.71 ms, 1024 at
    // 3 1.71, 2048 at 2 1.34; syscall-agg (8192 ids) 256 at 4 1.40, 512 at
    // 4 0.68, 1024 at 3 0.74; tail-call (per-CPU counters) 256 and 512 at 4
    // 1.63, 1024 2.41.  So: hint / 32 granules, a power of two in
    // [512, kCombMax] (1024 when the loader cannot bound the addresses)
    const uint32_t hint = (kind == CTX_XDP ? im.fx : im.fr).comb_hint;
    uint32_t e = 2 * kComb;
    if (hint == ~0u)
      e = 1024;
    else
      while (e < kCombMax && 32ull * e < hint) e *= 2;
    // (a block must still fit the CU's LDS beside the lanes' ctx and stacks;
    // the sets may be any count, gen_fast.py comb_add.  Measured: trading
    // reach for a resident block does not pay -- flow-hash 2048 entries at 2
    // blocks / CU 1.32 ms, 1792 at 3 1.57, 1536 at 3 1.42 -- nor does reach
    // beyond hint / 32 at the same residency: flow-hash 3072 1.29,
    // syscall-agg 768 / 984 0.672 / 0.677 against 512 0.664)
    while (e > kComb && bpftime_amd_occupancy(kind, prog.big_stack, dyn_of(e), greg, block, image) < 1) e /= 2;
    // one 1024-lane block per CU: a table that wants 2048 entries or more
    // takes the rest of the CU's LDS (multiples of 8 ways), since every
    // counter it misses is a memory-side atomic.  Measured (flow-hash, one
    // MI355X, same box): 2048 entries 1.027 ms, 2560 0.980, 3072 0.945,
    // 3584 0.914, 3840 0.898, 4032 0.891
    if (block == kBigBlock && e >= 2048) {
      static std::mutex fill_mu;
      static std::map<size_t, uint32_t> fill;  // (dyn_of(0), ctx kind) -> the largest table that fits
      std::lock_guard<std::mutex> g(fill_mu);
      const size_t key = dyn_of(0) * 4 + kind;
      auto it = fill.find(key);
      if (it == fill.end()) {
        uint32_t f = kCombMax;
        while (f > e && bpftime_amd_occupancy(kind, prog.big_stack, dyn_of(f), greg, block, image) < 1) f -= 32;
        it = fill.emplace(key, f).first;
      }
      e = it->second > e ? it->second : e;
    }
    // (an override that does not fit the CU fails the batch below, named)
    if (const char *ce = getenv("BPFTIME_AMD_COMB_ENTRIES")) e = (uint32_t)atoi(ce) & ~7u;
    p.comb_entries = e;
  }
  p.ncpu = r.ncpu;
  p.unwind_idx = unwind_helper;
  p.ifindex = b->ingress_ifindex;
  p.rxq = b->rx_queue_index;
  p.head = b->head;
  p.checked = (b->flags & EBPF_BATCH_UNCHECKED) ? 0 : 1;
  if (const char *d = getenv("BPFTIME_AMD_DBG")) p.dbg = (uint32_t)strtoul(d, nullptr, 0) & ~kDbgXlat;
  if (p.dbg & 512) p.dbg_counts = dbg_counts();
  // every block of the launch must fit the CU's LDS (env overrides of the
  // table / cache sizes included): a launch that needs more fails, named,
  // instead of running at an occupancy of zero
  // XDP images: the asm tier's frames of the first depths in LDS, as many
  // depths (kTailLdsMax at most) as keep the block's residency
  // (BPFTIME_AMD_TAIL_LDS: at most that many; 0 = every frame in global memory)
  if (image && kind == CTX_XDP && !(p.dbg & 8)) {
    const FastForm &ff = im.fx;
    const uint32_t sw = prog.stack_size / 8;
    const uint32_t words = 1 + ff.tail_max_live + (uint32_t)__builtin_popcount(ff.tail_ctx_mask & 0x3f) +
                           (uint32_t)__builtin_popcount(ff.tail_stack_mask & (sw >= 16 ? 0xffffu : (1u << sw) - 1));
    uint32_t most = kTailLdsMax;
    if (const char *t = getenv("BPFTIME_AMD_TAIL_LDS")) most = std::min<uint32_t>((uint32_t)atoi(t), kTailLdsMax);
    p.tail_lds = 0;
    const int occ0 = bpftime_amd_occupancy(kind, prog.big_stack, dyn_of(p.comb_entries), greg, block, image);
    auto depths = [&](uint32_t e) -> uint32_t {
      for (uint32_t dl = most; dl >= 1 && occ0 >= 1; dl--) {
        p.tail_lds = dl | words << 8;
        const bool ok = bpftime_amd_occupancy(kind, prog.big_stack, dyn_of(e), greg, block, image) >= occ0;
        p.tail_lds = 0;
        if (ok) return dl;
      }
      return 0;
    };
    uint32_t dl = depths(p.comb_entries);
    // a combining table above the size its counters need (the loader's hint:
    // kComb entries hold them) gives way to a deeper LDS frame stack
    if (dl < most && p.comb_entries > kComb && 32ull * kComb >= ff.comb_hint && !getenv("BPFTIME_AMD_COMB_ENTRIES")) {
      const uint32_t dl2 = depths(kComb);
      if (dl2 > dl) {
        dl = dl2;
        p.comb_entries = kComb;
      }
    }
    p.tail_lds = dl ? dl | words << 8 : 0;
  }
  const size_t lds_need = dyn_of(p.comb_entries);
  const int occ_fit = bpftime_amd_occupancy(kind, prog.big_stack, lds_need, greg, block, image);
  if (occ_fit < 1) {
    error = lds_fit_error(kind, prog.big_stack, prog.stack_size, p.comb_entries, p.lcache, !gctx, greg, block, image,
                          p.tail_lds);
    return -1;
  }
  {
    const hipError_t me = hipMemsetAsync(err, 0, 4, s);
    if (me != hipSuccess) {
      error = std::string("hipMemsetAsync failed: ") + hipGetErrorString(me) +
              " (an earlier operation on this stream or device may have failed)";
      return -1;
    }
  }
  // program-side LPM trie updates / deletes: the device changes a trie only
  // in ORDERED batches (one lane, the reference's order: dev_helpers.hpp
  // lpm_update), the host takes the replica back afterwards (lpm_pull)
  std::vector<int> lpm_w;
  uint32_t lpm_updates = 0;
  for (const auto &w : (kind == CTX_XDP ? im.fx : im.fr).lpm_writes) {
    lpm_updates += w.first == 2;
    if (!(b->flags & EBPF_BATCH_ORDERED)) {
      error = std::string(w.first == 2 ? "bpf_map_update_elem" : "bpf_map_delete_elem") +
              " on LPM_TRIE map fd " + std::to_string(w.second) +
              ": program-side LPM trie writes run only in EBPF_BATCH_ORDERED batches";
      return -1;
    }
    if (std::find(lpm_w.begin(), lpm_w.end(), w.second) == lpm_w.end()) lpm_w.push_back(w.second);
  }
  // the lookup cache trusts a found slot for the whole launch: no deletion
  // may run beside it (Runtime::lcache_inflight)
  if ((p.lcache && r.deleter_inflight.load()) || (prog.may_delete && r.lcache_inflight.load())) {
    if (hipDeviceSynchronize() != hipSuccess) {
      error = "device synchronize failed";
      return -1;
    }
    r.lcache_inflight = false;
    r.deleter_inflight = false;
  }
  // LPM tries: a launch of a program that writes one (ORDERED) never
  // overlaps another launch that may touch one, on any stream -- whichever
  // comes second waits for the device -- and the launch and its marking of
  // the tries as device-written happen under one lock, so a concurrent
  // launch's preparation sees them
  std::unique_lock<std::mutex> lpm_lk(r.lpm_launch_mu, std::defer_lock);
  // (only launches of programs that name a trie: others need
  // neither the lock nor the in-flight marks, and a writer waits for them)
  const bool names_lpm = (kind == CTX_XDP ? im.fx : im.fr).names_lpm;
  const bool touches_lpm = r.lpm_maps.load() > 0 && names_lpm;
  if (touches_lpm) {
    lpm_lk.lock();
    if ((!lpm_w.empty() && r.lpm_inflight.load()) || r.lpm_writer_inflight.load()) {
      if (hipDeviceSynchronize() != hipSuccess) {
        error = "device synchronize failed";
        return -1;
      }
      r.lpm_inflight = false;
      r.lpm_writer_inflight = false;
    }
  }
  if (r.prepare_ix(prog.may_delete, b->count, lpm_w, lpm_updates, names_lpm) < 0) {
    // (an LPM trie's report names itself; else the index rebuild failed)
    const std::string le = bpftime_amd_last_error() ? bpftime_amd_last_error() : "";
    error = le.rfind("LPM_TRIE", 0) == 0 ? le : "hash lookup index rebuild failed";
    return -1;
  }
  p.lru_seq = r.prepare_lru();
  if (!p.lru_seq) {
    error = "LRU table upkeep failed";
    return -1;
  }
  uint32_t grid = 1;
  if (!ordered) {
    static int cus = 0;
    if (!cus) {
      hipDeviceProp_t prop;
      int dev = 0;
      hipGetDevice(&dev);
      hipGetDeviceProperties(&prop, dev);
      cus = prop.multiProcessorCount;
    }
    const int occ = occ_fit;
    uint64_t want = (b->count + block - 1) / block;
    // one wave per resident wave slot (x 1): every wave launch writes the
    // kernel's register spills (ScratchSize ~200 B / lane) once, and at x 4
    // those writes were 12 B of memory-side traffic per packet
    // (tools/grid_write_probe.sh, xdp-counter WRITE_SIZE 39.1 / 42.3 / 48.5 /
    // 61.0 B per packet at x 1 / 2 / 4 / 8; 0.467 / 0.479 / 0.496 / 0.484 ms;
    // lpm-route 0.467 / 0.479 / 0.506 ms at x 1 / 2 / 4); a combining table
    // is flushed once per block (flow-hash 0.60 -> 1.09 ms at x 4).  Ring
    // staging too, with an 8-KiB budget per block (common.hpp kRbStageRec;
    // ringbuf-sample 1.10 / 1.21 / 1.47 ms at x 1 / 2 / 4; with the 2-KiB
    // budget 7.46 / 4.03 / 1.43).  BPFTIME_AMD_GRID_MULT overrides.
    uint32_t mult = 1;
    if (const char *g = getenv("BPFTIME_AMD_GRID_MULT"))
      if (atoi(g) > 0) mult = (uint32_t)atoi(g);
    uint64_t cap = (uint64_t)cus * (uint64_t)occ * mult;
    grid = (uint32_t)(want < cap ? want : cap);
    // (tests: few blocks, so that small batches take many units per lane)
    if (const char *g = getenv("BPFTIME_AMD_MAX_GRID"))
      if (atoi(g) > 0 && grid > (uint32_t)atoi(g)) grid = (uint32_t)atoi(g);
    if (im.d_tail_entry && grid > kTailGrid) grid = kTailGrid;  // one frame stack per lane of the grid
  }
  {
    const uint64_t ustep = (uint64_t)grid * block;
    p.full_q = p.n >= 64 ? (p.n - 64) / ustep : 0;
    p.full_r = p.n >= 64 ? (p.n - 64) % ustep : 0;
    p.step_cpu = ordered ? 0 : (uint32_t)((ustep / 64) % (p.ncpu ? p.ncpu : 1));
  }
  if (greg) {
    p.gregs = (uint64_t *)regs.get(s, (uint64_t)grid * 11 * block * 8);
    if (!p.gregs) {
      error = "register copy allocation failed";
      return -1;
    }
  }
  if (im.d_tail_entry) {
    // tail-call frames for the lanes of this launch ([depth][word][lane]),
    // one buffer per stream: concurrent batches never share frames
    p.tail_entry = im.d_tail_entry;
    p.tail_slots = im.d_tail_slots;
    p.frame_words = im.frame_words;
    p.tail_ctx_mask = im.fx.tail_ctx_mask;
    p.tail_stack_mask = im.fx.tail_stack_mask;
    const uint64_t fbytes = (uint64_t)grid * kBlock * kTailDepth * im.frame_words * 8;
    p.frames = (uint8_t *)frames.get(s, fbytes);
    if (!p.frames) {
      error = "tail-call frame allocation failed (" + std::to_string(fbytes >> 20) + " MiB)";
      return -1;
    }
  }
  // a scratch word per lane while prog arrays exist (device map_lookup_elem
  // on one hands out a copy of the fd there, prog_array.cpp:113-143), after
  // them the blocks' ring-buffer staging areas while ring buffers exist
  // (dev_helpers.hpp RbStage; not in ORDERED batches: exact order), then the
  // lanes' global XDP ctx (gctx)
  {
    if (prog_arrays || stage || gctx) {
      const uint64_t words = (uint64_t)grid * block * 8, sbytes = stage ? (uint64_t)grid * kRbStageBytes : 0;
      uint8_t *base = (uint8_t *)scratch.get(s, words + sbytes + (gctx ? 48ull * grid * block : 0));
      if (!base) {
        error = "lane scratch allocation failed";
        return -1;
      }
      p.lane_scratch = (uint64_t *)base;
      p.rb_stage = stage ? base + words : nullptr;
      p.gctx = gctx ? base + words + sbytes : nullptr;
    }
  }
  // a block-end flush log when the blocks hold per-lane counter tables:
  // merged by a second launch instead of every block adding its table
  if (p.comb_entries && grid > kMergeGroup && !getenv("BPFTIME_AMD_NO_MERGE")) {
    p.log_words = log_words_for(p.comb_entries, block);
    p.flush_log = (uint64_t *)logs.get(s, (uint64_t)grid * p.log_words * 8);
    if (!p.flush_log) {
      error = "flush log allocation failed";
      return -1;
    }
  }
  // the combining tables' miss log (common.hpp kMissParts): records per
  // block and partition for a quarter of the block's units missing with a
  // pair each, at most 256 MiB of log.  Opt-in (BPFTIME_AMD_MISS_LOG=1):
  // measured on flow-hash, the interpreter kernel gains 0.06 ms per 2^24
  // frames (0.89 -> 0.83) but k_miss_merge costs 0.18 ms -- the misses of
  // moderately hot flows reach one merge block from every source block and
  // serialize on its LDS atomics -- so by default misses add directly
  if (p.comb_entries && grid > 1 && getenv("BPFTIME_AMD_MISS_LOG") && atoi(getenv("BPFTIME_AMD_MISS_LOG")) > 0) {
    const uint64_t upb = (b->count + grid - 1) / grid;
    uint64_t cap = upb * 2 / 4 / kMissParts;
    const uint64_t most = (256ull << 20) / ((uint64_t)grid * kMissParts * 16);
    cap = cap < 16 ? 16 : cap;
    cap = cap > most ? most : cap;
    if (const char *mc = getenv("BPFTIME_AMD_MISS_CAP")) cap = strtoull(mc, nullptr, 0);  // (tests: overflow)
    cap &= ~1ull;
    if (cap >= 2) {
      // (the counts, then a u32 of records the merge refused: a log that
      // names an address outside the windows is never added)
      const uint64_t cbytes = ((uint64_t)grid * kMissParts * 4 + 4 + 255) & ~255ull;
      uint8_t *m = (uint8_t *)misses.get(s, cbytes + (uint64_t)grid * kMissParts * cap * 16);
      if (!m) {
        error = "miss log allocation failed";
        return -1;
      }
      p.miss_counts = (uint32_t *)m;
      if (hipMemsetAsync(m + (uint64_t)grid * kMissParts * 4, 0, 4, s) != hipSuccess) {
        error = "miss log reset failed";
        return -1;
      }
      p.miss_log = (uint64_t *)(m + cbytes);
      p.miss_cap = (uint32_t)cap;
    }
  }
  if (r.host_views_push() < 0) {  // host writes to mmap'd array maps first
    error = "host view upload failed";
    return -1;
  }
  if (getenv("BPFTIME_AMD_VERBOSE"))
    fprintf(stderr,
            "bpftime_amd: launch units %llu grid %u block %u comb %u lcache %u stage %u stack %u gregs %d gctx %d unwind %d "
            "miss cap %u tail lds %u x %u words occ %d\n",
            (unsigned long long)b->count, grid, block, p.comb_entries, p.lcache, p.stage, (unsigned)prog.stack_size,
            p.gregs ? 1 : 0, p.gctx ? 1 : 0, p.unwind_idx, p.miss_cap, p.tail_lds & 0xff, p.tail_lds >> 8, occ_fit);
  // EBPF_BATCH_TIMED: events around this batch's kernels only (the host
  // work above -- linking, buffers, index upkeep -- stays outside)
  const bool timed = (b->flags & EBPF_BATCH_TIMED) != 0;
  if (timed) {
    if ((!ev_t0 && hipEventCreate(&ev_t0) != hipSuccess) || (!ev_t1 && hipEventCreate(&ev_t1) != hipSuccess) ||
        hipEventRecord(ev_t0, s) != hipSuccess) {
      error = "timing event failed";
      return -1;
    }
  }
  hipError_t e = bpftime_amd_launch_interp(&p, kind, prog.big_stack, grid, ordered ? 1 : 0, block, s);
  // (BPFTIME_AMD_SYNC_EACH: synchronize after every launch, naming the one that failed)
  const bool sync_each = getenv("BPFTIME_AMD_SYNC_EACH") != nullptr;
  auto step = [&](const char *what, hipError_t le) {
    if (le == hipSuccess && sync_each) le = hipStreamSynchronize(s);
    if (le != hipSuccess && sync_each) fprintf(stderr, "bpftime_amd: %s: %s\n", what, hipGetErrorString(le));
    return le;
  };
  e = step("k_interp", e);
  if (e == hipSuccess && p.flush_log) e = step("k_comb_merge", bpftime_amd_launch_merge(p.flush_log, p.log_words, grid, s));
  if (e == hipSuccess && p.miss_log)
    e = step("k_miss_merge", bpftime_amd_launch_miss_merge(p.miss_log, p.miss_counts, p.miss_cap, grid, &p,
                                                           p.miss_counts + (uint64_t)grid * kMissParts, s));
  if (e == hipSuccess && p.miss_log && sync_each) {
    uint32_t bad = 0;
    hipMemcpy(&bad, p.miss_counts + (uint64_t)grid * kMissParts, 4, hipMemcpyDeviceToHost);
    if (bad) fprintf(stderr, "bpftime_amd: k_miss_merge: %u records outside the windows\n", bad);
  }
  if (e == hipSuccess && timed) e = hipEventRecord(ev_t1, s);
  if (e != hipSuccess) {
    error = std::string("kernel launch failed: ") + hipGetErrorString(e);
    return -1;
  }
  if (p.lcache) r.lcache_inflight = true;
  if (prog.may_delete) r.deleter_inflight = true;
  if (!lpm_w.empty()) {
    std::lock_guard<std::mutex> g(r.mu);
    for (const int fd : lpm_w) r.lpm_dev_dirty.insert(fd);
    r.lpm_writer_inflight = true;
  }
  if (touches_lpm) {
    r.lpm_inflight = true;
    lpm_lk.unlock();
  }
  if (b->flags & EBPF_BATCH_SYNC) {
    uint32_t failed = 0;
    hipError_t he = hipMemcpyAsync(&failed, err, 4, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he != hipSuccess || r.host_views_pull() < 0) {
      error = std::string("batch sync failed: ") + (he != hipSuccess ? hipGetErrorString(he) : "host view pull");
      return -1;
    }
    // a program-side LPM update that ran out of the device node pool fails
    // the batch here (maps.cpp lpm_pull; asynchronous batches report it at
    // the trie's next use)
    for (const int fd : lpm_w) {
      std::lock_guard<std::mutex> g(r.mu);
      if (lpm_pull(fd) < 0) {
        error = bpftime_amd_last_error();
        return -1;
      }
    }
    return (int)failed;
  }
  return 0;
}

// ebpf_exec: one unit, copied to the device and back.
int Mi355xVm::exec_one(void *mem, size_t mem_len, uint64_t *ret) {
  if (!loaded) {
    error = "no program loaded";
    return -1;
  }
  struct XdpMd {
    uint64_t data, data_end;
    uint32_t data_meta, ingress_ifindex, rx_queue_index, egress_ifindex;
    uint64_t buffer_start, buffer_end;
  };
  uint8_t *host_base;
  size_t slot_bytes;
  uint32_t head = 0, len;
  XdpMd *x = nullptr;
  if (ctx_kind == CTX_XDP) {
    x = (XdpMd *)mem;
    uint64_t lo = x->buffer_start && x->buffer_start <= x->data ? x->buffer_start : x->data;
    uint64_t hi = x->buffer_end && x->buffer_end >= x->data_end ? x->buffer_end : x->data_end;
    host_base = (uint8_t *)(uintptr_t)lo;
    slot_bytes = hi - lo;
    head = (uint32_t)(x->data - lo);
    len = (uint32_t)(x->data_end - x->data);
  } else {
    host_base = (uint8_t *)mem;
    slot_bytes = mem_len;
    len = (uint32_t)mem_len;
  }
  std::lock_guard<std::mutex> sg(stage_mu);  // one ebpf_exec at a time per VM uses the staging buffer
  size_t need = ((slot_bytes + 255) & ~(size_t)255) + 64;
  if (need > stage_size) {
    if (d_stage) hipFree(d_stage);
    if (hipMalloc((void **)&d_stage, need) != hipSuccess) {
      d_stage = nullptr;
      stage_size = 0;
      error = "staging alloc failed";
      return -1;
    }
    stage_size = need;
  }
  uint8_t *d_slot = d_stage + 64;
  uint64_t *d_ret = (uint64_t *)d_stage;
  int32_t *d_off = (int32_t *)(d_stage + 8);
  uint32_t *d_len = (uint32_t *)(d_stage + 12);
  if (slot_bytes && hipMemcpy(d_slot, host_base, slot_bytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
  ebpf_batch b{};
  b.ctx_kind = ctx_kind;
  b.flags = EBPF_BATCH_SYNC | EBPF_BATCH_ORDERED;
  b.count = 1;
  b.data = d_slot;
  b.stride = slot_bytes ? slot_bytes : 1;
  b.fixed_len = len;
  b.head = head;
  b.rets = d_ret;
  if (x) {
    b.data_off_out = d_off;
    b.len_out = d_len;
    b.ingress_ifindex = x->ingress_ifindex;
    b.rx_queue_index = x->rx_queue_index;
  }
  int failed = exec_batch(&b);
  if (failed < 0) return -1;
  uint8_t hdr[16];
  if (hipMemcpy(hdr, d_stage, 16, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (slot_bytes && hipMemcpy(host_base, d_slot, slot_bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (failed) {
    error = "program execution failed on device";
    return -1;
  }
  uint64_t r0;
  memcpy(&r0, hdr, 8);
  if (x) {
    int32_t off;
    uint32_t l;
    memcpy(&off, hdr + 8, 4);
    memcpy(&l, hdr + 12, 4);
    x->data = (uint64_t)(uintptr_t)host_base + (uint64_t)(int64_t)off;
    x->data_end = x->data + l;
  }
  *ret = r0;
  return 0;
}

}  // namespace bpftime_amd

using namespace bpftime_amd;

// ebpf-vm.cpp's struct ebpf_vm {vm_name; vm_instance} (bpftime_vm_compat.hpp:260-263)
struct ebpf_vm {
  std::string vm_name;
  Mi355xVm *impl;
};

namespace bpftime_amd {
int vm_prog_flags(const ::ebpf_vm *vm) {
  if (!vm || !vm->impl->loaded) return -1;
  auto im = vm->impl->image();
  if (!im) return -1;
  return (im->prog.sets_retval ? kProgSetsRetval : 0) | (im->fr.stores_unit ? kProgStoresCtx : 0);
}

int vm_map_effects(const ::ebpf_vm *vm, std::map<int32_t, uint8_t> &fx, uint8_t &any) {
  if (!vm || !vm->impl->loaded) return -1;
  auto im = vm->impl->image();
  if (!im) return -1;
  fx = im->fr.map_fx;
  any = im->fr.any_fx;
  return 0;
}

extern "C" hipError_t bpftime_amd_launch_sys_seq(const SeqParams *p, hipStream_t stream);

int64_t seq_dispatch(const std::vector<SeqAttach> &progs, const SysLayout &lay, uint64_t n, const uint32_t *perm,
                     const uint32_t *seg, uint64_t nseg, int64_t *out, uint32_t flags, uint32_t *err, hipStream_t s) {
  auto fail = [](const std::string &e) {
    set_error("thread-ordered dispatch: " + e);
    return (int64_t)-1;
  };
  if (progs.size() > kSeqMaxProgs)
    return fail(std::to_string(progs.size()) + " programs attached (at most " + std::to_string(kSeqMaxProgs) + ")");
  Runtime &r = rt();
  SeqParams p{};
  // the images stay referenced until the launch is queued (a relink by
  // another thread never frees what is read: Image, above)
  std::vector<std::shared_ptr<Image>> keep;
  const bool ordered = (flags & EBPF_BATCH_ORDERED) != 0;
  bool may_delete = false, names_lpm = false;
  std::vector<int> lpm_w;
  uint32_t lpm_updates = 0;
  uint64_t steps = 0;
  // the asm tier runs the callbacks when every stack fits the LDS stacks and
  // the threads are at most kSeqAsmThreads: measured (profiles/
  // r06_seq_xover.txt, syscount's pair) 2-3.7x the C++ tier up to 8192
  // threads, even at 16384, and behind it from 32768 on, where the waves no
  // longer wait on their own latency chains and the map helpers' coherent
  // atomics set the rate.  BPFTIME_AMD_SEQ_ASM=1 / 0 forces a tier.
  const char *asm_env = getenv("BPFTIME_AMD_SEQ_ASM");
  bool fast = asm_env && asm_env[0] ? asm_env[0] != '0' : nseg <= kSeqAsmThreads;
  // constant-address loads (loader.cpp const_loads: array storage nothing in
  // THAT program writes) stay scalar-cache loads only while no attached
  // program writes or adds to an array map: one launch runs them all
  bool array_writes = false;
  for (const SeqAttach &a : progs) {
    auto im = a.vm->impl->image();
    if (!im) continue;
    fast = fast && !im->prog.big_stack && im->prog.stack_size <= kLdsStackMax;
    const uint8_t w = FX_WRITE | FX_ADD;
    array_writes = array_writes || (im->fr.any_fx & w);
    for (const auto &kv : im->fr.map_fx)
      if ((kv.second & w) && kv.first >= 0 && kv.first < (int32_t)kMaxFds &&
          (r.maps[kv.first].type == MT_ARRAY || r.maps[kv.first].type == MT_PERCPU_ARRAY))
        array_writes = true;
  }
  for (const SeqAttach &a : progs) {
    Mi355xVm *vm = a.vm->impl;
    auto im = vm->image();
    if (!vm->loaded || !im) return fail("an attached program is not loaded");
    if (vm->has_tail) return fail("an attached program calls bpf_tail_call (program-major dispatch runs it)");
    const FInsn *f = im->linked(false, false, 0, 0, true, -1, 0, 0, array_writes && progs.size() > 1, fast);
    if (!f) return fail("device upload failed");
    SeqProg &q = p.progs[p.nprogs++];
    q.prog = im->d_prog;
    q.fast = f;
    q.sys_nr = a.sys_nr;
    q.enter = a.enter ? 1 : 0;
    may_delete |= im->prog.may_delete;
    names_lpm |= im->fr.names_lpm;
    for (const auto &w : im->fr.lpm_writes) {
      if (!ordered)
        return fail(std::string(w.first == 2 ? "bpf_map_update_elem" : "bpf_map_delete_elem") +
                    " on LPM_TRIE map fd " + std::to_string(w.second) +
                    ": program-side LPM trie writes run only in EBPF_BATCH_ORDERED batches");
      lpm_updates += w.first == 2;
      if (std::find(lpm_w.begin(), lpm_w.end(), w.second) == lpm_w.end()) lpm_w.push_back(w.second);
    }
    steps = std::max(steps, vm->step_limit);
    keep.push_back(std::move(im));
  }
  p.lay = lay;
  p.n = n;
  p.perm = perm;
  p.seg = seg;
  p.nseg = nseg;
  p.out = out;
  p.maps = r.d_maptab;
  p.ncpu = r.ncpu;
  p.checked = (flags & EBPF_BATCH_UNCHECKED) ? 0 : 1;
  p.arena_lo = (uint64_t)(uintptr_t)r.arena;
  p.arena_hi = p.arena_lo + r.arena_size;
  p.step_limit = steps;
  p.pid_tgid = ((uint64_t)(uint32_t)getpid() << 32) | (uint32_t)syscall(SYS_gettid);
  p.err_count = err;
  p.exact = ordered ? 1 : 0;
  p.fast = fast ? 1 : 0;
  // the map upkeep exec_batch does before a launch, for the union of the
  // programs (a deletion never runs beside a cached launch; LPM launches
  // under the LPM launch lock; lookup indexes; LRU stamps; host views)
  if (may_delete && r.lcache_inflight.load()) {
    if (hipDeviceSynchronize() != hipSuccess) return fail("device synchronize failed");
    r.lcache_inflight = false;
    r.deleter_inflight = false;
  }
  std::unique_lock<std::mutex> lpm_lk(r.lpm_launch_mu, std::defer_lock);
  const bool touches_lpm = r.lpm_maps.load() > 0 && names_lpm;
  if (touches_lpm) {
    lpm_lk.lock();
    if ((!lpm_w.empty() && r.lpm_inflight.load()) || r.lpm_writer_inflight.load()) {
      if (hipDeviceSynchronize() != hipSuccess) return fail("device synchronize failed");
      r.lpm_inflight = false;
      r.lpm_writer_inflight = false;
    }
  }
  if (r.prepare_ix(may_delete, n, lpm_w, lpm_updates, names_lpm) < 0) {
    const std::string le = bpftime_amd_last_error() ? bpftime_amd_last_error() : "";
    return fail(le.rfind("LPM_TRIE", 0) == 0 ? le : "hash lookup index rebuild failed");
  }
  p.lru_seq = r.prepare_lru();
  if (!p.lru_seq) return fail("LRU table upkeep failed");
  if (r.host_views_push() < 0) return fail("host view upload failed");
  hipError_t e = hipMemsetAsync(err, 0, 4, s);
  if (e == hipSuccess) e = bpftime_amd_launch_sys_seq(&p, s);
  if (e != hipSuccess) return fail(std::string("kernel launch failed: ") + hipGetErrorString(e));
  if (may_delete) r.deleter_inflight = true;
  if (!lpm_w.empty()) {
    std::lock_guard<std::mutex> g(r.mu);
    for (const int fd : lpm_w) r.lpm_dev_dirty.insert(fd);
    r.lpm_writer_inflight = true;
  }
  if (touches_lpm) {
    r.lpm_inflight = true;
    lpm_lk.unlock();
  }
  if (!(flags & EBPF_BATCH_SYNC)) return 0;
  uint32_t failed = 0;
  e = hipMemcpyAsync(&failed, err, 4, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess || r.host_views_pull() < 0)
    return fail(std::string("sync failed: ") + (e != hipSuccess ? hipGetErrorString(e) : "host view pull"));
  for (const int fd : lpm_w) {
    std::lock_guard<std::mutex> g(r.mu);
    if (lpm_pull(fd) < 0) return -1;
  }
  return failed;
}
}  // namespace bpftime_amd

extern "C" {

struct ebpf_vm *ebpf_create(const char *vm_name) {
  if (!vm_name || strcmp(vm_name, "mi355x") != 0) return nullptr;
  ebpf_vm *vm = new ebpf_vm;
  vm->impl = new Mi355xVm();
  return vm;
}

void ebpf_destroy(struct ebpf_vm *vm) {
  if (!vm) return;
  delete vm->impl;
  delete vm;
}

const char *ebpf_get_vm_name(struct ebpf_vm *vm) { return vm->vm_name.c_str(); }

bool ebpf_toggle_bounds_check(struct ebpf_vm *vm, bool enable) {
  bool prev = vm->impl->bounds_check;
  vm->impl->bounds_check = enable;
  return prev;
}

void ebpf_set_error_print(struct ebpf_vm *vm, int (*error_printf)(FILE *, const char *, ...)) {
  vm->impl->error_print = error_printf;
}

int ebpf_register(struct ebpf_vm *vm, unsigned int index, const char *name, void *fn) {
  return vm->impl->register_external_function(index, name ? name : "", fn);
}

int ebpf_load(struct ebpf_vm *vm, const void *code, uint32_t code_len, char **errmsg) {
  int err = vm->impl->load_code(code, code_len);
  if (err < 0 && errmsg) *errmsg = strdup(vm->impl->error.c_str());
  return err;
}

void ebpf_unload_code(struct ebpf_vm *vm) { vm->impl->unload(); }

int ebpf_exec(const struct ebpf_vm *vm, void *mem, size_t mem_len, uint64_t *bpf_return_value) {
  return vm->impl->exec_one(mem, mem_len, bpf_return_value);
}

ebpf_jit_fn ebpf_compile(struct ebpf_vm *vm, char **errmsg) {
  vm->impl->error = "mi355x is a device interpreter: use ebpf_exec / ebpf_exec_batch";
  if (errmsg) *errmsg = strdup(vm->impl->error.c_str());
  return nullptr;
}

// compat_ubpf.cpp:239-241 -> ubpf_set_unwind_function_index: a call of
// helper idx that returns 0 ends the program with r0 = 0 (interp.hip R_CALL)
// (idx is a ubpf helper id, the id register_external_function gave it)
int ebpf_set_unwind_function_index(struct ebpf_vm *vm, unsigned int idx) {
  if (idx >= 64) return -1;  // ubpf's MAX_EXT_FUNCS
  vm->impl->unwind_idx = (int)idx;
  return 0;
}

int ebpf_set_pointer_secret(struct ebpf_vm *vm, uint64_t secret) {
  (void)vm;
  (void)secret;
  return -1;
}

void ebpf_set_lddw_helpers(struct ebpf_vm *vm, uint64_t (*map_by_fd)(uint32_t), uint64_t (*map_by_idx)(uint32_t),
                           uint64_t (*map_val)(uint64_t), uint64_t (*var_addr)(uint32_t),
                           uint64_t (*code_addr)(uint32_t)) {
  LddwHelpers &l = vm->impl->lddw;
  l.map_by_fd = map_by_fd ? map_by_fd : nullptr;
  l.map_by_idx = map_by_idx;
  l.map_val = map_val;
  l.var_addr = var_addr;
  l.code_addr = code_addr;
}

ebpf_jit_fn ebpf_load_aot_object(struct ebpf_vm *vm, const void *buf, size_t buf_len) {
  (void)buf;
  (void)buf_len;
  vm->impl->error = "AOT objects are not supported by the mi355x interpreter";
  return nullptr;
}

int ebpf_exec_batch(const struct ebpf_vm *vm, const struct ebpf_batch *batch) {
  if (!vm) return -1;
  return vm->impl->exec_batch(batch);
}

int ebpf_set_ctx_kind(struct ebpf_vm *vm, uint32_t ctx_kind) {
  if (ctx_kind > EBPF_CTX_SYSCALL_EXIT) return -1;
  vm->impl->ctx_kind = ctx_kind;
  return 0;
}

// ---- runtime glue ----------------------------------------------------------
int bpftime_amd_register_default_helpers(struct ebpf_vm *vm) {
  // kernel helper group + shm maps group subset (bpf_helper.cpp:1177-1401)
  static const struct {
    unsigned id;
    const char *name;
  } h[] = {{8, "bpf_get_smp_processor_id"}, {28, "bpf_csum_diff"},    {44, "bpf_xdp_adjust_head"},
           {65, "bpf_xdp_adjust_tail"},      {5, "bpf_ktime_get_ns"}, {7, "bpf_get_prandom_u32"},
           {131, "bpf_ringbuf_reserve"},     {132, "bpf_ringbuf_submit"}, {133, "bpf_ringbuf_discard"},
           {130, "bpf_ringbuf_output"},      {12, "bpf_tail_call"},
           {1, "bpf_map_lookup_elem"},       {2, "bpf_map_update_elem"}, {3, "bpf_map_delete_elem"},
           {58, "bpf_override_return"},      {187, "bpf_set_retval"},
           {14, "bpf_get_current_pid_tgid"}};
  int err = 0;
  for (auto &e : h) err |= ebpf_register(vm, e.id, e.name, nullptr);
  return err ? -1 : 0;
}

struct ebpf_vm *bpftime_amd_prog_instantiate(int prog_fd, char **errmsg) {
  Runtime &r = rt();
  if (prog_fd < 0 || prog_fd >= (int)kMaxFds || r.kind[prog_fd] != HKind::PROG) {
    if (errmsg) *errmsg = strdup("not a prog fd");
    return nullptr;
  }
  std::vector<uint8_t> insns = r.progs[prog_fd].insns;
  int type = r.progs[prog_fd].type;
  ebpf_vm *vm = ebpf_create("mi355x");
  bpftime_amd_register_default_helpers(vm);
  if (type == BPFTIME_AMD_PROG_TYPE_XDP) vm->impl->ctx_kind = CTX_XDP;
  if (type == BPFTIME_AMD_PROG_TYPE_TRACEPOINT) vm->impl->ctx_kind = CTX_SYSCALL;
  if (ebpf_load(vm, insns.data(), (uint32_t)insns.size(), errmsg) < 0) {
    ebpf_destroy(vm);
    return nullptr;
  }
  return vm;
}

int bpftime_amd_vm_info(const struct ebpf_vm *vm, uint32_t *stack_size, int *big_stack, uint32_t *fused_rmw,
                        uint32_t *n_insns) {
  if (!vm || !vm->impl->loaded) return -1;
  auto im = vm->impl->image();
  if (stack_size) *stack_size = im->prog.stack_size;
  if (big_stack) *big_stack = im->prog.big_stack;
  if (fused_rmw) *fused_rmw = im->prog.fused_rmw;
  if (n_insns) *n_insns = (uint32_t)im->prog.prog.size();
  return 0;
}

int bpftime_amd_vm_fast_info(const struct ebpf_vm *vm, uint32_t ctx_kind, uint32_t *specialized) {
  if (!vm || !vm->impl->loaded) return -1;
  auto im = vm->impl->image();
  if (specialized) *specialized = ctx_kind == CTX_XDP ? im->fx.specialized : im->fr.specialized;
  return 0;
}

int bpftime_amd_vm_counter_info(const struct ebpf_vm *vm, uint32_t ctx_kind, uint32_t *deferred, uint32_t *direct) {
  if (!vm || !vm->impl->loaded) return -1;
  auto im = vm->impl->image();
  const FastForm &f = ctx_kind == CTX_XDP ? im->fx : im->fr;
  uint32_t nd = 0, nn = 0;
  for (size_t i = 0; i < f.add_site.size(); i++)
    if (f.add_site[i]) ((f.fast[i].w1 & FW_NODEFER) ? nn : nd)++;
  if (deferred) *deferred = nd;
  if (direct) *direct = nn;
  return 0;
}

void bpftime_amd_set_step_limit(struct ebpf_vm *vm, uint64_t limit) { vm->impl->step_limit = limit; }

float bpftime_amd_last_batch_ms(struct ebpf_vm *vm) {
  Mi355xVm *v = vm ? vm->impl : nullptr;
  float ms = -1.f;
  if (!v || !v->ev_t0 || !v->ev_t1 || hipEventSynchronize(v->ev_t1) != hipSuccess ||
      hipEventElapsedTime(&ms, v->ev_t0, v->ev_t1) != hipSuccess)
    return -1.f;
  return ms;
}

const char *bpftime_amd_vm_error(const struct ebpf_vm *vm) { return vm->impl->error.c_str(); }

// ---- experiment counters (BPFTIME_AMD_DBG 512) ----------------------------
int bpftime_amd_dbg_counters(uint64_t *out, int n, int reset) {
  uint64_t *d = bpftime_amd::dbg_counts();
  if (!d || !out || n < 0) return -1;
  if (n > kDbgCounts) n = kDbgCounts;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(out, d, 8 * n, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (reset && hipMemset(d, 0, 8 * kDbgCounts) != hipSuccess) return -1;
  return n;
}

// ---- device utilities ------------------------------------------------------
int bpftime_amd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
int bpftime_amd_set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : -1; }
int bpftime_amd_hip_runtime_version(void) {
  int v = 0;
  return hipRuntimeGetVersion(&v) == hipSuccess ? v : -1;
}
void *bpftime_amd_dev_alloc(uint64_t bytes) {
  void *p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  return p;
}
void bpftime_amd_dev_free(void *p) {
  if (p) hipFree(p);
}
int bpftime_amd_memcpy_htod(void *dst, const void *src, uint64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
int bpftime_amd_memcpy_dtoh(void *dst, const void *src, uint64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int bpftime_amd_memcpy_htod_async(void *dst, const void *src, uint64_t bytes, void *stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream) == hipSuccess ? 0 : -1;
}
int bpftime_amd_memcpy_dtoh_async(void *dst, const void *src, uint64_t bytes, void *stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream) == hipSuccess ? 0 : -1;
}
void *bpftime_amd_stream_create(void) {
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  return (void *)s;
}
void bpftime_amd_stream_destroy(void *stream) {
  if (stream) hipStreamDestroy((hipStream_t)stream);
}
int bpftime_amd_stream_sync(void *stream) {
  return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? 0 : -1;
}
int bpftime_amd_memset(void *dst, int v, uint64_t bytes) { return hipMemset(dst, v, bytes) == hipSuccess ? 0 : -1; }
int bpftime_amd_sync(void) { return hipDeviceSynchronize() == hipSuccess ? 0 : -1; }
void *bpftime_amd_host_alloc(uint64_t bytes) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}
void bpftime_amd_host_free(void *p) {
  if (p) hipHostFree(p);
}
void *bpftime_amd_event_create(void) {
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return (void *)e;
}
void bpftime_amd_event_destroy(void *ev) {
  if (ev) hipEventDestroy((hipEvent_t)ev);
}
int bpftime_amd_event_record(void *ev, void *stream) {
  return hipEventRecord((hipEvent_t)ev, (hipStream_t)stream) == hipSuccess ? 0 : -1;
}
int bpftime_amd_stream_wait_event(void *stream, void *ev) {
  return hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0) == hipSuccess ? 0 : -1;
}
float bpftime_amd_event_elapsed_ms(void *start, void *stop) {
  float ms = -1;
  if (hipEventSynchronize((hipEvent_t)stop) != hipSuccess) return -1;
  if (hipEventElapsedTime(&ms, (hipEvent_t)start, (hipEvent_t)stop) != hipSuccess) return -1;
  return ms;
}

}  // extern "C"
