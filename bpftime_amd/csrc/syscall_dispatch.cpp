// bpftime_amd: syscall-tracepoint dispatch over recorded syscalls (SURVEY.md
// §8a row a14).
//
// The reference attaches programs to the sys_enter or sys_exit tracepoint of
// one syscall or of every syscall (attach/syscall_trace_attach_impl/src/
// syscall_trace_attach_impl.cpp:121-166) and, per call, dispatch_syscall
// (:18-95) skips exit / exit_group, runs the per-syscall enter callbacks of
// that nr, then the global ones, each on its own copy of a zeroed
// trace_event_raw_sys_enter {id, args}; if one of them overrode the return
// (bpf_override_return / bpf_set_retval through the thread's return
// callback) it returns that value without running the syscall; else it runs
// the syscall and the exit callbacks (per-syscall, then global) on
// trace_event_raw_sys_exit {id, ret}, returning ret or an exit override.
// dispatch_syscall runs on the calling thread: a thread's calls one after
// another, threads side by side.
//
// Here the calls are recorded (include/bpftime_amd.h: 64-B enter records,
// 96-B enter + exit records with the caller's pid_tgid, 128-B records with
// the recorded clocks too, in device memory) and one of two plans runs them:
//  * program-major: each attached program runs once over the whole batch on
//    the device (ebpf_exec_batch), in the reference's program order:
//    per-syscall enter programs (filtered to their nr, EBPF_BATCH_SYS_NR),
//    global enter programs, per-syscall exit programs, global exit programs.
//    The override state lives in a per-record u32 beside the records (set by
//    helpers 58 / 187 on the device; an exit batch skips records whose enter
//    phase overrode), the returned value in the caller's out_rets.  For one
//    record that is the reference's order; across records the programs are
//    not interleaved, which is equivalent whenever their map effects commute;
//  * thread-ordered: records grouped by their recorded thread (group.hip),
//    one lane per thread walking its records in record order, each record's
//    callbacks run back to back as dispatch_syscall runs them (interp.hip
//    k_sys_seq; vm_api.cpp seq_dispatch) -- the reference's schedule.
// The dispatch takes thread-ordered when two attachments may not commute
// (the loader's map effects, loader.hpp FastForm::map_fx): one writes a map
// the other reads or writes, or adds to a map the other reads.  syscount's
// latency pair is the case (example/tracing/syscount/syscount.bpf.c:33-47,
// 71-76: sys_enter stores start[tid], sys_exit reads it).
// Host-side bookkeeping only; the work is on the device.
#include <errno.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "../../include/ebpf-vm.h"
#include "runtime.hpp"

extern "C" hipError_t bpftime_amd_launch_sys_init(const void *exits, uint64_t n, uint64_t xstride,
                                                  int64_t *out, uint32_t *state, hipStream_t stream);
extern "C" size_t bpftime_amd_group_scratch_bytes(uint64_t n);
extern "C" hipError_t bpftime_amd_group_threads(const void *pid, uint64_t stride, uint64_t n, void *scratch,
                                                uint32_t **perm, uint32_t **seg, uint64_t *nseg,
                                                hipStream_t stream);

using bpftime_amd::SysLayout;

namespace {

// syscall_trace_attach_impl.hpp:97-98: callback sets for nr in [0, 512)
constexpr int64_t kSysNrs = 512;

struct Attach {
  int id;
  int prog_fd;
  int64_t sys_nr;  // -1: every syscall
  bool enter;      // sys_enter (true) or sys_exit tracepoint
  int flags;       // bpftime_amd::vm_prog_flags
  // (shared: a dispatch in flight keeps the VMs it copied alive through a
  // detach or reset on another thread)
  std::shared_ptr<struct ebpf_vm> vm;
};

std::mutex g_mu;
std::vector<Attach> g_attach;
int g_next_id = 1;

// Per-stream device scratch of a dispatch (the records' override state, a
// copy of the records for programs that may store into their ctx, the thread
// grouping), and a per-stream lock that a dispatch holds from taking the
// scratch until it has queued its last launch: two dispatches on one stream
// never share the scratch, and a larger allocation frees the old buffer only
// after the dispatches that used it have queued everything (the stream sync
// then waits for them)
std::mutex g_buf_mu;
struct Buf {
  void *p = nullptr;
  uint64_t bytes = 0;
  std::shared_ptr<std::mutex> mu = std::make_shared<std::mutex>();
};
std::map<hipStream_t, Buf> g_bufs;

std::shared_ptr<std::mutex> stream_lock(hipStream_t s) {
  std::lock_guard<std::mutex> g(g_buf_mu);
  return g_bufs[s].mu;
}

// (called with the stream's lock held)
uint8_t *scratch(hipStream_t s, uint64_t bytes) {
  std::lock_guard<std::mutex> g(g_buf_mu);
  Buf &b = g_bufs[s];
  if (b.bytes < bytes) {
    if (b.p && (hipStreamSynchronize(s) != hipSuccess || hipFree(b.p) != hipSuccess)) return nullptr;
    b.p = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) return nullptr;
    b.bytes = bytes;
  }
  return (uint8_t *)b.p;
}

int fail(const std::string &what, int err) {
  bpftime_amd::set_error("syscall dispatch: " + what);
  errno = err;
  return -1;
}

// dispatch_syscall's order: enter per-syscall, enter global, exit
// per-syscall, exit global (attach order inside each group; the reference
// keeps each group in a std::set of entry pointers, syscall_trace_attach_impl.hpp:
// 93-96, whose order follows the entries' addresses)
std::vector<Attach> ordered_attachments() {
  std::vector<Attach> order;
  {
    std::lock_guard<std::mutex> g(g_mu);
    order = g_attach;
  }
  auto rank = [](const Attach &a) { return (a.enter ? 0 : 2) + (a.sys_nr >= 0 ? 0 : 1); };
  std::stable_sort(order.begin(), order.end(), [&](const Attach &a, const Attach &b) { return rank(a) < rank(b); });
  return order;
}

// Whether the attachments may not commute: two of them reach one map, and one
// writes it (a store, a fetching / non-add atomic, update / delete / ring
// calls) or adds to it while the other reads it.  Counter adds commute with
// counter adds; reads with reads.  Programs whose accesses the loader cannot
// place reach every map.  -1 when a program is not loaded.
int conflicts(const std::vector<Attach> &order) {
  using bpftime_amd::FX_ADD;
  using bpftime_amd::FX_READ;
  using bpftime_amd::FX_WRITE;
  struct Fx {
    std::map<int32_t, uint8_t> m;
    uint8_t any;
  };
  std::vector<Fx> fx(order.size());
  for (size_t i = 0; i < order.size(); i++)
    if (bpftime_amd::vm_map_effects(order[i].vm.get(), fx[i].m, fx[i].any) < 0) return -1;
  auto clash = [](uint8_t a, uint8_t b) {
    return ((a & FX_WRITE) && b) || ((b & FX_WRITE) && a) || ((a & FX_ADD) && (b & FX_READ)) ||
           ((b & FX_ADD) && (a & FX_READ));
  };
  for (size_t i = 0; i < fx.size(); i++)
    for (size_t j = i + 1; j < fx.size(); j++) {
      if (clash(fx[i].any, fx[j].any)) return 1;
      for (const auto &kv : fx[i].m) {
        auto it = fx[j].m.find(kv.first);
        if (clash(kv.second | fx[i].any, (it == fx[j].m.end() ? 0 : it->second) | fx[j].any)) return 1;
      }
      for (const auto &kv : fx[j].m)
        if (clash(kv.second | fx[j].any, fx[i].any)) return 1;
    }
  return 0;
}

// 1 thread-ordered, 0 program-major, -1 error
int plan_for(const std::vector<Attach> &order, uint32_t flags) {
  if (flags & EBPF_BATCH_ORDERED) return 1;  // one lane, record order: the serial run
  if (flags & BPFTIME_AMD_DISPATCH_PROGRAMS) return 0;
  if (flags & BPFTIME_AMD_DISPATCH_THREADS) return 1;
  const int c = conflicts(order);
  if (c < 0) return fail("an attached program is not loaded", EINVAL);
  return c;
}

// The records of a dispatch: their field layout (common.hpp SysLayout) and,
// per phase, the block a program's ctx lies in -- what a program that may
// store into its ctx gets a copy of (AoS: the whole records; SoA: the
// phase's array) and the ctx's offset in it
struct Records {
  SysLayout lay;
  uint64_t n;
  const uint8_t *block[2];  // [0] enter, [1] exit
  uint64_t block_bytes[2];
  uint32_t ctx_off[2];
};

int64_t dispatch_threads(const std::vector<Attach> &order, const Records &r, int64_t *out_rets, uint32_t flags,
                         hipStream_t s) {
  std::vector<bpftime_amd::SeqAttach> progs;
  for (const Attach &a : order) progs.push_back({a.vm.get(), a.sys_nr, a.enter});
  // one thread: an ORDERED dispatch (the serial reference run) or records
  // without a recorded caller (every call is the dispatching thread's)
  const bool one = (flags & EBPF_BATCH_ORDERED) || !r.lay.pid;
  const uint64_t gbytes = one ? 0 : bpftime_amd_group_scratch_bytes(r.n);
  if (!one && !gbytes) return fail("thread grouping of " + std::to_string(r.n) + " records", EINVAL);
  uint8_t *buf = scratch(s, 256 + gbytes);
  if (!buf) return fail("scratch allocation failed", ENOMEM);
  uint32_t *perm = nullptr, *seg = nullptr;
  uint64_t nseg = 1;
  if (!one) {
    const hipError_t e = bpftime_amd_group_threads(r.lay.pid, r.lay.pstride, r.n, buf + 256, &perm, &seg, &nseg, s);
    if (e != hipSuccess) return fail(std::string("thread grouping: ") + hipGetErrorString(e), EIO);
  }
  return bpftime_amd::seq_dispatch(progs, r.lay, r.n, perm, seg, nseg, out_rets, flags, (uint32_t *)buf, s);
}

int64_t dispatch_programs(const std::vector<Attach> &order, const Records &r, int64_t *out_rets, uint32_t flags,
                          hipStream_t s) {
  const uint64_t n = r.n;
  bool enter_ovr = false, any_ovr = false, copies = false;
  for (const Attach &a : order) {
    enter_ovr |= a.enter && (a.flags & bpftime_amd::kProgSetsRetval);
    any_ovr |= (a.flags & bpftime_amd::kProgSetsRetval) != 0;
    copies |= (a.flags & bpftime_amd::kProgStoresCtx) != 0;
  }
  // scratch: per-record override state, then (programs that may store into
  // their ctx) a copy of the records
  const bool state = out_rets || any_ovr;
  const uint64_t sbytes = state ? (4 * n + 255) & ~255ull : 0;
  const uint64_t cbytes = copies ? std::max(r.block_bytes[0], r.block_bytes[1]) : 0;
  uint8_t *buf = nullptr;
  if (state || copies) {
    buf = scratch(s, sbytes + cbytes);
    if (!buf) return fail("scratch allocation failed", ENOMEM);
  }
  uint32_t *st = state ? (uint32_t *)buf : nullptr;
  uint8_t *copy = copies ? buf + sbytes : nullptr;
  if (state) {
    // out_rets[i] = the recorded ret (or 0 without exit ctxs); state[i] = 0
    const hipError_t e = bpftime_amd_launch_sys_init(r.lay.exit, n, r.lay.xstride, out_rets, st, s);
    if (e != hipSuccess) return fail(std::string("state init: ") + hipGetErrorString(e), EIO);
  }
  // a field inside the unit's own record (AoS) is an offset from the unit
  // (the asm tier reads bpf_get_current_pid_tgid's there); else an array
  auto field = [](const uint8_t *f, uint64_t fs, const uint8_t *unit, uint64_t us, int32_t &off, const void *&arr,
                  uint64_t &stride) {
    if (!f) return;
    if (fs == us && f >= unit && f + 8 <= unit + us) {
      off = (int32_t)(f - unit);
    } else {
      arr = f;
      stride = fs;
    }
  };
  int64_t failed = 0;
  for (const Attach &a : order) {
    const int ph = a.enter ? 0 : 1;
    const uint8_t *unit = r.block[ph] + r.ctx_off[ph];
    const uint64_t ustride = a.enter ? r.lay.estride : r.lay.xstride;
    struct ebpf_batch b = {};
    // pid / clock addressed against the records the program reads
    field(r.lay.pid, r.lay.pstride, unit, ustride, b.pid_tgid_off, b.pid_tgid_arr, b.pid_tgid_stride);
    field(r.lay.clock ? r.lay.clock + (a.enter ? 0 : 8) : nullptr, r.lay.cstride, unit, ustride, b.ktime_off,
          b.ktime_arr, b.ktime_stride);
    if (a.flags & bpftime_amd::kProgStoresCtx) {
      // each reference callback runs on its own ctx copy (:43-45)
      const hipError_t e = hipMemcpyAsync(copy, r.block[ph], r.block_bytes[ph], hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return fail(std::string("record copy: ") + hipGetErrorString(e), EIO);
      unit = copy + r.ctx_off[ph];
    }
    b.ctx_kind = a.enter ? EBPF_CTX_SYSCALL : EBPF_CTX_SYSCALL_EXIT;
    b.flags = (flags & (EBPF_BATCH_SYNC | EBPF_BATCH_UNCHECKED)) | (a.sys_nr >= 0 ? EBPF_BATCH_SYS_NR : 0u);
    b.count = n;
    b.data = const_cast<uint8_t *>(unit);
    b.stride = ustride;
    b.sys_nr = a.sys_nr;
    b.stream = s;
    // the state where this program sets it, or (exit programs) where an
    // enter program may have overridden the record's return
    const bool sets = (a.flags & bpftime_amd::kProgSetsRetval) != 0;
    if (state && (sets || (!a.enter && enter_ovr))) {
      b.sys_state = st;
      b.sys_ret = sets ? out_rets : nullptr;
      b.sys_phase = a.enter ? 1 : 2;
    }
    const int rc = ebpf_exec_batch(a.vm.get(), &b);
    if (rc < 0) return -1;
    failed += rc;
  }
  return failed;
}

int64_t dispatch(const Records &r, int64_t *out_rets, uint32_t flags, void *stream) {
  const std::vector<Attach> order = ordered_attachments();
  bool enters = false, exits = false;
  for (const Attach &a : order) {
    exits |= !a.enter;
    enters |= a.enter;
  }
  if (exits && !r.lay.exit)
    return fail("sys_exit programs are attached: the records need the 96-B form (enter + exit ctx)", EINVAL);
  if (enters && !r.lay.enter) return fail("sys_enter programs are attached: the records need enter ctxs", EINVAL);
  const int plan = plan_for(order, flags);
  if (plan < 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (r.n == 0) return 0;
  if (order.empty()) {
    if (out_rets) {  // nothing attached: every call returns its recorded ret
      const hipError_t e = bpftime_amd_launch_sys_init(r.lay.exit, r.n, r.lay.xstride, out_rets, nullptr, s);
      if (e != hipSuccess) return fail(std::string("state init: ") + hipGetErrorString(e), EIO);
    }
    return 0;
  }
  const std::shared_ptr<std::mutex> mu = stream_lock(s);
  std::lock_guard<std::mutex> hold(*mu);
  return plan ? dispatch_threads(order, r, out_rets, flags, s) : dispatch_programs(order, r, out_rets, flags, s);
}

}  // namespace

void bpftime_amd::syscall_detach_all() {
  std::lock_guard<std::mutex> g(g_mu);
  g_attach.clear();  // (each VM goes with the last dispatch that holds it)
}

extern "C" {

int bpftime_amd_syscall_attach_ex(int prog_fd, int64_t sys_nr, int is_enter) {
  // :134-139: "Invalid sys nr"
  if (!bpftime_is_prog_fd(prog_fd) || sys_nr < -1 || sys_nr >= kSysNrs) {
    errno = EINVAL;
    return -1;
  }
  char *err = nullptr;
  struct ebpf_vm *vm = bpftime_amd_prog_instantiate(prog_fd, &err);
  if (!vm) {
    bpftime_amd::set_error(std::string("syscall attach: ") + (err ? err : "load failed"));
    free(err);
    errno = EINVAL;
    return -1;
  }
  std::shared_ptr<struct ebpf_vm> owned(vm, ebpf_destroy);
  ebpf_set_ctx_kind(vm, is_enter ? EBPF_CTX_SYSCALL : EBPF_CTX_SYSCALL_EXIT);
  const int flags = bpftime_amd::vm_prog_flags(vm);
  if (flags < 0) {  // (never attach a program whose flags are unknown)
    bpftime_amd::set_error("syscall attach: the program is not loaded");
    errno = EINVAL;
    return -1;
  }
  std::lock_guard<std::mutex> g(g_mu);
  g_attach.push_back(Attach{g_next_id, prog_fd, sys_nr, is_enter != 0, flags, std::move(owned)});
  return g_next_id++;
}

int bpftime_amd_syscall_attach(int prog_fd, int64_t sys_nr) { return bpftime_amd_syscall_attach_ex(prog_fd, sys_nr, 1); }

int bpftime_amd_syscall_detach(int id) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto it = g_attach.begin(); it != g_attach.end(); ++it)
    if (it->id == id) {
      g_attach.erase(it);
      return 0;
    }
  errno = ENOENT;  // detach_by_id :115-118
  return -1;
}

int bpftime_amd_syscall_dispatch_plan(uint32_t flags) { return plan_for(ordered_attachments(), flags); }

int64_t bpftime_amd_syscall_dispatch_records(const void *records, uint64_t n, uint32_t record_size,
                                             int64_t *out_rets, uint32_t flags, void *stream) {
  if (record_size != BPFTIME_AMD_SYSCALL_RECORD && record_size != BPFTIME_AMD_SYSCALL_RECORD_FULL &&
      record_size != BPFTIME_AMD_SYSCALL_RECORD_TIMED)
    return fail("record size " + std::to_string(record_size) + " (64, 96 or 128)", EINVAL);
  if (n && !records) return fail("no records", EINVAL);
  if (n > 0xffffffffull) return fail("more than 2^32 records", EINVAL);
  const uint8_t *b = (const uint8_t *)records;
  const bool full = record_size >= BPFTIME_AMD_SYSCALL_RECORD_FULL;
  Records r{};
  r.n = n;
  r.lay.enter = b;
  r.lay.estride = r.lay.xstride = r.lay.pstride = r.lay.cstride = record_size;
  r.lay.exit = full ? b + 64 : nullptr;
  r.lay.pid = full ? b + 88 : nullptr;
  r.lay.clock = record_size == BPFTIME_AMD_SYSCALL_RECORD_TIMED ? b + 96 : nullptr;
  r.block[0] = r.block[1] = b;
  r.block_bytes[0] = r.block_bytes[1] = n * record_size;
  r.ctx_off[0] = 0;
  r.ctx_off[1] = 64;
  return dispatch(r, out_rets, flags, stream);
}

int64_t bpftime_amd_syscall_dispatch_soa(const struct bpftime_amd_sys_records *recs, int64_t *out_rets,
                                         uint32_t flags, void *stream) {
  if (!recs) return fail("no records", EINVAL);
  const uint64_t n = recs->count;
  if (n && !recs->exit) return fail("struct-of-arrays records need the exit array", EINVAL);
  if (n > 0xffffffffull) return fail("more than 2^32 records", EINVAL);
  for (const void *a : {recs->enter, recs->exit, recs->clock})
    if ((uintptr_t)a % 8) return fail("struct-of-arrays records: arrays must be 8-aligned", EINVAL);
  Records r{};
  r.n = n;
  r.lay.enter = (const uint8_t *)recs->enter;
  r.lay.estride = 64;
  r.lay.exit = (const uint8_t *)recs->exit;
  r.lay.xstride = 32;
  r.lay.pid = r.lay.exit ? r.lay.exit + 24 : nullptr;
  r.lay.pstride = 32;
  r.lay.clock = (const uint8_t *)recs->clock;
  r.lay.cstride = 16;
  r.block[0] = r.lay.enter;
  r.block_bytes[0] = 64 * n;
  r.block[1] = r.lay.exit;
  r.block_bytes[1] = 32 * n;
  return dispatch(r, out_rets, flags, stream);
}

int64_t bpftime_amd_syscall_dispatch(const void *records, uint64_t n, uint32_t flags, void *stream) {
  return bpftime_amd_syscall_dispatch_records(records, n, BPFTIME_AMD_SYSCALL_RECORD, nullptr, flags, stream);
}

}  // extern "C"
