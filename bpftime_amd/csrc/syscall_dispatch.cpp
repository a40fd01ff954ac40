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
//
// Here the calls are recorded (include/bpftime_amd.h, 64-B enter records or
// 96-B enter + exit records in device memory) and each attached program runs
// once over the whole batch on the device, in the reference's program order:
// per-syscall enter programs (filtered to their nr, EBPF_BATCH_SYS_NR), global
// enter programs, per-syscall exit programs, global exit programs.  The
// override state lives in a per-record u32 beside the records (set by helpers
// 58 / 187 on the device; an exit batch skips records whose enter phase
// overrode), the returned value in the caller's out_rets.  For one record
// that is the reference's order; across records the programs are not
// interleaved, which is equivalent whenever their map effects commute.
// Host-side bookkeeping only; the work is ebpf_exec_batch.
#include <errno.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "../../include/ebpf-vm.h"
#include "runtime.hpp"

extern "C" hipError_t bpftime_amd_launch_sys_init(const void *records, uint64_t n, uint32_t record_size,
                                                  int64_t *out, uint32_t *state, hipStream_t stream);

namespace {

// syscall_trace_attach_impl.hpp:97-98: callback sets for nr in [0, 512)
constexpr int64_t kSysNrs = 512;

struct Attach {
  int id;
  int prog_fd;
  int64_t sys_nr;  // -1: every syscall
  bool enter;      // sys_enter (true) or sys_exit tracepoint
  int flags;       // bpftime_amd::vm_prog_flags
  struct ebpf_vm *vm;
};

std::mutex g_mu;
std::vector<Attach> g_attach;
int g_next_id = 1;

// per-stream device scratch of a dispatch (the records' override state, a
// copy of the records for programs that may store into their ctx): a
// dispatch's batches use it in stream order
std::mutex g_buf_mu;
struct Buf {
  void *p = nullptr;
  uint64_t bytes = 0;
};
std::map<hipStream_t, Buf> g_bufs;

uint8_t *scratch(hipStream_t s, uint64_t bytes) {
  std::lock_guard<std::mutex> g(g_buf_mu);
  Buf &b = g_bufs[s];
  if (b.bytes < bytes) {
    // (the stream may still run a dispatch that uses the old buffer)
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

}  // namespace

void bpftime_amd::syscall_detach_all() {
  std::lock_guard<std::mutex> g(g_mu);
  for (Attach &a : g_attach) ebpf_destroy(a.vm);
  g_attach.clear();
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
  ebpf_set_ctx_kind(vm, is_enter ? EBPF_CTX_SYSCALL : EBPF_CTX_SYSCALL_EXIT);
  const int flags = bpftime_amd::vm_prog_flags(vm);
  std::lock_guard<std::mutex> g(g_mu);
  g_attach.push_back(Attach{g_next_id, prog_fd, sys_nr, is_enter != 0, flags < 0 ? 0 : flags, vm});
  return g_next_id++;
}

int bpftime_amd_syscall_attach(int prog_fd, int64_t sys_nr) { return bpftime_amd_syscall_attach_ex(prog_fd, sys_nr, 1); }

int bpftime_amd_syscall_detach(int id) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto it = g_attach.begin(); it != g_attach.end(); ++it)
    if (it->id == id) {
      ebpf_destroy(it->vm);
      g_attach.erase(it);
      return 0;
    }
  errno = ENOENT;  // detach_by_id :115-118
  return -1;
}

int64_t bpftime_amd_syscall_dispatch_records(const void *records, uint64_t n, uint32_t record_size,
                                             int64_t *out_rets, uint32_t flags, void *stream) {
  if (record_size != BPFTIME_AMD_SYSCALL_RECORD && record_size != BPFTIME_AMD_SYSCALL_RECORD_FULL)
    return fail("record size " + std::to_string(record_size) + " (64 or 96)", EINVAL);
  if (n && !records) return fail("no records", EINVAL);
  std::vector<Attach> order;
  {
    std::lock_guard<std::mutex> g(g_mu);
    order = g_attach;
  }
  // dispatch_syscall's order: enter per-syscall, enter global, exit
  // per-syscall, exit global (attach order inside each group)
  auto rank = [](const Attach &a) { return (a.enter ? 0 : 2) + (a.sys_nr >= 0 ? 0 : 1); };
  std::stable_sort(order.begin(), order.end(), [&](const Attach &a, const Attach &b) { return rank(a) < rank(b); });
  bool exits = false, enter_ovr = false, any_ovr = false, copies = false;
  for (const Attach &a : order) {
    exits |= !a.enter;
    enter_ovr |= a.enter && (a.flags & bpftime_amd::kProgSetsRetval);
    any_ovr |= (a.flags & bpftime_amd::kProgSetsRetval) != 0;
    copies |= (a.flags & bpftime_amd::kProgStoresCtx) != 0;
  }
  if (exits && record_size != BPFTIME_AMD_SYSCALL_RECORD_FULL)
    return fail("sys_exit programs are attached: the records need the 96-B form (enter + exit ctx)", EINVAL);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  // scratch: per-record override state, then (programs that may store into
  // their ctx) a copy of the records
  const bool state = out_rets || any_ovr;
  const uint64_t sbytes = state ? (4 * n + 255) & ~255ull : 0, rbytes = n * record_size;
  uint8_t *buf = nullptr;
  if (state || copies) {
    buf = scratch(s, sbytes + (copies ? rbytes : 0));
    if (!buf) return fail("scratch allocation failed", ENOMEM);
  }
  uint32_t *st = state ? (uint32_t *)buf : nullptr;
  uint8_t *copy = copies ? buf + sbytes : nullptr;
  if (state) {
    // out_rets[i] = the recorded ret (96-B records) or 0; state[i] = 0
    const hipError_t e = bpftime_amd_launch_sys_init(records, n, record_size, out_rets, st, s);
    if (e != hipSuccess) return fail(std::string("state init: ") + hipGetErrorString(e), EIO);
  }
  int64_t failed = 0;
  for (const Attach &a : order) {
    const uint8_t *base = (const uint8_t *)records;
    if (a.flags & bpftime_amd::kProgStoresCtx) {
      // each reference callback runs on its own ctx copy (:43-45)
      const hipError_t e = hipMemcpyAsync(copy, records, rbytes, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return fail(std::string("record copy: ") + hipGetErrorString(e), EIO);
      base = copy;
    }
    struct ebpf_batch b = {};
    b.ctx_kind = a.enter ? EBPF_CTX_SYSCALL : EBPF_CTX_SYSCALL_EXIT;
    b.flags = (flags & (EBPF_BATCH_SYNC | EBPF_BATCH_ORDERED | EBPF_BATCH_UNCHECKED)) |
              (a.sys_nr >= 0 ? EBPF_BATCH_SYS_NR : 0u);
    b.count = n;
    b.data = const_cast<uint8_t *>(base + (a.enter ? 0 : 64));
    b.stride = record_size;
    b.sys_nr = a.sys_nr;
    b.stream = stream;
    // (96-B records: the recorded caller's pid_tgid at +88)
    if (record_size == BPFTIME_AMD_SYSCALL_RECORD_FULL) b.pid_tgid_off = a.enter ? 88 : 24;
    // the state where this program sets it, or (exit programs) where an
    // enter program may have overridden the record's return
    const bool sets = (a.flags & bpftime_amd::kProgSetsRetval) != 0;
    if (state && (sets || (!a.enter && enter_ovr))) {
      b.sys_state = st;
      b.sys_ret = sets ? out_rets : nullptr;
      b.sys_phase = a.enter ? 1 : 2;
    }
    const int rc = ebpf_exec_batch(a.vm, &b);
    if (rc < 0) return -1;
    failed += rc;
  }
  return failed;
}

int64_t bpftime_amd_syscall_dispatch(const void *records, uint64_t n, uint32_t flags, void *stream) {
  return bpftime_amd_syscall_dispatch_records(records, n, BPFTIME_AMD_SYSCALL_RECORD, nullptr, flags, stream);
}

}  // extern "C"
