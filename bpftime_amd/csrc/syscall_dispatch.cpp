// bpftime_amd: syscall-tracepoint dispatch over recorded sys_enter records
// (SURVEY.md §8a row a14).
//
// The reference attaches programs to the sys_enter tracepoint of one
// syscall or of every syscall (attach/syscall_trace_attach_impl/src/
// syscall_trace_attach_impl.cpp:18-95): for each call it skips exit /
// exit_group, runs the per-syscall callbacks of that nr, then the global
// ones, and ignores r0.  Here a replay batch runs each attached program once
// over the whole batch on the device: per-syscall programs first (each
// filtered to its nr, EBPF_BATCH_SYS_NR), then global ones.  For one record
// that is the reference's order; across records the programs are not
// interleaved, which is equivalent whenever their map updates commute.
// Host-side bookkeeping only; the work is ebpf_exec_batch.
#include <errno.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "../../include/ebpf-vm.h"
#include "runtime.hpp"

namespace {

struct Attach {
  int id;
  int prog_fd;
  int64_t sys_nr;  // -1: every syscall
  struct ebpf_vm *vm;
};

std::mutex g_mu;
std::vector<Attach> g_attach;
int g_next_id = 1;

}  // namespace

extern "C" {

int bpftime_amd_syscall_attach(int prog_fd, int64_t sys_nr) {
  if (!bpftime_is_prog_fd(prog_fd) || sys_nr < -1) {
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
  ebpf_set_ctx_kind(vm, EBPF_CTX_SYSCALL);
  std::lock_guard<std::mutex> g(g_mu);
  g_attach.push_back(Attach{g_next_id, prog_fd, sys_nr, vm});
  return g_next_id++;
}

int bpftime_amd_syscall_detach(int id) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto it = g_attach.begin(); it != g_attach.end(); ++it)
    if (it->id == id) {
      ebpf_destroy(it->vm);
      g_attach.erase(it);
      return 0;
    }
  errno = ENOENT;
  return -1;
}

int64_t bpftime_amd_syscall_dispatch(const void *records, uint64_t n, uint32_t flags, void *stream) {
  std::vector<Attach> order;
  {
    std::lock_guard<std::mutex> g(g_mu);
    order = g_attach;
  }
  // per-syscall programs (in attach order), then the global ones
  std::stable_sort(order.begin(), order.end(),
                   [](const Attach &a, const Attach &b) { return (a.sys_nr >= 0) > (b.sys_nr >= 0); });
  int64_t failed = 0;
  for (const Attach &a : order) {
    struct ebpf_batch b = {};
    b.ctx_kind = EBPF_CTX_SYSCALL;
    b.flags = (flags & (EBPF_BATCH_SYNC | EBPF_BATCH_ORDERED | EBPF_BATCH_UNCHECKED)) |
              (a.sys_nr >= 0 ? EBPF_BATCH_SYS_NR : 0u);
    b.count = n;
    b.data = const_cast<void *>(records);
    b.stride = 64;
    b.sys_nr = a.sys_nr;
    b.stream = stream;
    const int rc = ebpf_exec_batch(a.vm, &b);
    if (rc < 0) return -1;
    failed += rc;
  }
  return failed;
}

}  // extern "C"
