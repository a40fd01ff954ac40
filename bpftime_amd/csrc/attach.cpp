// bpftime_amd: the attach-plugin boundary for device batches.
//
// bpftime runs a program for an attach entry through an ebpf_run_callback,
// int(void *memory, size_t memory_size, uint64_t *return_value)
// (attach/base_attach_impl/base_attach_impl.hpp:24-25), built by
// bpf_attach_ctx around bpftime_prog_exec (runtime/src/attach/
// bpf_attach_ctx.cpp:381-389).  Here an attach entry is a program loaded on
// the device: bpftime_amd_attach_run has the ebpf_run_callback shape (one
// unit, staged through the device), bpftime_amd_attach_run_batch runs it
// over a device-resident batch.  The simple attach impl
// (attach/simple_attach_impl/simple_attach_impl.cpp:7-55) is restated over
// them: one attach per impl instance, the attach type checked, trigger()
// hands the user callback the attach-time argument, the trigger argument and
// the attach entry (1 when nothing is attached).
#include <errno.h>
#include <stdlib.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/bpftime_amd.h"
#include "../../include/ebpf-vm.h"
#include "runtime.hpp"

struct bpftime_amd_attach {
  struct ebpf_vm *vm;
  int prog_fd;
};

namespace {

struct SimpleImpl {
  int attach_type;
  bpftime_amd_simple_callback cb;
  int usable_id = -1;  // simple_attach_impl.hpp:114: one attach at a time
  int next_id = 1;     // base_attach_impl::allocate_id
  std::string argument;
  // held by trigger() for the duration of its callback: a detach or impl
  // destroy running beside it only drops its own reference, and the last
  // holder destroys the attach (the reference's detach_by_id never destroys
  // the callback at all)
  std::shared_ptr<bpftime_amd_attach> attach;
};

std::shared_ptr<bpftime_amd_attach> hold(bpftime_amd_attach *a) {
  return std::shared_ptr<bpftime_amd_attach>(a, bpftime_amd_attach_destroy);
}

std::mutex g_mu;
std::map<int, SimpleImpl> g_impls;
int g_next_impl = 1;

}  // namespace

extern "C" {

struct bpftime_amd_attach *bpftime_amd_attach_create(int prog_fd, int ctx_kind) {
  char *err = nullptr;
  struct ebpf_vm *vm = bpftime_amd_prog_instantiate(prog_fd, &err);
  if (!vm) {
    bpftime_amd::set_error(std::string("attach: ") + (err ? err : "not a loadable prog fd"));
    free(err);
    errno = EINVAL;
    return nullptr;
  }
  if (ctx_kind >= 0) ebpf_set_ctx_kind(vm, (uint32_t)ctx_kind);
  return new bpftime_amd_attach{vm, prog_fd};
}

void bpftime_amd_attach_destroy(struct bpftime_amd_attach *a) {
  if (!a) return;
  ebpf_destroy(a->vm);
  delete a;
}

// the ebpf_run_callback shape: bpftime_prog_exec's contract (0 / -1, *ret
// = r0, 0 when the program failed; bpftime_prog.cpp:231-260)
int bpftime_amd_attach_run(void *attach, void *memory, size_t memory_size, uint64_t *return_value) {
  bpftime_amd_attach *a = (bpftime_amd_attach *)attach;
  if (!a) return -1;
  uint64_t r = 0;
  const int rc = ebpf_exec(a->vm, memory, memory_size, &r);
  if (return_value) *return_value = rc < 0 ? 0 : r;
  return rc < 0 ? -1 : 0;
}

int bpftime_amd_attach_run_batch(struct bpftime_amd_attach *a, const struct ebpf_batch *b) {
  if (!a || !b) return -1;
  return ebpf_exec_batch(a->vm, b);
}

int bpftime_amd_simple_attach_impl_create(int attach_type, bpftime_amd_simple_callback cb) {
  if (!cb) {
    errno = EINVAL;
    return -1;
  }
  std::lock_guard<std::mutex> g(g_mu);
  SimpleImpl s;
  s.attach_type = attach_type;
  s.cb = cb;
  g_impls[g_next_impl] = s;
  return g_next_impl++;
}

// simple_attach_impl::create_attach_with_ebpf_callback
int bpftime_amd_simple_attach(int impl, int prog_fd, int ctx_kind, const char *argument, int attach_type) {
  bpftime_amd_attach *a = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_impls.find(impl);
    if (it == g_impls.end() || it->second.usable_id != -1 || it->second.attach_type != attach_type) {
      errno = EINVAL;  // "only supports one instance" / mismatched attach type
      return -1;
    }
  }
  a = bpftime_amd_attach_create(prog_fd, ctx_kind);
  if (!a) return -1;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_impls.find(impl);
  if (it == g_impls.end() || it->second.usable_id != -1) {
    bpftime_amd_attach_destroy(a);
    errno = EINVAL;
    return -1;
  }
  SimpleImpl &s = it->second;
  s.argument = argument ? argument : "";
  s.attach = hold(a);
  s.usable_id = s.next_id++;
  return s.usable_id;
}

// simple_attach_impl::detach_by_id
int bpftime_amd_simple_detach(int impl, int id) {
  std::shared_ptr<bpftime_amd_attach> a;  // released outside the lock
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_impls.find(impl);
    if (it == g_impls.end() || it->second.usable_id == -1 || it->second.usable_id != id) return -1;
    a = std::move(it->second.attach);
    it->second.usable_id = -1;
  }
  return 0;
}

// simple_attach_impl::trigger: 1 when nothing is attached, else the callback's result
int bpftime_amd_simple_trigger(int impl, void *trigger_argument) {
  bpftime_amd_simple_callback cb;
  std::string arg;
  std::shared_ptr<bpftime_amd_attach> a;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_impls.find(impl);
    if (it == g_impls.end()) return -1;
    if (it->second.usable_id == -1) return 1;
    cb = it->second.cb;
    arg = it->second.argument;
    a = it->second.attach;
  }
  return cb(arg.c_str(), trigger_argument, a.get());
}

int bpftime_amd_simple_attach_impl_destroy(int impl) {
  std::shared_ptr<bpftime_amd_attach> a;  // released outside the lock
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_impls.find(impl);
    if (it == g_impls.end()) return -1;
    a = std::move(it->second.attach);
    g_impls.erase(it);
  }
  return 0;
}

}  // extern "C"
