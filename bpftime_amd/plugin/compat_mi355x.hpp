// bpftime VM plugin for libbpftime_amd: the file a maintainer adds to the
// reference as vm/compat/mi355x-vm/compat_mi355x.cpp, beside compat_ubpf.cpp.
//
// VmBase is bpftime's bpftime_vm_impl (vm/compat/include/bpftime_vm_compat.hpp:27-198).
// bpftime_prog creates a VM by name, hands it the runtime's lddw helpers and
// helper table, loads the program and runs it per unit
// (runtime/src/bpftime_prog.cpp:106-127, 231-260).  This plugin forwards those
// calls to libbpftime_amd and keeps the runtime's maps transparent:
//   * map fds the program loads (lddw src 1 / 2) are mirrored on first use
//     into the device registry, at the same fd, from bpftime's own records
//     (attributes and contents, through host_maps: bpftime_shm.hpp:316-332);
//   * the device registry's map_ptr_by_fd / map_val become the VM's lddw
//     helpers (the device dereferences HBM addresses, not bpftime's shm);
//   * sync_maps_to_host() writes the mirrored maps' device contents back
//     through the same records, for callers that read maps from bpftime.
// The library exports bpftime's own names (ebpf_*, bpftime_map_*), so it is
// opened RTLD_LOCAL and called through the handle; it binds its internal
// calls to itself (-Bsymbolic), so the runtime's definitions never interpose.
#pragma once
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <set>
#include <string>
#include <vector>

#include "../../include/bpftime_amd.h"
#include "../../include/ebpf-vm.h"

namespace bpftime_amd_plugin {

struct api {
  void *h = nullptr;
  std::string error;
#define BPFTIME_AMD_SYM(n) decltype(&::n) n = nullptr
  BPFTIME_AMD_SYM(ebpf_create);
  BPFTIME_AMD_SYM(ebpf_destroy);
  BPFTIME_AMD_SYM(ebpf_register);
  BPFTIME_AMD_SYM(ebpf_load);
  BPFTIME_AMD_SYM(ebpf_unload_code);
  BPFTIME_AMD_SYM(ebpf_exec);
  BPFTIME_AMD_SYM(ebpf_exec_batch);
  BPFTIME_AMD_SYM(ebpf_set_lddw_helpers);
  BPFTIME_AMD_SYM(ebpf_toggle_bounds_check);
  BPFTIME_AMD_SYM(ebpf_set_error_print);
  BPFTIME_AMD_SYM(ebpf_set_ctx_kind);
  BPFTIME_AMD_SYM(bpftime_maps_create);
  BPFTIME_AMD_SYM(bpftime_is_map_fd);
  BPFTIME_AMD_SYM(bpftime_map_lookup_elem);
  BPFTIME_AMD_SYM(bpftime_map_update_elem);
  BPFTIME_AMD_SYM(bpftime_map_get_next_key);
  BPFTIME_AMD_SYM(bpftime_map_value_size_from_syscall);
  BPFTIME_AMD_SYM(bpftime_amd_map_ptr_by_fd);
  BPFTIME_AMD_SYM(bpftime_amd_map_val);
#undef BPFTIME_AMD_SYM
  bool ok() const { return h && error.empty(); }
};

inline api &lib() {
  static api a = [] {
    api x;
    const char *path = getenv("BPFTIME_AMD_LIB");
    x.h = dlopen(path && *path ? path : "libbpftime_amd.so", RTLD_NOW | RTLD_LOCAL);
    if (!x.h) {
      x.error = dlerror();
      return x;
    }
#define BIND(n)                                                 \
  x.n = (decltype(x.n))dlsym(x.h, #n);                          \
  if (!x.n && x.error.empty()) x.error = "missing symbol " #n;
    BIND(ebpf_create) BIND(ebpf_destroy) BIND(ebpf_register) BIND(ebpf_load) BIND(ebpf_unload_code)
    BIND(ebpf_exec) BIND(ebpf_exec_batch) BIND(ebpf_set_lddw_helpers) BIND(ebpf_toggle_bounds_check)
    BIND(ebpf_set_error_print) BIND(ebpf_set_ctx_kind) BIND(bpftime_maps_create) BIND(bpftime_is_map_fd)
    BIND(bpftime_map_lookup_elem) BIND(bpftime_map_update_elem) BIND(bpftime_map_get_next_key)
    BIND(bpftime_map_value_size_from_syscall) BIND(bpftime_amd_map_ptr_by_fd) BIND(bpftime_amd_map_val)
#undef BIND
    return x;
  }();
  return a;
}

// bpftime's map records, as the runtime's shm API exposes them
// (bpftime_shm.hpp:316-332; the maintainer's adapter converts
// bpftime::bpf_map_attr into the identical struct bpf_map_attr here)
struct host_maps {
  int (*get_info)(int fd, struct bpf_map_attr *attr, const char **name, int *type);
  int (*get_next_key)(int fd, const void *key, void *next_key);
  const void *(*lookup)(int fd, const void *key);
  long (*update)(int fd, const void *key, const void *value, uint64_t flags);
};

template <class VmBase>
class mi355x_vm : public VmBase {
 public:
  explicit mi355x_vm(const host_maps &host) : host_(host) {
    if (!lib().ok()) {
      err_ = "libbpftime_amd: " + lib().error;
      return;
    }
    vm_ = lib().ebpf_create("mi355x");
    if (!vm_) err_ = "ebpf_create(mi355x) failed";
  }
  ~mi355x_vm() override {
    if (vm_) lib().ebpf_destroy(vm_);
  }
  std::string get_error_message() override { return err_; }
  bool toggle_bounds_check(bool enable) override { return vm_ && lib().ebpf_toggle_bounds_check(vm_, enable); }
  void register_error_print_callback(int (*fn)(FILE *, const char *, ...)) override {
    if (vm_) lib().ebpf_set_error_print(vm_, fn);
  }
  // the device implementation of helper `index` runs; the host function is
  // not callable from the GPU
  int register_external_function(size_t index, const std::string &name, void *fn) override {
    return vm_ ? lib().ebpf_register(vm_, (unsigned)index, name.c_str(), fn) : -1;
  }
  int load_code(const void *code, size_t code_len) override {
    if (!vm_) return -1;
    if (mirror_maps((const uint8_t *)code, code_len) < 0) return -1;
    char *msg = nullptr;
    const int r = lib().ebpf_load(vm_, code, (uint32_t)code_len, &msg);
    if (msg) {
      err_ = msg;
      free(msg);
    }
    return r;
  }
  void unload_code() override {
    if (vm_) lib().ebpf_unload_code(vm_);
  }
  int exec(void *mem, size_t mem_len, uint64_t &ret) override {
    if (!vm_) return -1;
    return lib().ebpf_exec(vm_, mem, mem_len, &ret);
  }
  void set_lddw_helpers(uint64_t (*map_by_fd)(uint32_t), uint64_t (*map_by_idx)(uint32_t),
                        uint64_t (*map_val)(uint64_t), uint64_t (*var_addr)(uint32_t),
                        uint64_t (*code_addr)(uint32_t)) override {
    (void)map_by_idx;
    (void)map_val;
    (void)var_addr;
    (void)code_addr;
    host_map_by_fd_ = map_by_fd;  // which fds are the runtime's maps
    if (vm_)
      lib().ebpf_set_lddw_helpers(vm_, lib().bpftime_amd_map_ptr_by_fd, nullptr, lib().bpftime_amd_map_val, nullptr,
                                  nullptr);
  }

  // ---- beyond bpftime_vm_impl ----
  // how exec's `mem` is read (ebpf-vm.h: 0 raw, 1 XDP xdp_md_userspace, 2 syscall record)
  int set_ctx_kind(uint32_t kind) { return vm_ ? lib().ebpf_set_ctx_kind(vm_, kind) : -1; }
  int exec_batch(const struct ebpf_batch *b) { return vm_ ? lib().ebpf_exec_batch(vm_, b) : -1; }
  // device contents of the mirrored maps -> the runtime's records
  int sync_maps_to_host() {
    for (int fd : mirrored_) {
      const uint32_t vs = lib().bpftime_map_value_size_from_syscall(fd);
      struct bpf_map_attr a;
      const char *name = nullptr;
      int type = 0;
      if (host_.get_info(fd, &a, &name, &type) < 0 || vs != a.value_size) continue;  // per-CPU layouts differ
      std::vector<uint8_t> key(a.key_size), next(a.key_size);
      const void *kp = nullptr;
      while (lib().bpftime_map_get_next_key(fd, kp, next.data()) == 0) {
        const void *v = lib().bpftime_map_lookup_elem(fd, next.data());
        if (v && host_.update(fd, next.data(), v, 0) < 0) return -1;
        key = next;
        kp = key.data();
      }
    }
    return 0;
  }
  const std::set<int> &mirrored() const { return mirrored_; }

 private:
  int mirror_maps(const uint8_t *code, size_t len) {
    for (size_t i = 0; i + 16 <= len; i += 8) {
      const uint8_t op = code[i], src = code[i + 1] >> 4;
      if (op != 0x18) continue;
      int32_t imm;
      memcpy(&imm, code + i + 4, 4);
      i += 8;  // the second half of the lddw
      if ((src != 1 && src != 2) || imm < 0) continue;
      if (mirror(imm) < 0) return -1;
    }
    return 0;
  }
  int mirror(int fd) {
    if (mirrored_.count(fd) || lib().bpftime_is_map_fd(fd)) return 0;  // known to the device registry
    if (host_map_by_fd_ && host_map_by_fd_((uint32_t)fd) == ~0ull) return 0;  // not a runtime map: load decides
    struct bpf_map_attr a;
    memset(&a, 0, sizeof(a));
    const char *name = nullptr;
    int type = 0;
    if (host_.get_info(fd, &a, &name, &type) < 0) return 0;
    a.type = type;
    if (lib().bpftime_maps_create(fd, name ? name : "", a) != fd) {
      err_ = "mirroring map fd " + std::to_string(fd) + " into the device registry failed";
      return -1;
    }
    std::vector<uint8_t> key(a.key_size), next(a.key_size);
    const void *kp = nullptr;
    while (host_.get_next_key(fd, kp, next.data()) == 0) {
      const void *v = host_.lookup(fd, next.data());
      if (v && lib().bpftime_map_update_elem(fd, next.data(), v, 0) < 0) {
        err_ = "copying map fd " + std::to_string(fd) + " to the device failed";
        return -1;
      }
      key = next;
      kp = key.data();
    }
    mirrored_.insert(fd);
    return 0;
  }

  host_maps host_;
  struct ebpf_vm *vm_ = nullptr;
  std::string err_;
  uint64_t (*host_map_by_fd_)(uint32_t) = nullptr;
  std::set<int> mirrored_;
};

}  // namespace bpftime_amd_plugin
