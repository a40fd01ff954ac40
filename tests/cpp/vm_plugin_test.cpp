// Drives the bpftime VM plugin (bpftime_amd/plugin/compat_mi355x.hpp) the way
// bpftime_prog drives a bpftime_vm_impl (runtime/src/bpftime_prog.cpp:106-127,
// 231-260), with libbpftime_amd reached only through dlopen.  The runtime
// side is a stand-in for bpftime's shm map registry (array maps; map fds are
// their own "pointers", map_val is the first value's host address, as in
// bpftime_shm.cpp:639-676).
//
//   vm_plugin_test --symbols                     bind every symbol, create a VM (no GPU work)
//   vm_plugin_test --run PROG PKTS N CTL BSS OUT run N 64-B XDP frames one exec each
//
// --run: PROG = the program's raw records, PKTS = N*64 frame bytes, CTL / BSS
// = the map fds the program names; the .bss counter starts at 1000 in the
// runtime's record (mirroring carries it over).  Writes OUT.verdicts (u32),
// OUT.frames (the frames after the program) and prints the runtime-side
// counter after sync_maps_to_host().
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#include "../../bpftime_amd/plugin/compat_mi355x.hpp"

// the method set of bpftime_vm_impl (vm/compat/include/bpftime_vm_compat.hpp:27-198)
class vm_impl {
 public:
  virtual ~vm_impl() {}
  virtual std::string get_error_message() { return ""; }
  virtual bool toggle_bounds_check(bool) { return false; }
  virtual void register_error_print_callback(int (*)(FILE *, const char *, ...)) {}
  virtual int register_external_function(size_t, const std::string &, void *) { return -1; }
  virtual int load_code(const void *code, size_t code_len) = 0;
  virtual void unload_code() {}
  virtual int exec(void *mem, size_t mem_len, uint64_t &ret) = 0;
  virtual void set_lddw_helpers(uint64_t (*)(uint32_t), uint64_t (*)(uint32_t), uint64_t (*)(uint64_t),
                                uint64_t (*)(uint32_t), uint64_t (*)(uint32_t)) {}
};

// ---- the runtime stand-in: array maps by fd ----
struct host_map {
  bpf_map_attr attr;
  std::string name;
  std::vector<uint8_t> data;
};
static std::map<int, host_map> g_maps;

extern "C" uint64_t host_map_ptr_by_fd(uint32_t fd) { return g_maps.count((int)fd) ? fd : ~0ull; }
extern "C" uint64_t host_map_val(uint64_t p) {
  auto it = g_maps.find((int)p);
  return it == g_maps.end() ? 0 : (uint64_t)(uintptr_t)it->second.data.data();
}
static int h_info(int fd, bpf_map_attr *a, const char **name, int *type) {
  auto it = g_maps.find(fd);
  if (it == g_maps.end()) return -1;
  *a = it->second.attr;
  *name = it->second.name.c_str();
  *type = it->second.attr.type;
  return 0;
}
static int h_next(int fd, const void *key, void *next) {  // array_map.cpp:66-81
  auto it = g_maps.find(fd);
  if (it == g_maps.end()) return -1;
  uint32_t k = key ? *(const uint32_t *)key : 0;
  if (!key || k >= it->second.attr.max_ents) k = 0;
  else if (k + 1 == it->second.attr.max_ents) return -1;
  else k++;
  memcpy(next, &k, 4);
  return 0;
}
static const void *h_lookup(int fd, const void *key) {
  auto it = g_maps.find(fd);
  const uint32_t k = *(const uint32_t *)key;
  if (it == g_maps.end() || k >= it->second.attr.max_ents) return nullptr;
  return it->second.data.data() + (size_t)k * it->second.attr.value_size;
}
static long h_update(int fd, const void *key, const void *value, uint64_t) {
  auto it = g_maps.find(fd);
  const uint32_t k = *(const uint32_t *)key;
  if (it == g_maps.end() || k >= it->second.attr.max_ents) return -1;
  memcpy(it->second.data.data() + (size_t)k * it->second.attr.value_size, value, it->second.attr.value_size);
  return 0;
}
static void add_array(int fd, const char *name, uint32_t vs, uint32_t max) {
  host_map m;
  memset(&m.attr, 0, sizeof(m.attr));
  m.attr.type = 2;  // BPF_MAP_TYPE_ARRAY
  m.attr.key_size = 4;
  m.attr.value_size = vs;
  m.attr.max_ents = max;
  m.name = name;
  m.data.assign((size_t)vs * max, 0);
  g_maps[fd] = m;
}

static std::vector<uint8_t> slurp(const char *path) {
  std::vector<uint8_t> b;
  FILE *f = fopen(path, "rb");
  if (!f) return b;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) b.insert(b.end(), buf, buf + n);
  fclose(f);
  return b;
}

// xdp_md_userspace (runtime/extension/userspace_xdp.h:6-17)
struct xdp_md_userspace {
  uint64_t data, data_end;
  uint32_t data_meta, ingress_ifindex, rx_queue_index, egress_ifindex;
  uint64_t buffer_start, buffer_end;
};

using plugin_vm = bpftime_amd_plugin::mi355x_vm<vm_impl>;
static const bpftime_amd_plugin::host_maps kHost = {h_info, h_next, h_lookup, h_update};

int main(int argc, char **argv) {
  if (argc >= 2 && !strcmp(argv[1], "--symbols")) {
    if (!bpftime_amd_plugin::lib().ok()) {
      fprintf(stderr, "FAIL %s\n", bpftime_amd_plugin::lib().error.c_str());
      return 1;
    }
    vm_impl *vm = new plugin_vm(kHost);
    const std::string e = vm->get_error_message();
    delete vm;
    if (!e.empty()) {
      fprintf(stderr, "FAIL %s\n", e.c_str());
      return 1;
    }
    printf("OK symbols\n");
    return 0;
  }
  if (argc != 8 || strcmp(argv[1], "--run")) {
    fprintf(stderr, "usage: %s --symbols | --run PROG PKTS N CTL BSS OUT\n", argv[0]);
    return 2;
  }
  const std::vector<uint8_t> prog = slurp(argv[2]);
  std::vector<uint8_t> frames = slurp(argv[3]);
  const size_t n = strtoull(argv[4], nullptr, 0);
  const int ctl = atoi(argv[5]), bss = atoi(argv[6]);
  if (prog.empty() || frames.size() != n * 64) {
    fprintf(stderr, "FAIL inputs\n");
    return 1;
  }
  add_array(ctl, "ctl_array", 4, 2);
  add_array(bss, "xdp_cou.bss", 4096, 1);
  const uint64_t start = 1000;
  memcpy(g_maps[bss].data.data(), &start, 8);

  // bpftime_prog's sequence: create, lddw helpers, helpers, load
  plugin_vm vm(kHost);
  vm.set_lddw_helpers(host_map_ptr_by_fd, nullptr, host_map_val, nullptr, nullptr);
  vm.register_external_function(1, "bpf_map_lookup_elem", (void *)h_lookup);
  vm.set_ctx_kind(1 /* XDP */);
  if (vm.load_code(prog.data(), prog.size()) < 0) {
    fprintf(stderr, "FAIL load: %s\n", vm.get_error_message().c_str());
    return 1;
  }
  std::vector<uint32_t> verdicts(n);
  for (size_t i = 0; i < n; i++) {
    xdp_md_userspace x;
    memset(&x, 0, sizeof(x));
    x.data = x.buffer_start = (uint64_t)(uintptr_t)(frames.data() + 64 * i);
    x.data_end = x.buffer_end = x.data + 64;
    x.ingress_ifindex = 5;
    uint64_t ret = 0;
    if (vm.exec(&x, sizeof(x), ret) < 0) {
      fprintf(stderr, "FAIL exec %zu: %s\n", i, vm.get_error_message().c_str());
      return 1;
    }
    verdicts[i] = (uint32_t)ret;
  }
  if (vm.sync_maps_to_host() < 0) {
    fprintf(stderr, "FAIL sync\n");
    return 1;
  }
  const std::string out = argv[7];
  FILE *f = fopen((out + ".verdicts").c_str(), "wb");
  fwrite(verdicts.data(), 4, n, f);
  fclose(f);
  f = fopen((out + ".frames").c_str(), "wb");
  fwrite(frames.data(), 1, frames.size(), f);
  fclose(f);
  uint64_t cnt;
  memcpy(&cnt, g_maps[bss].data.data(), 8);
  printf("{\"mirrored\": %zu, \"counter\": %llu}\n", vm.mirrored().size(), (unsigned long long)cnt);
  return 0;
}
