// bpftime_amd: the bpf(2) command handler an interposed loader talks to.
//
// Restates syscall_context::handle_sysbpf's userspace branch
// (runtime/syscall-server/syscall_context.cpp:429-668, run_with_kernel off)
// over this runtime's records: an unmodified libbpf loader whose bpf()
// calls an LD_PRELOAD shim forwards here creates its maps in HBM, its
// programs and its BPF_XDP links at fds this runtime allocates, and reads
// maps back with the syscall-side semantics (from_syscall = true), and links
// programs to syscall tracepoint perf events (BPF_PROG_ATTACH).
#include <errno.h>
#include <linux/bpf.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/bpftime_amd.h"

extern "C" long bpftime_amd_handle_sysbpf(int cmd, void *attr_, uint32_t size) {
  union bpf_attr *attr = (union bpf_attr *)attr_;
  if (!attr) {
    errno = EFAULT;
    return -1;
  }
  (void)size;
  switch (cmd) {
    case BPF_MAP_CREATE: {  // :429-489
      struct bpf_map_attr a;
      memset(&a, 0, sizeof(a));
      a.type = (int)attr->map_type;
      a.key_size = attr->key_size;
      a.value_size = attr->value_size;
      a.max_ents = attr->max_entries;
      a.flags = attr->map_flags;
      a.ifindex = attr->map_ifindex;
      a.btf_vmlinux_value_type_id = attr->btf_vmlinux_value_type_id;
      a.btf_id = attr->btf_fd;
      a.btf_key_type_id = attr->btf_key_type_id;
      a.btf_value_type_id = attr->btf_value_type_id;
      char name[BPF_OBJ_NAME_LEN + 1];
      memcpy(name, attr->map_name, BPF_OBJ_NAME_LEN);
      name[BPF_OBJ_NAME_LEN] = 0;
      return bpftime_maps_create(-1, name, a);
    }
    case BPF_MAP_LOOKUP_ELEM: {  // :490-514: the value is copied out
      const void *v = bpftime_map_lookup_elem((int)attr->map_fd, (const void *)(uintptr_t)attr->key);
      if (!v) {
        errno = ENOENT;
        return -1;
      }
      memcpy((void *)(uintptr_t)attr->value, v, bpftime_map_value_size_from_syscall((int)attr->map_fd));
      return 0;
    }
    case BPF_MAP_UPDATE_ELEM:  // :515-528
      return bpftime_map_update_elem((int)attr->map_fd, (const void *)(uintptr_t)attr->key,
                                     (const void *)(uintptr_t)attr->value, (uint64_t)attr->flags);
    case BPF_MAP_DELETE_ELEM:  // :529-539
      return bpftime_map_delete_elem((int)attr->map_fd, (const void *)(uintptr_t)attr->key);
    case BPF_MAP_GET_NEXT_KEY:  // :552-563
      return bpftime_map_get_next_key((int)attr->map_fd, (const void *)(uintptr_t)attr->key,
                                      (void *)(uintptr_t)attr->next_key);
    case BPF_PROG_LOAD: {  // :564-639 (no userspace verifier in this build)
      char name[BPF_OBJ_NAME_LEN + 1];
      memcpy(name, attr->prog_name, BPF_OBJ_NAME_LEN);
      name[BPF_OBJ_NAME_LEN] = 0;
      return bpftime_progs_create(-1, (const void *)(uintptr_t)attr->insns, (size_t)attr->insn_cnt, name,
                                  (int)attr->prog_type);
    }
    case BPF_LINK_CREATE: {  // :640-668
      struct bpf_link_create_args a;
      memset(&a, 0, sizeof(a));
      a.prog_fd = attr->link_create.prog_fd;
      a.target_fd = attr->link_create.target_fd;
      a.attach_type = attr->link_create.attach_type;
      a.flags = attr->link_create.flags;
      return bpftime_link_create(-1, &a);
    }
    case BPF_MAP_FREEZE:  // :669-678: accepted, not implemented
      return 0;
    case BPF_MAP_LOOKUP_AND_DELETE_ELEM:  // :540-551 -> bpf_map_handler::map_pop_elem
      // (map_handler.cpp:1411-1434): queue / stack maps only, -ENOTSUP for
      // every other map type; -1 for an fd without a map handler
      if (!bpftime_is_map_fd((int)attr->map_fd)) return -1;
      return -ENOTSUP;
    case BPF_OBJ_GET_INFO_BY_FD: {  // :679-722
      const int fd = (int)attr->info.bpf_fd;
      if (bpftime_is_map_fd(fd)) {
        struct bpf_map_attr a;
        const char *name = nullptr;
        int type = 0;
        if (bpftime_map_get_info(fd, &a, &name, &type) < 0) return -1;
        struct bpf_map_info *p = (struct bpf_map_info *)(uintptr_t)attr->info.info;
        p->btf_id = a.btf_id;
        p->btf_key_type_id = a.btf_key_type_id;
        p->btf_value_type_id = a.btf_value_type_id;
        p->type = (uint32_t)type;
        p->value_size = a.value_size;
        p->btf_vmlinux_value_type_id = a.btf_vmlinux_value_type_id;
        p->key_size = a.key_size;
        p->id = (uint32_t)fd;
        p->ifindex = a.ifindex;
        // map_extra follows btf_value_type_id and a pad word in the kernel
        // ABI (newer than this image's linux/bpf.h): written when the
        // caller's buffer has room for it
        const size_t xoff = (offsetof(struct bpf_map_info, btf_value_type_id) + 4 + 7) & ~(size_t)7;
        if (attr->info.info_len >= xoff + 8) memcpy((uint8_t *)p + xoff, &a.map_extra, 8);
        p->max_entries = a.max_ents;
        p->map_flags = (uint32_t)a.flags;
        strncpy(p->name, name ? name : "", sizeof(p->name) - 1);
      } else if (bpftime_is_prog_fd(fd)) {
        struct bpf_prog_info *p = (struct bpf_prog_info *)(uintptr_t)attr->info.info;
        p->id = (uint32_t)fd;
      }
      return 0;
    }
    case BPF_PROG_ATTACH:  // :723-735 -> bpftime_attach_perf_to_bpf(target perf fd, prog fd)
      return bpftime_attach_perf_to_bpf((int)attr->target_fd, (int)attr->attach_bpf_fd);
  }
  errno = ENOTSUP;  // commands the data path does not serve
  return -1;
}
