// bpftime_amd: syscall tracepoint ids -> (syscall number, enter / exit).
//
// A tracepoint perf event carries the kernel's tracepoint id (the `id` file
// of its tracefs directory), not a syscall number.  The reference turns one
// into the other when it attaches (attach/syscall_trace_attach_impl/src/
// syscall_trace_attach_private_data.cpp:8-63): the tracefs directory name
// of the id (syscall_table.cpp:66-98: events/syscalls/*/id, plus
// raw_syscalls/sys_enter and sys_exit as the global enter / exit), then the
// syscall's number from <sys/syscall.h> (syscall_table.cpp:17-44, with
// umount2 named umount).  Same steps here; the tracefs events directory is
// /sys/kernel/tracing/events unless BPFTIME_AMD_TRACEFS_EVENTS or
// bpftime_amd_set_tracefs_events names another (a copy of one, or a test's).
// Host-only code.
#include <dirent.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <map>
#include <mutex>
#include <string>

#include "../../include/bpftime_amd.h"
#include "runtime.hpp"

namespace {

const std::pair<const char *, int> kSyscalls[] = {
#include "syscall_names.inc"
};

const char *kGlobalEnter = "sys_enter", *kGlobalExit = "sys_exit";  // GLOBAL_SYS_{ENTER,EXIT}_NAME

std::mutex g_mu;
std::string g_root;
bool g_loaded = false;
std::map<int32_t, std::string> g_tp;  // tracepoint id -> name (syscall_tracepoint_table)

bool read_id(const std::string &dir, int32_t *id) {
  FILE *f = fopen((dir + "/id").c_str(), "r");
  if (!f) return false;
  const bool ok = fscanf(f, "%d", id) == 1;
  fclose(f);
  return ok;
}

// create_syscall_tracepoint_id_table (syscall_table.cpp:66-98); a missing
// tracefs leaves the table empty (the reference throws there), so every id
// fails to resolve
void load_locked() {
  if (g_loaded) return;
  g_loaded = true;
  g_tp.clear();
  if (g_root.empty()) {
    const char *env = getenv("BPFTIME_AMD_TRACEFS_EVENTS");
    g_root = env && *env ? env : "/sys/kernel/tracing/events";
  }
  const std::string sys = g_root + "/syscalls";
  if (DIR *d = opendir(sys.c_str())) {
    while (dirent *e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      const std::string p = sys + "/" + e->d_name;
      struct stat st;
      int32_t id;
      if (stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode) && read_id(p, &id)) g_tp[id] = e->d_name;
    }
    closedir(d);
  }
  int32_t id;
  if (read_id(g_root + "/raw_syscalls/sys_enter", &id)) g_tp[id] = kGlobalEnter;
  if (read_id(g_root + "/raw_syscalls/sys_exit", &id)) g_tp[id] = kGlobalExit;
}

int64_t nr_of(const std::string &name) {
  for (const auto &kv : kSyscalls)
    if (name == kv.first) return kv.second;
  return -1;
}

}  // namespace

extern "C" {

int bpftime_amd_set_tracefs_events(const char *dir) {
  std::lock_guard<std::mutex> g(g_mu);
  g_root = dir ? dir : "";
  g_loaded = false;
  return 0;
}

int64_t bpftime_amd_syscall_nr(const char *name) { return name ? nr_of(name) : -1; }

// syscall_trace_attach_private_data::initialize_from_string
int bpftime_amd_tracepoint_resolve(int32_t tp_id, int64_t *sys_nr, int *is_enter) {
  std::string name;
  {
    std::lock_guard<std::mutex> g(g_mu);
    load_locked();
    auto it = g_tp.find(tp_id);
    if (it == g_tp.end()) {
      bpftime_amd::set_error("Unable to find tp id " + std::to_string(tp_id) + " in syscall tracepoints");
      return -EEXIST;
    }
    name = it->second;
  }
  int64_t nr = -1;
  int enter = 1;
  if (name == kGlobalEnter || name == kGlobalExit) {
    enter = name == kGlobalEnter;
  } else {
    std::string sc;
    if (name.rfind("sys_enter_", 0) == 0) {
      sc = name.substr(10);
    } else if (name.rfind("sys_exit_", 0) == 0) {
      sc = name.substr(9);
      enter = 0;
    }
    nr = sc.empty() ? -1 : nr_of(sc);
    if (nr < 0) {
      bpftime_amd::set_error("Unable to lookup sys nr for syscall tracepoint " + name + ", syscall name " + sc);
      return -EEXIST;
    }
  }
  if (sys_nr) *sys_nr = nr;
  if (is_enter) *is_enter = enter;
  return 0;
}

// the id of the tracepoint a (sys_nr, enter) pair resolves from, -1 if the
// events directory has none
int32_t bpftime_amd_tracepoint_id(int64_t sys_nr, int is_enter) {
  std::string want;
  if (sys_nr < 0) {
    want = is_enter ? kGlobalEnter : kGlobalExit;
  } else {
    for (const auto &kv : kSyscalls)
      if (kv.second == sys_nr) want = std::string(is_enter ? "sys_enter_" : "sys_exit_") + kv.first;
    if (want.empty()) return -1;
  }
  std::lock_guard<std::mutex> g(g_mu);
  load_locked();
  for (const auto &kv : g_tp)
    if (kv.second == want) return kv.first;
  return -1;
}

}  // extern "C"
