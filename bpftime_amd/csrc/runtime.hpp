// bpftime_amd: process-wide runtime state (device map registry, prog/link
// records).  Mirrors the role of bpftime's handler_manager in shared memory
// (runtime/src/handler/handler_manager.hpp:84-133) for one GPU per process.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "common.hpp"

namespace bpftime_amd {

struct MapRec {
  std::string name;
  uint32_t type = 0, key_size = 0, value_size = 0, max_entries = 0;
  uint64_t flags = 0;
  DMap d{};
  uint64_t bytes = 0;  // storage bytes at d.data
  uint64_t ix_addr = 0;    // hash lookup index storage (common.hpp ix_pos), 0 = none
  bool ix_valid = false;   // d.ix = ix_addr while the index holds exactly the reachable keys
  std::shared_ptr<struct LpmTrie> lpm;  // LPM_TRIE: the authoritative host trie
};

struct ProgRec {
  std::string name;
  std::vector<uint8_t> insns;  // raw 8-byte ebpf_inst records
  int type = 0;
};

struct LinkRec {
  uint32_t prog_fd = 0, target = 0, attach_type = 0, flags = 0;
};

enum class HKind : uint8_t { NONE, MAP, PROG, LINK };

struct Runtime {
  std::mutex mu;
  std::vector<HKind> kind = std::vector<HKind>(kMaxFds, HKind::NONE);
  std::vector<MapRec> maps = std::vector<MapRec>(kMaxFds);
  std::vector<ProgRec> progs = std::vector<ProgRec>(kMaxFds);
  std::vector<LinkRec> links = std::vector<LinkRec>(kMaxFds);
  int device = -1;
  DMap *d_maptab = nullptr;     // device table indexed by fd
  uint8_t *arena = nullptr;     // device map arena
  uint64_t arena_size = 0, arena_used = 0;
  uint32_t ncpu = 64;
  std::string last_error;
  uint64_t prog_gen = 1;        // bumped when a prog, a prog array or its contents change

  int ensure_device();          // lazily picks the current device, allocates arena + table
  uint64_t arena_alloc(uint64_t bytes);
  int push_map(int fd);         // upload DMap entry for fd
  std::set<int> ix_stale;       // hash maps whose lookup index needs a rebuild
  std::set<int> lpm_stale;      // LPM tries whose device replica needs an upload
  // before a launch: a program that can delete invalidates every hash
  // lookup index; any other rebuilds the stale ones
  int prepare_ix(bool may_delete);
};

// hash lookup index upkeep for host-side writes (maps.cpp)
void ix_invalidate(int fd);

Runtime &rt();
void set_error(const std::string &e);

}  // namespace bpftime_amd
