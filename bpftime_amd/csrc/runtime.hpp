// bpftime_amd: process-wide runtime state (device map registry, prog/link
// records).  Mirrors the role of bpftime's handler_manager in shared memory
// (runtime/src/handler/handler_manager.hpp:84-133) for one GPU per process.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "common.hpp"

struct ebpf_vm;  // include/ebpf-vm.h

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
  // LPM_TRIE: an ORDERED batch's device update ran out of the node pool;
  // every host op on the trie and every launch naming a trie reports it
  // (ENOMEM) until bpftime_amd_map_ack_error
  bool lpm_pool_out = false;
  // BPF_MAP_CREATE attributes as given (BPF_OBJ_GET_INFO_BY_FD reports them)
  uint32_t ifindex = 0, btf_vmlinux_value_type_id = 0, btf_id = 0, btf_key_type_id = 0, btf_value_type_id = 0;
  uint64_t map_extra = 0;
  uint32_t kernel_bpf_map_id = 0;
  // host view of an ARRAY map (bpftime_get_array_map_raw_data, the mmap a
  // libbpf loader makes of .bss / .data): page-aligned host bytes kept
  // coherent with the device copy at batch boundaries (maps.cpp host_view_*)
  uint8_t *host_view = nullptr;
  uint64_t host_view_bytes = 0;
  std::vector<uint8_t> host_shadow;  // the bytes last exchanged with the device
};

// A perf event record (bpf_perf_event_handler, runtime/src/handler/
// perf_event_handler.hpp:161-215): what a link's target_fd names.  Only a
// syscall sys_enter / sys_exit tracepoint drives anything here (the syscall
// replay dispatch); the other kinds are kept as records, so state that holds
// them imports, exports and links unchanged.
struct PerfRec {
  int type = 2;                // bpf_event_type (bpftime_shm.hpp:48-64); 2 = PERF_TYPE_TRACEPOINT
  int pid = -1;
  bool enabled = false;        // perf_event_enable / _disable (a flag only, as in the reference)
  int32_t tracepoint_id = -1;  // tracepoint: the kernel id (tracepoints.cpp), or -1 when made from
  int64_t sys_nr = -1;         // ... a syscall number (bpftime_amd_perf_event_syscall; -1: every syscall)
  uint64_t offset = 0, ref_ctr_off = 0;  // uprobe / uretprobe / uprobe override
  std::string module;
  int cpu = 0;                 // software perf event
  int32_t sample_type = 0;
  int64_t config = 0;
};

struct ProgRec {
  std::string name;
  std::vector<uint8_t> insns;  // raw 8-byte ebpf_inst records
  int type = 0;
};

struct LinkRec {
  uint32_t prog_fd = 0, target = 0, attach_type = 0, flags = 0;
  bool perf = false;  // target is a perf event record (maps.cpp link_perf)
  int attach_id = 0;  // a perf link to a sys_enter / sys_exit tracepoint: its syscall attachment (syscall_dispatch.cpp)
};

enum class HKind : uint8_t { NONE, MAP, PROG, LINK, PERF };

struct Runtime {
  std::mutex mu;
  std::vector<HKind> kind = std::vector<HKind>(kMaxFds, HKind::NONE);
  std::vector<MapRec> maps = std::vector<MapRec>(kMaxFds);
  std::vector<ProgRec> progs = std::vector<ProgRec>(kMaxFds);
  std::vector<LinkRec> links = std::vector<LinkRec>(kMaxFds);
  std::vector<PerfRec> perfs = std::vector<PerfRec>(kMaxFds);
  std::set<int> host_views;     // ARRAY maps with a host view
  // before a launch: host writes to host views reach the device; after a
  // synchronous batch (or bpftime_amd_map_msync): device bytes reach them
  int host_views_push();
  int host_views_pull();
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
  std::set<int> lpm_flat_pending;  // IPv4 LPM tries whose flat table is not built (DMap.ix = 0: walk)
  // LPM tries an ORDERED batch of a program that writes them may have
  // changed on the device: the replica is authoritative until the host pulls
  // it back (maps.cpp lpm_pull) before its next operation on the trie
  std::set<int> lpm_dev_dirty;
  // before a launch: a program that can delete invalidates every hash
  // lookup index; any other rebuilds the stale ones.  `lpm_written`: the LPM
  // tries the launch's program may update / delete (ORDERED batches only):
  // their lookups walk the replica (no flat table) while they change
  // `lpm`: the program names an LPM trie (loader.cpp lpm_write_sites); a
  // launch of one that does not leaves the tries as they are (their next
  // user uploads them, under the LPM launch lock)
  int prepare_ix(bool may_delete, uint64_t units, const std::vector<int> &lpm_written = {},
                 uint32_t lpm_update_sites = 0, bool lpm = true);
  // launches that may still run: one whose hash lookups use the block LDS
  // lookup cache (a found slot is trusted for the rest of the launch), one of
  // a program that can delete.  A cached launch never overlaps a deletion
  // (a program's, on any stream, or the host's): whichever comes second
  // waits for the device first (vm_api.cpp exec_batch, maps.cpp host delete)
  std::atomic<bool> lcache_inflight{false}, deleter_inflight{false};
  // LPM tries (vm_api.cpp exec_batch): launches of a runtime holding any are
  // prepared and launched under lpm_launch_mu; a launch that may write a
  // trie (ORDERED) waits for every launch that may still touch one, and any
  // launch after a writer waits for it
  std::mutex lpm_launch_mu;
  std::atomic<int> lpm_maps{0};
  std::atomic<bool> lpm_inflight{false}, lpm_writer_inflight{false};
  std::set<int> lru_maps;                // LRU_HASH maps
  std::atomic<uint64_t> lru_seq{1};      // LRU stamp sequence: launches and host-side ops (common.hpp)
  uint32_t lru_launches = 0;             // launches since the last tombstone check
  // before a launch: renumbers the LRU stamps before the sequence runs out,
  // compacts tombstone-heavy LRU tables now and then; returns the launch's
  // stamp sequence (0 on failure)
  uint64_t prepare_lru();
};

// hash lookup index upkeep for host-side writes (maps.cpp)
void ix_invalidate(int fd);
// the device replica of an LPM trie an ORDERED batch wrote, back into the
// host trie (no-op unless the trie is in lpm_dev_dirty)
int lpm_pull(int fd);

Runtime &rt();
void set_error(const std::string &e);

// What the syscall dispatch needs to know of a loaded VM's program
// (vm_api.cpp): bit 0 it calls bpf_override_return / bpf_set_retval (58 /
// 187), bit 1 it may store into the memory r1 points to (its unit: the
// dispatch then runs it on a copy of the records).  -1: no program loaded.
constexpr int kProgSetsRetval = 1, kProgStoresCtx = 2;
int vm_prog_flags(const ::ebpf_vm *vm);
// Drops every syscall attachment (bpftime_amd_reset; syscall_dispatch.cpp).
void syscall_detach_all();
// A loaded program's map effects (loader.hpp FastForm::map_fx, the syscall /
// raw entry form): per map fd FX_* bits and the bits that may reach any map.
// -1: no program loaded.
int vm_map_effects(const ::ebpf_vm *vm, std::map<int32_t, uint8_t> &fx, uint8_t &any);
// The thread-ordered syscall dispatch's launch (interp.hip k_sys_seq):
// `progs` in the reference's order (syscall_dispatch.cpp), over n device
// records laid out as `lay`; thread t's records perm[seg[t] .. seg[t + 1])
// (null perm / seg: one thread over every record in record order).  `err`: a
// device u32 (failed callbacks).  Returns the failed-callback count with
// EBPF_BATCH_SYNC, else 0; -1 on errors (set_error).
struct SeqAttach {
  const ::ebpf_vm *vm;
  int64_t sys_nr;
  bool enter;
};
int64_t seq_dispatch(const std::vector<SeqAttach> &progs, const SysLayout &lay, uint64_t n, const uint32_t *perm,
                     const uint32_t *seg, uint64_t nseg, int64_t *out, uint32_t flags, uint32_t *err, hipStream_t s);

}  // namespace bpftime_amd
