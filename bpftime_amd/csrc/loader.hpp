// bpftime_amd: host-side program loader for the device interpreter.
#pragma once
#include <stdint.h>
#include <map>
#include <string>
#include <vector>
#include "common.hpp"
#include "fast_ops.hpp"

namespace bpftime_amd {

// ebpf_inst (vm/compat/include/ebpf_inst.h:22-28)
struct RawInsn {
  uint8_t code;
  uint8_t dst : 4;
  uint8_t src : 4;
  int16_t off;
  int32_t imm;
};
static_assert(sizeof(RawInsn) == 8, "ebpf_inst is 8 bytes");

struct LddwHelpers {
  uint64_t (*map_by_fd)(uint32_t) = nullptr;
  uint64_t (*map_by_idx)(uint32_t) = nullptr;
  uint64_t (*map_val)(uint64_t) = nullptr;
  uint64_t (*var_addr)(uint32_t) = nullptr;
  uint64_t (*code_addr)(uint32_t) = nullptr;
};

// A packet / slot access at a constant offset (resolved per launch by
// link_fast once the batch head and staged window are known).
struct FStatic {
  uint8_t kind = 0;  // 0 none, 1 packet (ctx->data + at), 2 slot (+ at)
  uint8_t op = 0;    // 0 LDX, 1 STX, 2 ST, 3 bpf_ringbuf_output source (imm: the ring fd)
  uint8_t sz = 0;
  uint8_t pad = 0;
  int32_t at = 0;
  int32_t imm = 0;   // ST immediate (op 3: the ring fd)
};

// Threaded-code form of a program for one entry convention.
// The blocks' hash-lookup cache sets (common.hpp kLcacheSets; a power of two
// in [256, 4096] from BPFTIME_AMD_LCACHE_SETS, read once)
uint32_t lcache_sets();

struct FastForm {
  std::vector<FInsn> fast;     // templates (generic handlers for static accesses)
  std::vector<FStatic> stat;   // per insn
  uint32_t specialized = 0;    // accesses / calls with statically typed bases
  bool needs_comb = true;      // per-lane counter adds (LDS combining table)
  bool needs_ctx = true;       // XDP: the ctx must exist in LDS
  bool needs_lcache = false;   // a hash lookup uses the block's LDS lookup cache (FW_LCACHE)
  // counter addresses a block's deferred per-lane adds can reach (an upper
  // bound from the maps they target; ~0u: unknown): sizes the combining table
  uint32_t comb_hint = ~0u;
  std::vector<uint8_t> add_site;  // per insn: a counter add (fused RMW, atomic add without fetch)
  std::vector<uint8_t> join;      // per insn: a jump target or an entry (no superinstruction ends there)
  // linked images, XDP form: the ctx words (bit k = bytes [8k, 8k+8)) and
  // LDS stack words (bit j = the j-th 8 bytes from the stack bottom) that a
  // tail-call target may write -- what a frame must save for its caller
  uint32_t tail_ctx_mask = 0x3f, tail_stack_mask = 0xffffffffu;
  uint32_t tail_max_live = 9;  // the most registers a tail call's frame keeps (FInsn imm popcount)
  // map_update_elem (2) / map_delete_elem (3) call sites that may reach an
  // LPM trie: {helper id, map fd}.  The device changes a trie only in ORDERED
  // batches (dev_helpers.hpp lpm_update); vm_api.cpp refuses other batches
  std::vector<std::pair<uint32_t, int32_t>> lpm_writes;
  bool names_lpm = false;  // an lddw names an LPM trie (its launches take the LPM launch lock)
  // a store may reach the unit r1 points to at entry (the pointer kinds
  // cannot place every store on the stack, a map value or a constant)
  bool stores_unit = true;
  // What the program does to each map it can reach (the syscall dispatch
  // decides from it whether attached programs commute, syscall_dispatch.cpp):
  // per map fd FX_* bits, and the bits of accesses the pointer kinds cannot
  // attribute to one map (they may reach any)
  std::map<int32_t, uint8_t> map_fx;
  uint8_t any_fx = FX_READ | FX_WRITE;
};

struct LoadOut {
  std::vector<DInsn> prog;
  std::vector<uint8_t> lddw_src;  // per pc: the lddw pseudo source (BPF_PSEUDO_MAP_FD = 1, ...)
  uint32_t stack_size = 8;   // per-lane bytes (LDS)
  bool big_stack = false;    // 512-B scratch stack
  uint32_t fused_rmw = 0;
  uint32_t comb_entries = 0;  // per-block LDS combining entries (0 = none needed)
  bool may_delete = false;    // calls map_delete_elem: hash lookup indexes stop being valid
  bool tail_call = false;     // calls bpf_tail_call: linked with the prog arrays' targets at launch
  bool sets_retval = false;   // calls bpf_override_return (58) / bpf_set_retval (187)
  bool multi_entry = false;   // a linked image (tail-call targets are extra entries)
  std::vector<uint32_t> entries;  // the linked targets' entry pcs
  std::vector<uint16_t> tail_live;  // per pc: registers r1..r9 live after a bpf_tail_call (bit r)
};

// Helper ids the device implements (interp.hip helper switch).
bool device_helper_supported(uint32_t id);

// Threaded-code records for the asm fast path: one per DInsn; instructions
// without a fast handler dispatch to F_SLOW (the C++ interpreter).  `xdp`
// selects the entry convention (r1 = XDP ctx, else r1 = the unit's slot);
// loads/stores/calls whose base pointer kind is known statically get
// specialized handlers (count in out.specialized).
void build_fast(const LoadOut &lo, bool xdp, FastForm &out);

// Staged bytes the static packet / slot accesses need for a batch head
// (0..64, multiple of 16).
uint32_t stage_need(const FastForm &f, uint32_t head);

// Final FInsn array for one launch configuration: static accesses inside a
// `stage`-byte window get the staged handlers (dword index, shift, masks
// precomputed), the rest keep their generic templates.
// `ordered`: every counter add gets its direct (FW_NODEFER) handler.
// `unwind_idx`: the VM's unwind helper (-1 none); its calls run in C++.
// `pid_off` (1..255): bpf_get_current_pid_tgid reads the u64 at the unit +
// pid_off in asm (recorded syscalls, KParams pid_off); else it runs in C++.
// `lc_sets` 0: no lookup cache in the launch (FW_LCACHE cleared).
// `no_kldx`: constant-address loads through the vector path (the launch
// runs other programs that may write them).  `rec_helpers`: caller and
// clock from beside the ctx copy (the thread-ordered kernel).
void link_fast(const FastForm &f, uint32_t head, uint32_t stage, bool ordered, const std::vector<DInsn> &prog,
               std::vector<FInsn> &out, int32_t unwind_idx = -1, uint32_t lc_sets = 0, uint32_t pid_off = 0,
               bool no_kldx = false, bool rec_helpers = false);

// Runs the compat_ubpf.cpp:61-200 patching (call remap check, lddw pseudo
// sources), ubpf-style validation, pre-decoding and the dataflow analyses
// (liveness for RMW fusion, stack depth).  Returns 0 or <0 with `err`.
int load_program(const RawInsn *code, size_t n, const std::map<size_t, size_t> &helper_id_map,
                 const std::map<size_t, std::string> &helper_names, const LddwHelpers &lddw,
                 LoadOut &out, std::string &err, const std::vector<uint32_t> &entries = {});

}  // namespace bpftime_amd
