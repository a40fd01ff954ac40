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

struct LoadOut {
  std::vector<DInsn> prog;
  std::vector<FInsn> fast;   // threaded-code form of `prog` (gen_fast.py)
  uint32_t stack_size = 8;   // per-lane bytes (LDS)
  bool big_stack = false;    // 512-B scratch stack
  uint32_t fused_rmw = 0;
  uint32_t comb_entries = 0;  // per-block LDS combining entries (0 = none needed)
};

// Helper ids the device implements (interp.hip helper switch).
bool device_helper_supported(uint32_t id);

// Threaded-code records for the asm fast path: one per DInsn; instructions
// without a fast handler dispatch to F_SLOW (the C++ interpreter).  `xdp`
// selects the entry convention (r1 = XDP ctx, else r1 = the unit's slot);
// loads/stores whose base pointer kind is known statically get
// specialized handlers (count in *specialized).
void build_fast(const std::vector<DInsn> &prog, bool xdp, bool big_stack, uint32_t stack_size,
                std::vector<FInsn> &fast, uint32_t *specialized, bool *needs_comb);

// Runs the compat_ubpf.cpp:61-200 patching (call remap check, lddw pseudo
// sources), ubpf-style validation, pre-decoding and the dataflow analyses
// (liveness for RMW fusion, stack depth).  Returns 0 or <0 with `err`.
int load_program(const RawInsn *code, size_t n, const std::map<size_t, size_t> &helper_id_map,
                 const std::map<size_t, std::string> &helper_names, const LddwHelpers &lddw,
                 LoadOut &out, std::string &err);

}  // namespace bpftime_amd
