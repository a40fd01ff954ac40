// bpftime_amd: data structures shared by the host loader/runtime and the
// gfx950 interpreter kernel.  Everything here is plain-old-data so it can be
// hipMemcpy'd and read with scalar loads on the device.
#pragma once
#include <stdint.h>

// functions shared by the host runtime (g++) and the kernel (hipcc)
#ifdef __HIPCC__
#define BA_HD __host__ __device__
#else
#define BA_HD
#endif

namespace bpftime_amd {

constexpr uint32_t kMaxInsts = 65536;   // vm/vm-core/include/ebpf-vm.h:33-35
constexpr uint32_t kStackSize = 512;    // ebpf-vm.h:47-49
constexpr uint32_t kMaxFds = 1024;      // device map table size
constexpr uint32_t kBlock = 256;        // threads per workgroup (4 waves)
// KParams::dbg bit of the host linker's query launch (bpftime_amd_launch_fast_xlat):
// the kernel writes the asm tier's handler offsets and returns
constexpr uint32_t kDbgXlat = 1u << 30;
constexpr uint32_t kLdsStackMax = 64;   // per-lane stack bytes kept in LDS
constexpr uint32_t kComb = 256;         // per-block LDS combining entries (counter adds), minimum
constexpr uint32_t kCombMax = 4096;     // ... and maximum (a multiple of 8 in between, vm_api.cpp)
constexpr uint32_t kMissParts = 256;    // miss-log partitions (KParams::miss_log)

// Internal (pre-decoded) opcodes.  The device switch dispatches on these; the
// set is dense so the compiler's binary search over cases stays shallow.
enum XOp : uint8_t {
  X_BAD = 0,
  // ALU, same result for 32/64 after masking with `mask` (see DInsn::aux)
  X_ADD, X_SUB, X_MUL, X_OR, X_AND, X_XOR, X_MOV,
  // 64-bit only forms
  X_DIV64, X_MOD64, X_LSH64, X_RSH64, X_ARSH64, X_NEG64,
  // 32-bit only forms
  X_DIV32, X_MOD32, X_LSH32, X_RSH32, X_ARSH32, X_NEG32,
  X_LE, X_BE,
  // memory
  X_LDX, X_ST, X_STX, X_ATOMIC, X_LDDW,
  // fused "ldx r,[b+o]; add r,v; stx [b+o],r": one atomic add (A_FETCH: r
  // stays live and receives the old value + v)
  X_RMW_ADD,
  // control
  X_JA, X_JEQ, X_JGT, X_JGE, X_JSET, X_JNE, X_JSGT, X_JSGE, X_JLT, X_JLE, X_JSLT, X_JSLE,
  X_CALL, X_EXIT,
  X_NOP,  // second slot of lddw (never executed)
  X_COUNT
};

// DInsn::aux bits
constexpr uint8_t A_SRCREG = 0x01;  // second operand is a register
constexpr uint8_t A_W32 = 0x02;     // 32-bit ALU / JMP32
constexpr uint8_t A_SIZE_SHIFT = 4; // memory access size = 1 << ((aux >> 4) & 3)
constexpr uint8_t A_FETCH = 0x08;   // X_RMW_ADD: the loaded register stays live (DInsn::hi = it):
                                    // r = fetch_add(addr, v) + v, the ldx/add/stx in one atomic

// FInsn::w1 flags (per entry form and launch, loader.cpp build_fast / link_fast)
constexpr uint32_t FW_LCACHE = 2;   // hash lookup: probe / fill the block's LDS lookup cache (gen_fast.py)
constexpr uint32_t FW_MOVI = 4;     // a jump / exit with a fused `mov64 r, imm32` in front of it
                                    // (loader.cpp fuse_pairs: r in bits 3..6, the imm in aux)
constexpr uint32_t FW_MOVI_REG_SHIFT = 3;
constexpr uint32_t FW_NODEFER = 1;  // counter add: apply it to memory now (a later access of
                                    // the same unit may read or overwrite it, or the batch is
                                    // ORDERED): no per-wave delta cache, no LDS combining table

// 16-byte pre-decoded instruction: fetched with one s_load_dwordx4.
struct DInsn {
  uint8_t op;
  uint8_t dst;
  uint8_t src;
  uint8_t aux;
  int16_t off;
  uint16_t tgt;   // absolute jump target / next pc for fused ops
  int32_t imm;    // sign-extended immediate, or low half of lddw
  int32_t hi;     // high half of lddw, helper id (CALL), atomic op (ATOMIC)
};
static_assert(sizeof(DInsn) == 16, "DInsn must be 16 bytes");

// Map types (linux/bpf.h)
constexpr uint32_t MT_HASH = 1;
constexpr uint32_t MT_ARRAY = 2;
constexpr uint32_t MT_PROG_ARRAY = 3;
constexpr uint32_t MT_PERCPU_HASH = 5;
constexpr uint32_t MT_PERCPU_ARRAY = 6;
constexpr uint32_t MT_LRU_HASH = 9;
constexpr uint32_t MT_LPM_TRIE = 11;
constexpr uint32_t MT_RINGBUF = 27;

// Device-side map descriptor (64 B), indexed by fd.
//   ARRAY          data = value_size * max_entries, stride value_size
//   PERCPU_ARRAY   data = [idx][cpu][value_size]  (per_cpu_array_map.hpp:25-28)
//   HASH/PERCPU_HASH  nbuckets = next_prime(max_entries) slots of slot_size:
//                  [u32 state][u32 pad][key, padded to 8][value(s), padded to 8]
//                  state 0 = empty, 1 = filled, 2 = being written
//                  ix: lookup index beside that layout (see ix_pos), 0 = none
//   LRU_HASH       the HASH slot layout over nbuckets = next_prime(2 x
//                  max_entries + 1), state 3 = tombstone (deleted / evicted;
//                  probes go past it, inserts reuse it); at count_addr the u64
//                  element count and (+8) the u64 tombstone count, at
//                  count_addr + 128 a u64 last-use stamp per bucket (see
//                  lru_stamp); no lookup index
//   RINGBUF        u64 consumer position at data, u64 producer position at
//                  data + 128 (own cache lines), 2 x max_entries record bytes
//                  at data + 256 (ringbuf_map.cpp layout and record format)
//   PROG_ARRAY     int32 prog fd per index, -1 = empty (prog_array.cpp's
//                  INVALID_ENTRY; host-authoritative, read-only on the device)
//   LPM_TRIE       device replica of the host trie: a 16-B header {i32 root
//                  node, u32 nodes, u32 entries, u32 pool capacity} then nodes
//                  of slot_size bytes {u32 prefixlen, u32 intermediate, i32
//                  child[2], prefix data at key_off = 16, value at val_off};
//                  read-only except in ORDERED batches of a program that
//                  updates / deletes (dev_helpers.hpp lpm_update)
struct DMap {
  uint32_t type;
  uint32_t key_size;
  uint32_t value_size;
  uint32_t max_entries;
  uint64_t data;        // device address
  uint32_t nbuckets;
  uint32_t ix_mask;     // lookup index entries - 1 (a power of two minus one)
  uint32_t slot_size;
  uint32_t key_off;     // = 8
  uint32_t val_off;     // = 8 + round8(key_size)
  uint32_t ncpu;        // per-CPU slot count
  uint64_t count_addr;  // device address of the u64 element counter (hash)
  uint64_t ix;          // device address of the u32 lookup index, 0 = not valid (LPM_TRIE: its flat table)
};
static_assert(sizeof(DMap) == 64, "DMap must be 64 bytes");

// Hash-map lookup index.  bpftime_hash_map's linear probing (kept as the
// storage layout, so get_next_key walks buckets in the reference's order)
// degrades to cluster walks of thousands of slots as the table fills (65536
// flows in 65537 buckets at config 3).  Beside it sits an open-addressing
// table of u32 {bucket + 1} entries, at most half full, keyed by a mix of the
// same h*31 hash: a lookup that finds its key through it returns the slot the
// reference probe would return, because the index only holds keys that
// probe reaches (no deletions since the index was built, or a rebuild that
// skipped keys orphaned by deletions, bpftime_hash_map.hpp:182-199).
// Anything else falls back to the reference probe.
inline BA_HD uint32_t ix_pos(uint64_t h, uint32_t mask) {
  uint32_t g = ((uint32_t)h ^ ((uint32_t)(h >> 32) * 0x85EBCA6Bu)) * 0x9E3779B1u;
  return (g ^ (g >> 16)) & mask;
}
constexpr uint32_t kIxProbes = 8;  // asm tier: index probes before the C++ tier's lookup
// An index entry an insert holds while it claims a bucket for its key
// (dev_helpers.hpp hash_find_ix), and the table's bucket bitmap after the
// index: bit b = bucket b is not EMPTY (bits past nbuckets set), kept by
// device inserts while the index is valid and rebuilt with it (maps.cpp)
constexpr uint32_t kIxRes = 0xffffffffu;
// Keyed indexes (keys of at most 16 B): beside the u32 entries, the key of
// each entry at the same position in an array of 8-B (keys <= 8 B) or 16-B
// slots, so a probe loads entry and key together and never reads the bucket
// (one round trip per probe instead of entry, then bucket: flow-hash 0.83 ->
// 0.67 ms; config 3's index of 262,144 positions is 5 MiB, a lookup touching
// one key line as the reference probe touches one bucket line; at 131,072
// positions the waves' longest probes made it slower, 0.85 ms).  Longer keys
// keep only the entries and compare in the bucket.  An
// insert writes the key before it publishes the entry (dev_helpers.hpp
// ix_insert).  Layout: entries, keys, then the bucket bitmap.
BA_HD constexpr uint32_t ix_key_stride(uint32_t key_size) { return key_size <= 8 ? 8 : key_size <= 16 ? 16 : 0; }
inline BA_HD uint64_t ix_keys(uint64_t ix, uint32_t mask) { return ix + 4ull * ((uint64_t)mask + 1); }
inline BA_HD uint64_t ix_bitmap(uint64_t ix, uint32_t mask, uint32_t key_size) {
  return ix + (4ull + ix_key_stride(key_size)) * ((uint64_t)mask + 1);
}
inline BA_HD uint64_t ix_bitmap_words(uint64_t nbuckets) { return (nbuckets + 63) / 64; }

// LRU_HASH recency (lru_var_hash_map.cpp keeps a doubly linked list, head =
// most recently used).  Here every element carries the stamp of its last
// use, and the list order is the stamp order: move_to_head = a larger stamp,
// the tail = the smallest.  A stamp is {sequence:24 | unit:32 | op:8}: the
// sequence counts launches and host-side operations (Runtime::lru_seq), the
// unit is the unit's index in its batch, the op counts the unit's LRU
// operations.  Units of a parallel batch raise a stamp with an atomic max, so
// after the batch every element holds the stamp of its last use in unit
// order -- the order a serial run of the batch leaves.
constexpr uint32_t kLruUnitShift = 8;
constexpr uint32_t kLruSeqShift = 40;
constexpr uint64_t kLruSeqLimit = 1ull << 23;  // renumber the stamps before the sequence gets here
constexpr uint32_t kLruScan = 256;             // parallel batches: buckets examined per eviction

// bpf_tail_call (helper 12, bpf_helper.cpp:568-650).  The reference runs the
// target as a nested exec over a 64-B copy of the ctx and returns its r0 to
// the caller (depth <= 32).  Here the caller and every program a PROG_ARRAY
// can name are linked into one image at launch (vm_api.cpp), the targets'
// exits become calls of kRetHelper, and a call pushes a per-lane frame
// {r1..r10, return pc, ctx bytes, stack bytes} that the matching return pops:
// the callee runs on the same stack and ctx, restored afterwards, which is
// what a copy gives it.
constexpr uint32_t kTailHelper = 12;
constexpr int32_t kRetHelper = 0x7fff0001;  // internal: a linked target's exit
constexpr uint32_t kTailDepth = 32;          // MAX_TAIL_CALL_CNT
constexpr uint32_t kTailGrid = 1024;         // blocks per launch of an image with tail calls
constexpr uint32_t kFrameCtx = 64;
constexpr uint32_t kFrameHdr = 96;           // r1..r10, ctx address, ret pc, ctx bytes
constexpr uint32_t kFrameBytes = kFrameHdr + kFrameCtx + kStackSize;
// Frame header word 11: return pc | ctx bytes << 32 (a full frame: r1..r10,
// the ctx address and cb ctx bytes from it, the whole stack), or with
// kFrameMasked: the lane's own LDS ctx, and only the registers of the live
// mask (bit r: r1..r9, header bits 41..), the ctx / stack words of the
// image's save masks (KParams tail_ctx_mask / tail_stack_mask); r10 is the
// stack top again after the return
constexpr uint64_t kFrameMasked = 1ull << 40;
constexpr uint32_t kFrameLiveShift = 40;  // + r: the bit of register r (1..9)
// ... and bit kFrameRematShift + r: register r held the lane's own ctx
// pointer at the call (not saved; the return sets it again)
constexpr uint32_t kFrameRematShift = 50;
// LDS frames (XDP images, depth < KParams tail_lds & 0xff): a masked frame of
// a lane at depth d is the words [d][w][lane] of the block's LDS frame area
// (after the combining table): w = 0 the header (as word 11; 0 = the frame is
// in global memory, a full frame the C++ tier pushed), then the live
// registers in order, the ctx words of the ctx mask, the stack words of the
// stack mask (vm_api.cpp sizes words = 1 + the most live registers of a tail
// call + both masks' words, and the depths to keep the block's residency)
constexpr uint32_t kTailLdsMax = 4;  // depths held in LDS at most

// Map effects of a program (loader.hpp FastForm::map_fx): loads (and lookups), counter adds whose order no
// one observes (fused ld/add/st and atomic adds without fetch), every other
// write (stores, fetching or non-add atomics, update / delete / ring calls)
constexpr uint8_t FX_READ = 1, FX_ADD = 2, FX_WRITE = 4;

// Context kinds for a batch
constexpr uint32_t CTX_RAW = 0;      // r1 = unit memory, r2 = length
constexpr uint32_t CTX_XDP = 1;      // r1 = xdp_md_userspace (48 B, LDS)
constexpr uint32_t CTX_SYSCALL = 2;  // r1 = trace_event_raw_sys_enter (64 B) or, for
                                     // EBPF_CTX_SYSCALL_EXIT batches, trace_event_raw_sys_exit (24 B)

// Launches of at least this many units build the flat table of an IPv4 LPM
// trie changed since the last one (maps.cpp prepare_ix); smaller ones walk
constexpr uint64_t kLpmFlatMinUnits = 1ull << 16;
// LPM replica header word 3: an ORDERED batch's update found the node pool
// full (dev_helpers.hpp lpm_update; the host fails the batch, maps.cpp)
constexpr uint32_t kLpmPoolOut = 0x80000000u;

// Ring-buffer staging per block (dev_helpers.hpp RbStage)
// (8 KiB: a block at one wave per resident slot holds its units' samples;
// ringbuf-sample 1.45 ms with 2 KiB at 4 waves per slot, 1.10 ms with 8 KiB
// at one)
constexpr uint32_t kRbStageRec = 8192;                                // record bytes (a ring budget) per block
constexpr uint32_t kRbStageMaxRec = kRbStageRec / 8;                  // records per block (>= 8 B each)
constexpr uint32_t kRbStageBytes = kRbStageRec + 4 * kRbStageMaxRec;  // + u32 record offsets

// Kernel launch parameters (passed by value).
struct FInsn;
// (k_interp copies every field through an SGPR barrier, interp.hip: a new
// field must be copied there too)
struct KParams {
  const DInsn *prog;
  const FInsn *fast;      // threaded-code form for the asm fast path
  uint32_t fast_div;      // lane groups (divergence) may be scheduled in asm
  uint32_t comb_entries;  // LDS combining entries per block (0: none; sized per launch, vm_api.cpp)
  const DMap *maps;
  uint8_t *data;          // base of unit slots (device)
  const uint32_t *lens;   // per-unit lengths or nullptr
  uint32_t *verdicts;     // u32 r0 per unit (nullable)
  uint64_t *rets;         // u64 r0 per unit (nullable)
  int32_t *out_data_off;  // XDP: data - slot after the program (nullable)
  uint32_t *out_len;      // XDP: data_end - data after the program (nullable)
  uint32_t *err_count;    // device counter of units whose exec failed
  uint64_t n;
  uint64_t stride;
  uint64_t first_unit;    // global index of unit 0 (virtual-cpu assignment)
  // (host-computed for the launch's grid, so the kernel divides nothing:
  // (n - 64) / (grid x block) and its remainder -- a wave's chained
  // iterations, interp.hip `full` -- and (grid x block / 64) % ncpu)
  uint64_t full_q, full_r;
  uint32_t step_cpu;
  uint64_t data_lo, data_hi;    // allowed global window #1 (the batch)
  uint64_t arena_lo, arena_hi;  // allowed global window #2 (map arena)
  uint64_t step_limit;    // max executed insns per unit
  uint32_t fixed_len;
  uint32_t stack_size;    // per-lane stack bytes (multiple of 8)
  uint32_t ncpu;          // virtual CPU count (helper 8, per-CPU maps)
  uint32_t ifindex;
  uint32_t rxq;
  uint32_t checked;       // 1 = confine global accesses to the two windows
  uint32_t head;          // XDP: initial data offset inside each slot
  uint32_t ordered;       // 1 = a single lane runs the units in index order
  uint32_t stage;         // bytes of each unit staged in VGPRs by the fast path (0 = none)
  uint32_t needs_ctx;     // XDP: the program reads its ctx generically (build it in LDS)
  const uint64_t *descs;  // AF_XDP descriptors {u64 addr; u32 len; u32 options} or nullptr
  uint64_t umem_bytes;    // descriptor mode: bytes at data
  int64_t sys_nr;         // CTX_SYSCALL: run only records with this id (-1: every record)
  const int32_t *tail_entry;  // prog fd -> entry pc in the linked image, -1 = not linked (nullable)
  uint8_t *frames;        // tail-call frames: [kTailDepth][frame_words][grid * kBlock lanes] u64 (per stream)
  uint32_t frame_words;   // header + ctx + the image's stack bytes, / 8
  uint64_t *flush_log;    // block-end counter deltas: [grid][log_words] (k_comb_merge adds them), or nullptr
  uint32_t log_words;     // u64 words per block: count, then {tag, delta} pairs
  uint64_t *lane_scratch; // a u64 per lane of the grid (PROG_ARRAY lookups hand out a copy there), or nullptr
  uint32_t dbg;           // BPFTIME_AMD_DBG experiment bits (0 in production)
  uint64_t *dbg_counts;   // dbg 512: lookup-cache hits, misses (u64 each), or nullptr
  int32_t unwind_idx;     // ebpf_set_unwind_function_index: helper whose 0 return ends the unit (-1 none)
  uint64_t lru_seq;       // this launch's LRU stamp sequence (common.hpp kLruSeqShift)
  uint32_t tail_ctx_mask;    // XDP images: ctx words / stack words a frame keeps (loader.cpp tail_save_masks)
  uint32_t tail_stack_mask;
  // XDP images: frames of the first (tail_lds & 0xff) depths pushed by the asm
  // tier live in LDS, (tail_lds >> 8) u64 words each (common.hpp kFrameLds*)
  uint32_t tail_lds;
  uint32_t lcache;           // the block's hash-lookup cache: its sets (0 = none; lcache_sets())
  uint64_t *gregs;           // r0..r10 copies for the C++ tier: [grid][11][kBlock] u64 (k_interp G), or nullptr (LDS)
  uint8_t *rb_stage;         // ring-buffer staging: [grid][kRbStageBytes] right after lane_scratch's words, or nullptr
  uint8_t *gctx;             // XDP: the lanes' ctx in global memory ([grid lane] x 48 B, after the staging), or nullptr (LDS)
  uint64_t *miss_log;        // combining-table misses: [grid][kMissParts][miss_cap] {tag, delta} records, or nullptr
  uint32_t *miss_counts;     // [grid][kMissParts] records each block wrote (k_miss_merge reads them)
  uint32_t miss_cap;         // records per block and partition (even)
  const int32_t *tail_slots; // images: per PROG_ARRAY fd the offset of its slots' entry pcs, then those (vm_api.cpp)
  // syscall dispatch state (include/ebpf-vm.h struct ebpf_batch): per unit
  // override flags and return value, the phase bit (1 enter, 2 exit), or null
  uint32_t *sys_state;
  int64_t *sys_ret;
  uint32_t sys_phase;
  // bpf_get_current_pid_tgid: a u64 at this offset from the unit (recorded
  // syscalls), or (0) the launching thread's value
  int32_t pid_off;
  uint64_t pid_tgid;
  // the C++ tier's view of both (include/ebpf-vm.h): unit i's recorded
  // caller at pid_base + i * pid_stride (pid_base null: the launching
  // thread's), its recorded clock at kt_base + i * kt_stride (null: the
  // device clock) -- offsets from the unit and struct-of-arrays alike
  const uint8_t *pid_base;
  uint64_t pid_stride;
  const uint8_t *kt_base;
  uint64_t kt_stride;
  // per-lane LDS strides of the XDP ctx and the stack (lane_stride)
  uint32_t ctx_stride, stack_stride;
};

// Where a syscall replay's fields live (include/bpftime_amd.h): record i's
// enter ctx (64 B) at enter + i * estride (null: no enter ctx, the id comes
// from the exit ctx), its exit ctx (24 B) at exit + i * xstride (null: 64-B
// enter records, which hold no ret), its caller's pid_tgid at pid + i *
// pstride (null: the dispatching thread's), its clocks {enter ns, exit ns}
// at clock + i * cstride (null: the device clock)
struct SysLayout {
  const uint8_t *enter;
  uint64_t estride;
  const uint8_t *exit;
  uint64_t xstride;
  const uint8_t *pid;
  uint64_t pstride;
  const uint8_t *clock;
  uint64_t cstride;
};

// Thread-ordered syscall dispatch (interp.hip k_sys_seq, syscall_dispatch.cpp):
// one lane per recorded thread walks that thread's records in record order
// and, per record, runs the attached programs the way dispatch_syscall does
// (attach/syscall_trace_attach_impl/src/syscall_trace_attach_impl.cpp:18-95).
// The programs in the reference's order: per-syscall enter programs, global
// enter, per-syscall exit, global exit (attach order inside each group).
struct SeqProg {
  const DInsn *prog;
  const FInsn *fast;    // its ORDERED link (every counter add reaches memory at once)
  int64_t sys_nr;       // -1: every syscall
  uint32_t enter;       // 1 sys_enter, 0 sys_exit
  uint32_t pad;
};
static_assert(sizeof(SeqProg) == 32, "SeqProg is read with scalar loads");
constexpr uint32_t kSeqMaxProgs = 64;  // attached programs a thread-ordered dispatch runs (kernel arguments)
// k_sys_seq's per-lane ctx copy: the 64-B ctx, then the record's caller
// (pid_tgid) and the clock of the callback's phase, read by the asm tier's
// CALL_REC handler (loader.cpp link_fast rec_helpers)
constexpr uint32_t kSeqPidOff = 64, kSeqClockOff = 72, kSeqCtxWords = 10;
// threads up to which the thread-ordered dispatch runs its callbacks in the
// asm tier (vm_api.cpp seq_dispatch)
constexpr uint64_t kSeqAsmThreads = 16384;
struct SeqParams {
  uint32_t nprogs;
  // the records' fields (include/bpftime_amd.h: 64- / 96- / 128-B records or
  // struct-of-arrays), record i's at base + i * stride:
  SysLayout lay;
  uint64_t n;
  // thread t's records: perm[seg[t] .. seg[t + 1]) (record indexes in record
  // order); null perm: the identity; null seg: one thread over [0, n)
  const uint32_t *perm;
  const uint32_t *seg;
  uint64_t nseg;
  int64_t *out;           // what dispatch_syscall returns per record (nullable)
  const DMap *maps;
  uint32_t ncpu;
  uint32_t checked;
  uint64_t arena_lo, arena_hi;
  uint64_t step_limit;
  uint64_t lru_seq;
  uint64_t pid_tgid;      // 64-B records: the dispatching thread's
  uint32_t *err_count;    // failed callbacks
  uint32_t exact;         // one lane over every record (EBPF_BATCH_ORDERED)
  // 1: every program keeps its stack within kLdsStackMax bytes: the stacks
  // live in LDS and the callbacks run in the asm tier (seq_lds_bytes); 0:
  // private stacks, the C++ tier only
  uint32_t fast;
  SeqProg progs[kSeqMaxProgs];  // in the kernel arguments: scalar loads, no upload
};
static_assert(sizeof(SeqParams) <= 4096, "kernel arguments");

// Combining-table misses.  A deferred counter add that finds no table entry
// (the set is full of other granules) does not become a memory-side atomic
// at once: its lane appends {tag, delta} records (tag = address | (4-byte ?
// 1 : 0); two records per lane, the second {address + 8, delta} for fused
// pairs, else empty) to its block's region of a miss log, partitioned by a
// hash of the address (gen_fast.py comb_add), counting in LDS.  A second
// launch, k_miss_merge, gives every partition a block that combines the
// records of all blocks in an LDS table and adds each address's sum with one
// device atomic: the long tail of a Zipf key set appears in many blocks, a
// few times in each.  A full partition region, or a merge table, adds
// directly.  (kMissParts partitions: with the constants at the top)

// Block-end counter deltas.  Every block holds its counter deltas (the wave
// caches of uniform counters, the LDS combining table) until it ends; with a
// flush log it appends them to its own log region instead of adding them to
// memory, and k_comb_merge (a second launch on the same stream) merges
// kMergeGroup blocks' logs in an LDS table before adding: the same addresses
// are hot in every block, and same-address device atomics serialize at the
// memory side (a map of a few hundred values sits in a handful of channels).
BA_HD constexpr uint32_t wave_cache_entries(uint32_t block) { return (block / 64) * 2; }
// A combining-table entry e = set * 8 + way: its u32 tag sits in the tags of
// ways 0-3 of every set ([set][4]) or, for ways 4-7, in the same array after
// them (gen_fast.py comb_add: a set's first four tags are one 16-byte LDS
// slot, and consecutive sets take consecutive slots of a bank row)
BA_HD constexpr uint32_t comb_tag_pos(uint32_t e, uint32_t entries) {
  return (e & 7) < 4 ? (e >> 3) * 4 + (e & 3) : entries / 2 + (e >> 3) * 4 + (e & 3);
}
// The delta granules after the tags, a row of 8 x 16 B per set padded to
// kCombRowBytes: way k of set s starts at bank ((s * 36 + k * 4) mod 32), so
// lanes adding to the first ways of different sets no longer queue on the
// same banks (with 128-B rows every set's way 0 sat on banks 0-3: flow-hash
// 9.6 conflict cycles per LDS instruction)
constexpr uint32_t kCombRowBytes = 144;
BA_HD constexpr size_t comb_bytes(uint32_t entries) { return 4 * (size_t)entries + (size_t)(entries / 8) * kCombRowBytes; }
BA_HD constexpr uint32_t comb_granule_off(uint32_t e) { return (e >> 3) * kCombRowBytes + (e & 7) * 16; }
constexpr uint32_t kMergeGroup = 16;
constexpr uint32_t kMergeEntries = 4096;  // merge table entries (64 KiB of LDS)
// (a combining-table entry flushes up to four counters: gen_fast.py comb_add)
inline uint32_t log_words_for(uint32_t comb_entries, uint32_t block = kBlock) {
  return 1 + 2 * (wave_cache_entries(block) + 4 * comb_entries);
}

// Launches whose C++-tier register copy lives in global memory (k_interp G:
// a combining table or lookup cache, no tail-call image, no ring staging)
// run kBigBlock-lane blocks: one combining table and lookup cache serve 16
// waves instead of 4, so the LDS a table takes no longer caps the CU at 2
// blocks of 4 waves (flow-hash: 8 -> 16 resident waves per CU at the same
// or a larger table reach)
constexpr uint32_t kBigBlock = 1024;
constexpr size_t kCuLds = 160 * 1024;  // LDS per CU (gfx950)

// Dynamic LDS of an interpreter block: the lanes' XDP ctx (48 B each), their
// stacks (LDS-stack programs), 48 B of launch constants (interp.hip
// tenv; the asm finds them 48 B before the combining table), the combining
// table (a u32 tag per entry, then the delta rows: comb_bytes).
// tenv: 8 u64 launch constants (tail calls, the register copy base, the
// block's miss-log region and its capacity), then kMissParts u32 miss counters,
// then the block's ring staging area (u64, 0 = none) and the LDS address of
// its counters (dev_helpers.hpp RbLds; gen_fast.py call_rbout)
constexpr uint32_t kTenvRb = 64 + 4 * kMissParts;     // (u64 index kTenvRb / 8)
// then (XDP images) the LDS tail-call frames: their LDS address minus the
// lane columns' (interp.hip Rf), the depths they hold | words per frame << 8
// (KParams tail_lds; gen_fast.py tail_env)
constexpr uint32_t kTenvLf = kTenvRb + 16;
constexpr uint32_t kTenvBytes = kTenvLf + 16;          // gen_fast.py TENV
// k_sys_seq's dynamic LDS with the asm tier on: the lanes' stacks, then the
// asm's launch constants (tenv, zero: no tail calls, staging or tables) in
// front of an empty combining table
inline size_t seq_lds_bytes(uint32_t block, bool fast) {
  return fast ? (size_t)block * kLdsStackMax + kTenvBytes : 0;
}
// Hash-lookup cache of a block (programs whose hash lookups the loader marks
// FW_LCACHE: no deletions): `sets` 2-way sets, the ways' 16-B keys
// ([set][way]) then their u32 entries {(slot + 1) | fd << 22}, right below
// the tail-call constants (gen_fast.py lcache_probe; the lookup's FInsn w4
// carries the set count).  A slot found for a key stays that key's slot for
// the rest of a launch when nothing deletes.
constexpr uint32_t kLcacheSets = 1024;  // default set count (BPFTIME_AMD_LCACHE_SETS: vm_api.cpp lcache_sets)
BA_HD inline size_t lcache_bytes(uint32_t sets) { return (size_t)(32 + 8) * sets; }
// ... and after the table, the LDS tail-call frames of an XDP image
// (tail_lds: depths | words per frame << 8; [depth][word][lane] u64)
BA_HD constexpr uint32_t tail_lds_lane_bytes(uint32_t tail_lds) { return (tail_lds & 0xff) * (tail_lds >> 8) * 8; }
// Per-lane LDS areas (the XDP ctx, the stack) at a lane stride of 8 x an odd
// number of bytes (BPFTIME_AMD_LANE_PAD=1; off by default, vm_api.cpp
// lane_pad): the same offset in 16 lanes' areas then falls on 16 different
// bank pairs (dword d of lane t at bank (stride / 4 * t + d) mod 32, stride
// / 4 = 2 x odd), where a power-of-two stride puts every fourth lane on one
// bank (flow-hash's 32-B stacks: 4-way conflicts on every stack access).
// Host side; the kernel takes the strides from KParams.
bool lane_pad();
inline uint32_t lane_stride(uint32_t bytes) {
  return !lane_pad() || ((bytes / 8) & 1) || bytes == 0 ? bytes : bytes + 8;
}
constexpr uint32_t kXdpCtxBytes = 48;  // xdp_md_userspace (runtime/extension/userspace_xdp.h:6-17)

inline size_t dyn_lds_for(uint32_t kind, bool big_stack, uint32_t stack_size, uint32_t comb_entries,
                          uint32_t lcache_sets = 0, bool ctx_lds = true, uint32_t block = kBlock,
                          uint32_t tail_lds = 0) {
  return (size_t)block * ((kind == CTX_XDP && ctx_lds ? lane_stride(kXdpCtxBytes) : 0) +
                          (big_stack ? 0 : lane_stride(stack_size)) +
                          tail_lds_lane_bytes(tail_lds)) +
         lcache_bytes(lcache_sets) + kTenvBytes + comb_bytes(comb_entries);
}

// Error codes recorded per unit (err_count counts units with any error)
constexpr uint32_t E_OK = 0;
constexpr uint32_t E_OOB = 1;
constexpr uint32_t E_STEPS = 2;
constexpr uint32_t E_BADOP = 3;

}  // namespace bpftime_amd
