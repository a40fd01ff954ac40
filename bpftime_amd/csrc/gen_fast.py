"""Generates the gfx950 threaded-code fast path of the interpreter.

    python gen_fast.py  ->  fast_asm.inc, fast_ops.hpp   (run by the Makefile)

The uniform interpreter loop (every live lane of the wave at one pc) is one
inline-asm block.  Each eBPF instruction is pre-decoded by the loader into a
32-byte FInsn whose first word is the byte offset of its handler's entry in
a table of `s_branch` instructions; dispatch is

    s_load_dwordx8 W, PROG, IP    ; fetch (scalar cache, IP = byte offset)
    s_add_u32/s_addc_u32 T, TB, W0
    s_setpc_b64 T                 ; -> table entry -> handler

instead of a compare tree.  exec = the wave's live lanes inside the block, so
compare results and stores need no per-lane predication.

Cost model (MI355X_MICROARCH.md): a CU has ONE scalar unit shared by its four
SIMD-32s, each of which retires a wave64 VALU instruction every 2 cycles, so
at 16 waves per CU the SALU is the first pipe to saturate.  The handlers are
written to minimise SALU instructions per eBPF instruction: one SALU to
advance IP, two to form the handler address, no per-instruction step count
(steps are counted at taken jumps, the only way to loop), and register
operands read and written in place under GPR-index mode.

Registers.  r0..r10 live in VGPRs v[60:81] (r_i = v[60+2i : 61+2i]) while the
block runs; an instruction's register fields are VGPR indices used with
`s_set_gpr_idx_on` (register numbers are wave-uniform).  Where the eBPF
operation is `dst op= y` the VALU instruction itself runs in index mode
(SRC0/SRC1 and DST indexed by dst*2), so the register is neither copied out
nor back.  The C++ side keeps its LDS copy (lane-major, 2 KiB per register):
a fresh unit initialises the VGPRs from operands, a re-entry loads them from
LDS, and every exit other than `exit` stores them back.

Unit staging.  On a fresh unit the first %[stage] bytes (16..64, sized per
launch from the program's statically typed packet/slot accesses) of the
unit's slot are loaded into v[84:99] with global_load_dwordx4.  The loader's
pointer-kind analysis gives every packet / slot access at a constant offset a
*staged* handler (resolved per launch, when the batch head is known): its
dword index, bit shift, byte mask and dirty-chunk bits are precomputed in the
FInsn, so the access is one or two index-mode moves.  Generic loads/stores
whose address falls inside the window at a wave-uniform offset are served
from the same VGPRs (v_alignbit / v_bfi).  Dirty 16-byte chunks are written
back (global_store_dwordx4) before any exit and before any other access that
overlaps the window (which also ends staging for the unit).

Map-bound handlers.  lddw of a map fd is bound at load time (as the kernel
binds BPF_PSEUDO_MAP_FD): an ARRAY lookup with a constant map and a stack key
is a bounds compare and one multiply-add; loads/stores/counters through a
non-null map-value pointer need no window check; a fused counter on a
constant map-value address needs no address uniformity test.

The handlers cover ALU64/ALU32 (reg and imm), byte swaps, loads/stores of
every size with the batch/arena/LDS window check, lddw, ja, every
conditional jump (uniform outcome, or split into lane groups), array / hash
lookups, atomics add/or/and/xor (+fetch), fused counters and exit.  Anything
else (other helpers, div/mod, cmpxchg/xchg, an access failing the window
check) leaves the block at that pc, and the C++ interpreter executes that one
instruction (interp.hip, run_loop<true, true>).

Fixed registers (declared as clobbers; the compiler keeps nothing live in
them across the block).  The handlers are written against the numbering
below; main() relocates every VGPR by +26 to the top of a 128-register
budget (v40..v101 -> v66..v127):
  s[40:47] W   current FInsn: w0 handler offset, w1 flags | next handler offset << 8, w[2:3] imm64 or off64
               (staged: w2 dword index, w3 bit shift), w4 dst*2 (staged
               stores: dirty-chunk bits; lookups: max_entries), w5 src*2
               (staged imm stores: the imm; lookups: value size), w6 jump
               target IP / static offset / continuation IP, w7 imm32 (ST, RMW)
               or byte mask (staged stores)
  s48 IP (byte offset of the current FInsn from PROG)   s49 scratch
  s[50:51] TB  handler base + 8 (divergent: + 0)   s[52:53] T scratch / target
  s[54:55], s[56:57], s[60:61] masks             s[58:59] saved exec
  s[62:63] A0 (wave-uniform address)             s[64:65] V0 (uniform value)
  s[66:67] TOT (wave total)                      s68 exit reason
  s69/s70/s71 scratch                            s[72:75] DMap words 0-3
  s[76:77] DMap data pointer                     s[78:79] PROG (FInsn base)
  s80 S (staged bytes; 0 = staging off)  s81 0   s[82:83] O (uniform offset)
  s84 dirty 16-B chunk mask                      s85 scratch
  s86/s87/s93, s[88:89]/s[90:91]/s[94:95], s92  pending lane groups
               (divergence): IPs, lane masks, count
  v40 lane's R[0] LDS address  v41, v[42:43] scratch
  v[44:45] X  v[46:47] Y  v[48:49] Z (address)  v[50:51] E (address end)
  v[52:53] slot address (staging base)           v[54:55] O (per-lane offset)
  v56..v59 scratch (hash probing)                v[60:81] r0..r10
  v[84:99] staged bytes
Loop-invariant inputs (window bounds, apertures, step limit, map table,
output addresses) and the per-wave counter cache are asm operands, so they
stay in the registers the compiler already holds them in.

Exit reasons (s68 -> why): 0 run the instruction at pc in C++, 1 step limit
crossed at a taken jump, 2 every live lane executed exit (r0 stored), 3 the
wave is split into lane groups: lpc holds each lane's pc for the C++
divergent loop.  aliveout = the lanes that have not exited.
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# handler entries aligned to 2^HANDLER_ALIGN bytes (0: packed); 64-B entries
# measured 0.4406 -> 0.4366 ms on the headline (same box, best of 4)
HANDLER_ALIGN = int(os.environ.get("BPFTIME_AMD_HANDLER_ALIGN", "6"))
# cache policy of the unit-slot staging loads and write-backs (" nt": the
# streamed slots as non-temporal, so they do not push hash tables, indexes
# and tail-call frames out of the XCD's L2; "" default policy)
SLOT_POLICY = os.environ.get("BPFTIME_AMD_GEN_SLOT_POLICY", "")
SLOT_STORE_POLICY = os.environ.get("BPFTIME_AMD_GEN_SLOT_STORE_POLICY", "")

ALU_OPS = ["ADD", "SUB", "MUL", "OR", "AND", "XOR", "MOV", "LSH", "RSH", "ARSH"]
JCC = ["EQ", "GT", "GE", "SET", "NE", "SGT", "SGE", "LT", "LE", "SLT", "SLE"]
CMP64 = {"EQ": "eq_u64", "GT": "gt_u64", "GE": "ge_u64", "NE": "ne_u64", "SGT": "gt_i64",
         "SGE": "ge_i64", "LT": "lt_u64", "LE": "le_u64", "SLT": "lt_i64", "SLE": "le_i64"}
CMP32 = {k: v.replace("64", "32") for k, v in CMP64.items()}
R0 = 60        # first VGPR of the eBPF register file
STG = 84       # first VGPR of the staged bytes
NREG = 11
INSN = 32      # FInsn bytes
# pending lane groups (divergence): IPs, lane masks, capacity
PIP = ["s86", "s87", "s93"]
PM = ["s[88:89]", "s[90:91]", "s[94:95]"]
KP = 3
WAYS = 8  # combining-table associativity
COMB_ROW = 144  # bytes per set of delta granules (common.hpp kCombRowBytes)
MISS_PARTS = 256  # miss-log partitions (common.hpp kMissParts)
RB_TENV = 64 + 4 * MISS_PARTS  # the block's ring staging slots in the launch constants (common.hpp kTenvRb)
LF_TENV = RB_TENV + 16  # the LDS tail-call frames' offset and shape (common.hpp kTenvLf)
TENV = LF_TENV + 16  # launch constants + miss counters + ring slots + LDS frames below the combining table (common.hpp kTenvBytes)


def _common_const(name):
    """A constexpr of common.hpp (kept in one place)."""
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "common.hpp")) as f:
        m = re.search(r"constexpr uint32_t %s = (\d+);" % name, f.read())
    return int(m.group(1))


RB_STAGE_REC = _common_const("kRbStageRec")  # ring staging budget per block
# hash-lookup cache: w4 of a FW_LCACHE lookup = its 2-way set count (common.hpp
# lcache_bytes: the ways' 16-B keys, then their u32 entries)

# staged (link-resolved) packet / slot accesses
STAGED_LD = ["LDXS1", "LDXS2", "LDXS4", "LDXS2X", "LDXS4X", "LDXS8A", "LDXS8U"]
STAGED_ST = ["STXS1", "STXS2", "STXS4", "STXS8", "STS1", "STS2", "STS4", "STS8"]


def handler_ids():
    ids = ["SLOW"]
    for w in ("64", "32"):
        for op in ALU_OPS:
            for k in ("R", "I"):
                ids.append(f"A{w}_{op}_{k}")
        ids.append(f"A{w}_NEG")
    ids += ["LE16", "LE32", "BE16", "BE32", "BE64", "NOP", "LEA"]
    for sz in (1, 2, 4, 8):
        ids += [f"LDX{sz}", f"STX{sz}", f"ST{sz}"]
    for sz in (1, 2, 4, 8):
        ids += [f"LDX{sz}_STK", f"STX{sz}_STK", f"ST{sz}_STK"]
    for sz in (1, 2, 4, 8):
        ids += [f"LDX{sz}_MV", f"STX{sz}_MV"]
    ids += STAGED_LD + STAGED_ST
    ids += ["LDX_CTXDATA", "LDX_CTXEND"]
    for sz in (4, 8):
        for op in ("ADD", "OR", "AND", "XOR"):
            ids += [f"ATOM{sz}_{op}", f"ATOM{sz}_{op}_F"]
        ids += [f"ATOMMV{sz}_ADD"]
    ids += ["ATOMMV8_ADD2"]
    ids += ["LDDW", "JA", "CALL_LOOKUP", "CALL_LOOKUP_STK", "CALL_LOOKUP_AK", "CALL_RBOUT", "EXIT"]
    for sz in (4, 8):
        for k in ("R", "I"):
            ids += [f"RMW{sz}_{k}", f"RMWMV{sz}_{k}", f"RMWK{sz}_{k}", f"RMWD{sz}_{k}"]
        ids += [f"ATOMD{sz}"]
    for w in ("64", "32"):
        for cc in JCC:
            for k in ("R", "I"):
                ids.append(f"J{w}_{cc}_{k}")
    ids += ["TAIL", "TRET", "CALL_PID", "KLDX"]  # rare / new: after the hot handlers
    # a map lookup with its argument set-up (lddw r1 = map; r2 = r10 + k;
    # call 1) as one dispatch (loader.cpp fuse_pairs)
    ids += ["CALL_LOOKUP_STK3", "CALL_LOOKUP_AK3"]
    for sz in (1, 2, 4, 8):  # the lane's own LDS XDP ctx at a static offset
        ids += [f"LDX{sz}_CTX", f"STX{sz}_CTX", f"ST{sz}_CTX"]
    ids += ["CALL_REC"]  # thread-ordered dispatch: the caller / clock beside the ctx copy
    ids += ["CALL_UPDATE_STK"]  # HASH update of a key every lane finds, key and value on the stack
    return ids


def L(name):
    return f".Lf%=_{name}"


class Gen:
    def __init__(self, greg=False):
        """greg: r0..r10's spill copy lives in global memory (%[rgb] + v40 +
        r * 2048, interp.hip k_interp<.., G = true>) and the lane's LDS column
        holds only its dummy and tail-call depth slots."""
        self.out = []
        self.uid = 0
        self.greg = greg
        self.depth_off = 2048 if greg else 12 * 2048  # the lane's tail-call depth slot
        self.span = 1  # FInsn slots a sequential next_seq steps over (fused lookups: 5)

    def e(self, *lines):
        self.out.extend(lines)

    def label(self, stem):
        self.uid += 1
        return L(f"{stem}{self.uid}")

    # ---- dispatch ----
    def dispatch(self):
        """IP is the byte offset of the next FInsn: fetch it and jump to its
        handler through the table."""
        self.e("s_load_dwordx8 s[40:47], s[78:79], s48",
               "s_waitcnt lgkmcnt(0)",
               "s_add_u32 s52, s50, s40",
               "s_addc_u32 s53, s51, 0",
               "s_setpc_b64 s[52:53]")

    def next_seq(self, slots=None):
        """Fall through: the handler offset of the next FInsn is w1 >> 8 of
        this one (link_fast), so the jump does not wait for the fetch; the
        handler waits for it on entry (lgkmcnt), overlapping the scalar load
        with the two control transfers."""
        slots = self.span if slots is None else slots
        self.e(f"s_add_u32 s48, s48, {INSN * slots}",
               "s_lshr_b32 s52, s41, 8",
               "s_load_dwordx8 s[40:47], s[78:79], s48",
               "s_add_u32 s52, s50, s52",
               "s_addc_u32 s53, s51, 0",
               "s_setpc_b64 s[52:53]")

    def jump_taken(self, hsrc):
        """IP = target; a taken jump is the only way back, so the step limit
        is enforced here.  The target's handler offset is in this FInsn
        (`hsrc`: w2 for JA and register jumps, w5 for immediate ones;
        vm_api.cpp Image::linked), so the jump does not wait for the
        target's fetch: the handler waits for it on entry, as after
        next_seq."""
        self.e("s_mov_b32 s48, s46",
               "s_add_u32 %[steps], %[steps], 1",
               "s_cmp_gt_u32 %[steps], %[limit]", f"s_cbranch_scc1 {L('steps')}",
               f"s_mov_b32 s52, {hsrc}",
               "s_load_dwordx8 s[40:47], s[78:79], s48",
               "s_add_u32 s52, s50, s52",
               "s_addc_u32 s53, s51, 0",
               "s_setpc_b64 s[52:53]")

    # ---- register file (VGPRs, indexed by a wave-uniform SGPR) ----
    def idx(self, sreg, modes):
        self.e(f"s_set_gpr_idx_on {sreg}, gpr_idx({modes})")

    def idx_off(self):
        self.e("s_set_gpr_idx_off")

    def rd(self, sidx, v):
        """v[v:v+1] = r[sidx / 2]"""
        self.idx(sidx, "SRC0")
        self.e(f"v_mov_b32 v{v}, v{R0}", f"v_mov_b32 v{v + 1}, v{R0 + 1}")
        self.idx_off()

    def rd_lo(self, sidx, v):
        """v[v] = low half of r[sidx / 2]"""
        self.idx(sidx, "SRC0")
        self.e(f"v_mov_b32 v{v}, v{R0}")
        self.idx_off()

    def wr(self, sidx, v, hi=None):
        """r[sidx / 2] = v[v:v+1] (hi: another source for the upper half)"""
        self.idx(sidx, "DST")
        self.e(f"v_mov_b32 v{R0}, v{v}", f"v_mov_b32 v{R0 + 1}, {hi if hi is not None else 'v%d' % (v + 1)}")
        self.idx_off()

    def rd_fixed(self, r, v):
        self.e(f"v_mov_b32 v{v}, v{R0 + 2 * r}", f"v_mov_b32 v{v + 1}, v{R0 + 2 * r + 1}")

    def imm_y(self):     # Y = imm64 (sign-extended by the loader)
        self.e("v_mov_b32 v46, s42", "v_mov_b32 v47, s43")

    def imm32_x(self):   # X = imm32 (w7) sign-extended to 64 bits
        self.e("v_mov_b32 v44, s47", "v_ashrrev_i32 v45, 31, v44")

    # ---- memory ----
    def check(self, sz):
        """Every live lane's [Z, Z+sz) inside the batch window, the map arena,
        or the LDS / scratch aperture; else leave for the C++ path (which
        fails the offending lanes)."""
        self.e(f"v_lshl_add_u64 v[50:51], v[48:49], 0, {sz}",
               "v_cmp_le_u64 s[54:55], %[dlo], v[48:49]",
               "v_cmp_ge_u64 s[56:57], %[dhi], v[50:51]",
               "s_and_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_le_u64 s[56:57], %[alo], v[48:49]",
               "v_cmp_ge_u64 s[60:61], %[ahi], v[50:51]",
               "s_and_b64 s[56:57], s[56:57], s[60:61]",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_eq_u32 s[56:57], %[shi], v49",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_eq_u32 s[56:57], %[phi], v49",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "s_andn2_b64 s[54:55], exec, s[54:55]",
               f"s_cbranch_scc1 {L('slow')}")

    def check_global(self, sz):
        """Every live lane's [Z, Z+sz) inside the batch window or the map
        arena and not in the LDS / scratch apertures (global atomics need a
        global address even when window checks are off); else leave."""
        self.e(f"v_lshl_add_u64 v[50:51], v[48:49], 0, {sz}",
               "v_cmp_le_u64 s[54:55], %[dlo], v[48:49]",
               "v_cmp_ge_u64 s[56:57], %[dhi], v[50:51]",
               "s_and_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_le_u64 s[56:57], %[alo], v[48:49]",
               "v_cmp_ge_u64 s[60:61], %[ahi], v[50:51]",
               "s_and_b64 s[56:57], s[56:57], s[60:61]",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_ne_u32 s[56:57], %[shi], v49",
               "s_and_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_ne_u32 s[56:57], %[phi], v49",
               "s_and_b64 s[54:55], s[54:55], s[56:57]",
               "s_andn2_b64 s[54:55], exec, s[54:55]",
               f"s_cbranch_scc1 {L('slow')}")

    def comb_add(self, sz, direct_only=False, pair=False):
        """Per-lane add of Y (v46, v[46:47] for 8 B) at the global address Z
        through the workgroup's LDS combining table (interp.hip: %[combn] u32
        tags, then a row of eight 16-byte delta granules per set, padded to
        COMB_ROW bytes so the sets' first ways spread over the banks
        (common.hpp kCombRowBytes), flushed when the block
        ends; the tags of ways 0-3 of every set, [set][4], then those of ways
        4-7, so a set's first four tags are one 16-byte slot and sets spread
        over all sixteen slots of a bank row, common.hpp comb_tag_pos): Zipf-hot counters cost an LDS add instead of a same-address
        device atomic per lane (those serialize at the memory side, ~12 ns
        each).  An entry stands for the 16-byte granule of the map arena
        holding the counter (for fused pairs: the 16 bytes at the pair's
        8-byte aligned address): tag = the granule's arena offset | 2 |
        (4-byte ? 1 : 0); its deltas are two u64 (8-byte counters at +0 / +8)
        or four u32 (4-byte counters), so the {packets, bytes} pair of a flow
        value shares one entry.  (A counter may have deltas in two entries;
        both reach it at the flush.)  The table is 8-way set associative, any
        number of sets (multiply-shift index): a lane reads its set's eight
        tags (three ds_reads), adds to the way holding its
        granule (a tag never changes once set: no atomic claim), else claims
        an empty way with a compare-and-swap (a lane that loses the race to
        another granule re-reads its set once), else adds to memory directly;
        so do misaligned lanes and counters outside the arena.  Lanes sharing
        a counter are serialized by the LDS itself.  pair: also Y2 (v[44:45])
        at Z + 8 (fused atomic pairs).  direct_only: every
        lane adds to memory now (FW_NODEFER counters)."""
        glob_add = ["global_atomic_add_x2 v[48:49], v[46:47], off" if sz == 8
                    else "global_atomic_add v[48:49], v46, off"]
        if pair:
            glob_add.append("global_atomic_add_x2 v[48:49], v[44:45], off offset:8")
        if direct_only:
            self.e(*glob_add)
            return
        done, direct, retry = self.label("cd"), self.label("cx"), self.label("cr")
        miss, lost, noclaim = self.label("cm"), self.label("cl"), self.label("cnc")

        def add(va):
            if sz == 8:
                self.e(f"ds_add_u64 {va}, v[46:47]")
                if pair:
                    self.e(f"ds_add_u64 {va}, v[44:45] offset:8")
            else:
                self.e(f"ds_add_u32 {va}, v46")
        self.e("s_mov_b64 s[60:61], exec", "s_mov_b64 s[54:55], 0",
               "s_cmp_eq_u32 %[combn], 0", f"s_cbranch_scc1 {direct}",
               f"v_and_b32 v41, {sz - 1}, v48", "v_cmp_eq_u32 vcc, 0, v41",   # aligned lanes
               "s_and_b64 exec, exec, vcc", f"s_cbranch_execz {direct}",
               "s_mov_b64 s[72:73], %[alo]",
               "v_mov_b32 v55, s73",
               "v_subrev_co_u32 v54, vcc, s72, v48", "v_subb_co_u32 v55, vcc, v49, v55, vcc",
               "v_cmp_eq_u32 vcc, 0, v55",                                       # inside the arena's 4 GiB
               "s_and_b64 exec, exec, vcc", f"s_cbranch_execz {direct}",
               # the granule: 16-byte aligned for single counters (byte offset
               # v43), the pair's own 8-byte aligned address for pairs
               "v_mov_b32 v43, 0" if pair else "v_and_b32 v43, 15, v54",
               f"v_and_b32 v54, {-8 if pair else -16}, v54",
               f"v_or_b32 v54, {3 if sz == 4 else 2}, v54",                      # tag
               "v_lshrrev_b32 v41, 4, v54", "s_mov_b32 s69, 0x9e3779b1", "v_mul_lo_u32 v41, v41, s69",
               f"s_lshr_b32 s69, %[combn], {WAYS.bit_length() - 1}",             # sets (any count)
               "v_mul_hi_u32 v41, v41, s69",                                     # the set: multiply-shift
               f"v_mul_u32_u24 v55, {COMB_ROW}, v41",                             # its first way's delta
               "v_lshlrev_b32 v41, 4, v41",
               "v_add_u32 v41, %[comb], v41",                                   # ways 0-3's tags
               "s_lshl_b32 s70, %[combn], 2", "s_add_u32 s70, s70, %[comb]",
               "v_add3_u32 v55, s70, v55, v43",                                 # way 0's delta + byte
               "s_lshl_b32 s71, %[combn], 1",                                   # ways 4-7's tags: + sets * 16
               "s_sub_u32 s69, s71, 16",
               "s_mov_b32 s85, 0",
               f"{retry}:",
               "s_mov_b64 s[62:63], exec",                                       # lanes of this pass
               "v_add_u32 v42, s71, v41",
               "ds_read_b128 v[56:59], v41",
               "ds_read_b64 v[82:83], v42",
               "ds_read_b64 v[50:51], v42 offset:8",
               "s_waitcnt lgkmcnt(0)",
               "v_mov_b32 v42, -1")
        tags = ["v56", "v57", "v58", "v59", "v82", "v83", "v50", "v51"]
        for k in range(WAYS - 1, -1, -1):                                        # the granule's way
            self.e(f"v_cmp_eq_u32 vcc, v54, {tags[k]}", f"v_cndmask_b32_e64 v42, v42, {k}, vcc")
        self.e("v_cmp_ne_u32 s[56:57], -1, v42", "s_and_b64 exec, s[62:63], s[56:57]",
               f"s_cbranch_execz {miss}",
               "v_lshl_add_u32 v43, v42, 4, v55")
        add("v43")
        self.e("s_or_b64 s[54:55], s[54:55], exec",
               f"{miss}:",
               "s_andn2_b64 exec, s[62:63], s[54:55]", f"s_cbranch_execz {noclaim}",
               "v_mov_b32 v42, -1")
        for k in range(WAYS - 1, -1, -1):                                        # first empty way
            self.e(f"v_cmp_eq_u32 vcc, 0, {tags[k]}", f"v_cndmask_b32_e64 v42, v42, {k}, vcc")
        self.e("v_cmp_ne_u32 s[56:57], -1, v42", "s_and_b64 exec, exec, s[56:57]",
               f"s_cbranch_execz {noclaim}",                                    # a full set: direct
               "v_lshl_add_u32 v43, v42, 2, v41",                                # way k's tag: k < 4
               "v_cmp_le_u32 vcc, 4, v42", "v_mov_b32 v50, s69",
               "v_cndmask_b32 v50, 0, v50, vcc", "v_add_u32 v43, v43, v50",     # ... else + sets * 16 - 16
               "v_mov_b32 v50, 0",
               "ds_cmpst_rtn_b32 v51, v43, v50, v54",
               "s_waitcnt lgkmcnt(0)",
               "v_cmp_eq_u32 s[56:57], 0, v51", "v_cmp_eq_u32 vcc, v54, v51",
               "s_or_b64 s[56:57], s[56:57], vcc",                              # claimed (or claimed for us)
               "s_and_b64 s[64:65], exec, s[56:57]",
               "s_andn2_b64 s[66:67], exec, s[56:57]",                           # lost to another granule
               "s_mov_b64 exec, s[64:65]", f"s_cbranch_execz {lost}",
               "v_lshl_add_u32 v43, v42, 4, v55")
        add("v43")
        self.e("s_or_b64 s[54:55], s[54:55], exec",
               f"{lost}:",
               "s_cmp_eq_u64 s[66:67], 0", f"s_cbranch_scc1 {noclaim}",
               "s_add_u32 s85, s85, 1", "s_cmp_gt_u32 s85, 1", f"s_cbranch_scc1 {noclaim}",
               "s_mov_b64 exec, s[66:67]", f"s_branch {retry}",
               f"{noclaim}:")
        self.e(f"{direct}:",
               "s_andn2_b64 exec, s[60:61], s[54:55]", f"s_cbranch_execz {done}",
               "s_bitcmp1_b32 %[oflags], 2", f"s_cbranch_scc1 {done}")         # (BPFTIME_AMD_DBG 128: timing only)
        self.miss_log(sz, pair, done)
        self.e(*glob_add)
        self.e(f"{done}:", "s_mov_b64 exec, s[60:61]")

    def miss_log(self, sz, pair, done):
        """exec = lanes whose add found no table entry: append their {tag,
        delta} records (two per lane: the pair's second counter, or an empty
        record) to the block's miss-log region (tenv[5], 0 = none; tenv[6] =
        records per partition) in the partition of their address, claimed
        with an LDS counter per partition (common.hpp kMissParts,
        interp.hip k_miss_merge).  Lanes whose partition is full, or that are
        misaligned, are left in exec for a direct add."""
        atom, back = self.label("mla"), self.label("mlb")
        self.e(f"s_sub_u32 s69, %[comb], {TENV - 40}", "v_mov_b32 v41, s69",
               "ds_read_b64 v[50:51], v41", "ds_read_b32 v56, v41 offset:8",
               "s_waitcnt lgkmcnt(0)",
               "v_readfirstlane_b32 s52, v50", "v_readfirstlane_b32 s53, v51", "v_readfirstlane_b32 s71, v56",
               "s_cmp_eq_u64 s[52:53], 0", f"s_cbranch_scc1 {atom}",
               "s_mov_b64 s[62:63], exec",                                       # the direct lanes
               f"v_and_b32 v41, {sz - 1}, v48", "v_cmp_eq_u32 vcc, 0, v41",
               "s_and_b64 exec, exec, vcc", f"s_cbranch_execz {back}",
               "v_lshrrev_b32 v41, 3, v48", "s_mov_b32 s69, 0x9e3779b1", "v_mul_lo_u32 v41, v41, s69",
               f"v_lshrrev_b32 v41, {32 - (MISS_PARTS.bit_length() - 1)}, v41",   # the partition
               f"s_sub_u32 s69, %[comb], {TENV - 64}", "v_lshl_add_u32 v42, v41, 2, s69",
               "v_mov_b32 v43, 2",
               "ds_add_rtn_u32 v43, v42, v43",                                   # its slot (even)
               "s_waitcnt lgkmcnt(0)",
               "v_cmp_gt_u32 vcc, s71, v43", "s_and_b64 exec, exec, vcc", f"s_cbranch_execz {back}",
               "s_andn2_b64 s[62:63], s[62:63], exec",                           # logged: not direct
               "v_mad_u32_u24 v42, v41, s71, v43", "v_lshlrev_b32 v42, 4, v42",
               f"v_or_b32 v56, {1 if sz == 4 else 0}, v48", "v_mov_b32 v57, v49",
               "v_mov_b32 v58, v46", "v_mov_b32 v59, v47" if sz == 8 else "v_mov_b32 v59, 0",
               "global_store_dwordx4 v42, v[56:59], s[52:53]",
               # (a store of more than 8 bytes reads its data registers after
               # issue: a VALU write of them needs a wait state in between)
               "s_nop 1")
        if pair:
            self.e("v_add_co_u32 v56, vcc, 8, v48", "v_addc_co_u32 v57, vcc, 0, v49, vcc",
                   "v_mov_b32 v58, v44", "v_mov_b32 v59, v45")
        else:
            self.e("v_mov_b32 v56, 0", "v_mov_b32 v57, 0", "v_mov_b32 v58, 0", "v_mov_b32 v59, 0")
        self.e("global_store_dwordx4 v42, v[56:59], s[52:53] offset:16", "s_nop 1",
               f"{back}:",
               "s_mov_b64 exec, s[62:63]", f"s_cbranch_execz {done}",
               f"{atom}:")

    def atomic_pair(self):
        """Two fused BPF_ATOMIC adds without fetch (loader: same map-value
        base, 8-byte counters at off and off + 8, the second FInsn skipped):
        one combining-table probe for both (w5 / w7 = the two value
        registers times two)."""
        self.rd("s44", 48)
        self.rd("s45", 46)
        self.rd("s47", 44)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        self.comb_add(8, pair=True)
        self.next_seq(2)

    def comb_peel(self, sz, direct_only=False):
        """Per-lane adds of Y to addresses Z (exec = the adding lanes).  When
        every lane adds the same value (a counter += constant), lanes that
        share the first lane's address are folded into one add of
        popcount * value by that lane, up to four distinct addresses per
        wave (Zipf-hot keys put most of a wave on a few map values); when
        the values differ (a sum of latencies), the lanes sharing an address
        fold their values' sum the same way, summed lane by lane in SGPRs;
        the rest add lane by lane (comb_add).  Masks survive comb_add in
        lanes of v56."""
        loop, rest, out = self.label("pl"), self.label("pr"), self.label("po")
        dloop, dsum = self.label("pdl"), self.label("pds")
        self.e("v_writelane_b32 v56, exec_lo, 2", "v_writelane_b32 v56, exec_hi, 3",
               "v_readfirstlane_b32 s64, v46", "v_readfirstlane_b32 s65, v47",
               "v_cmp_ne_u64 s[54:55], s[64:65], v[46:47]",
               "s_mov_b32 s85, 0",
               "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {dloop}",      # values differ
               f"{loop}:",
               "s_ff1_i32_b64 s69, exec",
               "v_readlane_b32 s62, v48, s69", "v_readlane_b32 s63, v49, s69",
               "v_cmp_eq_u64 s[54:55], s[62:63], v[48:49]",
               "s_bcnt1_i32_b64 s70, s[54:55]",
               "s_cmp_lt_u32 s70, 2", f"s_cbranch_scc1 {rest}",             # no sharing left
               "s_andn2_b64 s[56:57], exec, s[54:55]",
               "v_writelane_b32 v56, s56, 0", "v_writelane_b32 v56, s57, 1",
               "s_mul_i32 s66, s64, s70", "s_mul_hi_u32 s67, s64, s70",
               "s_mul_i32 s71, s65, s70", "s_add_u32 s67, s67, s71",
               "s_lshl_b64 exec, 1, s69",                                   # the first lane adds for all
               "v_mov_b32 v46, s66", "v_mov_b32 v47, s67")
        self.comb_add(sz, direct_only)
        self.e("v_readlane_b32 s56, v56, 0", "v_readlane_b32 s57, v56, 1",
               "s_mov_b64 exec, s[56:57]",
               f"s_cbranch_execz {out}",
               "s_add_u32 s85, s85, 1", "s_cmp_lt_u32 s85, 4", f"s_cbranch_scc1 {loop}",
               f"s_branch {rest}")
        # values differ: the first lane's address group adds the sum of its
        # lanes' values (s[66:67], a scalar loop over the group), up to four
        # groups; groups of one lane end the folding
        self.e(f"{dloop}:",
               "s_ff1_i32_b64 s69, exec",
               "v_readlane_b32 s62, v48, s69", "v_readlane_b32 s63, v49, s69",
               "v_cmp_eq_u64 s[54:55], s[62:63], v[48:49]",
               "s_bcnt1_i32_b64 s70, s[54:55]",
               "s_cmp_lt_u32 s70, 2", f"s_cbranch_scc1 {rest}",             # no sharing left
               "s_andn2_b64 s[56:57], exec, s[54:55]",
               "v_writelane_b32 v56, s56, 0", "v_writelane_b32 v56, s57, 1",
               "s_mov_b32 s66, 0", "s_mov_b32 s67, 0",
               f"{dsum}:",
               "s_ff1_i32_b64 s70, s[54:55]",
               "v_readlane_b32 s64, v46, s70", "v_readlane_b32 s65, v47, s70",
               "s_add_u32 s66, s66, s64", "s_addc_u32 s67, s67, s65",
               "s_bitset0_b64 s[54:55], s70",
               "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {dsum}",
               "s_lshl_b64 exec, 1, s69",                                   # the first lane adds for all
               "v_mov_b32 v46, s66", "v_mov_b32 v47, s67")
        self.comb_add(sz, direct_only)
        self.e("v_readlane_b32 s56, v56, 0", "v_readlane_b32 s57, v56, 1",
               "s_mov_b64 exec, s[56:57]",
               f"s_cbranch_execz {out}",
               "s_add_u32 s85, s85, 1", "s_cmp_lt_u32 s85, 4", f"s_cbranch_scc1 {dloop}",
               f"{rest}:")
        self.comb_add(sz, direct_only)
        self.e(f"{out}:", "v_readlane_b32 s56, v56, 2", "v_readlane_b32 s57, v56, 3",
               "s_mov_b64 exec, s[56:57]")

    def flush(self, clear=True):
        """Write dirty staged chunks back to the slots of the exec lanes."""
        for c in range(4):
            skip = self.label("fl")
            self.e(f"s_bitcmp1_b32 s84, {c}", f"s_cbranch_scc0 {skip}",
                   f"global_store_dwordx4 v[52:53], v[{STG + 4 * c}:{STG + 4 * c + 3}], off offset:{16 * c}"
                   + SLOT_STORE_POLICY,
                   f"{skip}:")
        if clear:
            self.e("s_mov_b32 s84, 0")

    def union_exec(self):
        """exec |= the masks of the pending lane groups (divergence)."""
        for i in range(KP):
            self.e(f"s_cmp_ge_u32 s92, {i + 1}", f"s_cselect_b64 s[56:57], {PM[i]}, 0",
                   "s_or_b64 exec, exec, s[56:57]")

    def flush_all(self):
        """Write back the dirty chunks of every live lane, pending groups
        included (staging is about to end for the whole wave)."""
        self.e("s_mov_b64 s[60:61], exec")
        self.union_exec()
        self.flush()
        self.e("s_mov_b64 exec, s[60:61]")

    def staged_or(self, sz, on_staged, on_global):
        """Z is the access address.  If staging is on and every live lane
        accesses [Z, Z+sz) at the same offset O inside its staged window,
        continue at `on_staged` with s82 = O.  Otherwise, if any lane's access
        overlaps its window, write back dirty chunks and end staging; then
        continue at `on_global`."""
        conflict = self.label("cf")
        self.e("s_cmp_eq_u32 s80, 0", f"s_cbranch_scc1 {on_global}",
               "v_sub_co_u32 v54, vcc, v48, v52", "v_subb_co_u32 v55, vcc, v49, v53, vcc",
               "v_readfirstlane_b32 s82, v54", "v_readfirstlane_b32 s83, v55",
               "v_cmp_ne_u64 s[54:55], s[82:83], v[54:55]",
               "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {conflict}",
               f"s_add_u32 s69, s82, {sz}", "s_addc_u32 s70, s83, 0",
               "s_cmp_lg_u32 s70, 0", f"s_cbranch_scc1 {conflict}",
               "s_cmp_gt_u32 s69, s80", f"s_cbranch_scc0 {on_staged}",
               f"{conflict}:",
               # overlap per lane: O < S, or the access starts below the
               # window and reaches into it (-sz <= O < 0 as a signed value)
               "v_cmp_gt_u64 s[54:55], s[80:81], v[54:55]",
               f"v_cmp_le_i64 s[56:57], -{sz}, v[54:55]",
               "v_cmp_gt_i64 s[60:61], 0, v[54:55]",
               "s_and_b64 s[56:57], s[56:57], s[60:61]",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "s_and_b64 s[54:55], s[54:55], exec",
               "s_cmp_eq_u64 s[54:55], 0", f"s_cbranch_scc1 {on_global}")
        self.flush_all()
        self.e("s_waitcnt vmcnt(0)", "s_mov_b32 s80, 0", f"s_branch {on_global}")

    def staged_load(self, sz):
        """X = sz bytes at window offset s82 (zero-extended)."""
        self.e("s_waitcnt vmcnt(0)",                       # staging loads landed
               "s_lshr_b32 s70, s82, 2", "s_and_b32 s71, s82, 3", "s_lshl_b32 s71, s71, 3")
        self.idx("s70", "SRC0")
        self.e(f"v_mov_b32 v44, v{STG}", f"v_mov_b32 v45, v{STG + 1}", f"v_mov_b32 v46, v{STG + 2}")
        self.idx_off()
        self.e("v_alignbit_b32 v44, v45, v44, s71")
        if sz == 8:
            self.e("v_alignbit_b32 v45, v46, v45, s71")
        elif sz == 4:
            self.e("v_mov_b32 v45, 0")
        else:
            self.e(f"v_and_b32 v44, {'0xff' if sz == 1 else '0xffff'}, v44", "v_mov_b32 v45, 0")

    def staged_store(self, sz, on_unaligned):
        """Window offset s82 = X (low sz bytes).  Needs the access inside one
        dword (sz <= 2) or dword-aligned (sz 4, 8); else `on_unaligned`."""
        self.e("s_and_b32 s71, s82, 3")
        if sz >= 4:
            self.e("s_cmp_lg_u32 s71, 0", f"s_cbranch_scc1 {on_unaligned}")
        else:
            self.e(f"s_add_u32 s69, s71, {sz}", "s_cmp_gt_u32 s69, 4", f"s_cbranch_scc1 {on_unaligned}")
        self.e("s_waitcnt vmcnt(0)", "s_lshr_b32 s70, s82, 2")
        if sz == 8:
            self.idx("s70", "DST")
            self.e(f"v_mov_b32 v{STG}, v44", f"v_mov_b32 v{STG + 1}, v45")
            self.idx_off()
        elif sz == 4:
            self.idx("s70", "DST")
            self.e(f"v_mov_b32 v{STG}, v44")
            self.idx_off()
        else:
            self.e("s_lshl_b32 s71, s71, 3",
                   f"s_bfm_b32 s69, {8 * sz}, s71",
                   "v_lshlrev_b32 v44, s71, v44")
            self.idx("s70", "SRC0")
            self.e(f"v_mov_b32 v46, v{STG}")
            self.idx_off()
            self.e("v_bfi_b32 v46, s69, v44, v46")
            self.idx("s70", "DST")
            self.e(f"v_mov_b32 v{STG}, v46")
            self.idx_off()
        # dirty chunks: the 16-B chunks of the first and the last byte
        self.e("s_lshr_b32 s69, s82, 4", "s_lshl_b32 s69, 1, s69", "s_or_b32 s84, s84, s69",
               f"s_add_u32 s69, s82, {sz - 1}", "s_lshr_b32 s69, s69, 4", "s_lshl_b32 s69, 1, s69",
               "s_or_b32 s84, s84, s69")

    # ---- handlers ----
    # dst op= y with the VALU instruction itself in index mode: (y-is-register
    # body, y-is-imm body).  VOP2 encodings (_e32): one SGPR operand at most,
    # and src1 must be a VGPR, so the imm forms put the SGPR in src0 and index
    # src1; the carry chains take the imm's high half from a VGPR.
    INPLACE64 = {
        "ADD": (["v_add_co_u32_e32 v60, vcc, v60, v46", "v_addc_co_u32_e32 v61, vcc, v61, v47, vcc"],
                ["v_add_co_u32_e32 v60, vcc, s42, v60", "v_addc_co_u32_e32 v61, vcc, v47, v61, vcc"]),
        "SUB": (["v_sub_co_u32_e32 v60, vcc, v60, v46", "v_subb_co_u32_e32 v61, vcc, v61, v47, vcc"],
                ["v_subrev_co_u32_e32 v60, vcc, s42, v60", "v_subbrev_co_u32_e32 v61, vcc, v47, v61, vcc"]),
        "OR": (["v_or_b32_e32 v60, v60, v46", "v_or_b32_e32 v61, v61, v47"],
               ["v_or_b32_e32 v60, s42, v60", "v_or_b32_e32 v61, s43, v61"]),
        "AND": (["v_and_b32_e32 v60, v60, v46", "v_and_b32_e32 v61, v61, v47"],
                ["v_and_b32_e32 v60, s42, v60", "v_and_b32_e32 v61, s43, v61"]),
        "XOR": (["v_xor_b32_e32 v60, v60, v46", "v_xor_b32_e32 v61, v61, v47"],
                ["v_xor_b32_e32 v60, s42, v60", "v_xor_b32_e32 v61, s43, v61"]),
        "MOV": (["v_mov_b32_e32 v60, v46", "v_mov_b32_e32 v61, v47"],
                ["v_mov_b32_e32 v60, s42", "v_mov_b32_e32 v61, s43"]),
    }
    INPLACE32 = {
        "ADD": ("v_add_u32_e32 v60, v60, v46", "v_add_u32_e32 v60, s42, v60"),
        "SUB": ("v_sub_u32_e32 v60, v60, v46", "v_subrev_u32_e32 v60, s42, v60"),
        "OR": ("v_or_b32_e32 v60, v60, v46", "v_or_b32_e32 v60, s42, v60"),
        "AND": ("v_and_b32_e32 v60, v60, v46", "v_and_b32_e32 v60, s42, v60"),
        "XOR": ("v_xor_b32_e32 v60, v60, v46", "v_xor_b32_e32 v60, s42, v60"),
        "MOV": ("v_mov_b32_e32 v60, v46", "v_mov_b32_e32 v60, s42"),
        # shift amount in src0, the shifted register in src1 (& 31 in hardware)
        "LSH": ("v_lshlrev_b32_e32 v60, v46, v60", "v_lshlrev_b32_e32 v60, s42, v60"),
        "RSH": ("v_lshrrev_b32_e32 v60, v46, v60", "v_lshrrev_b32_e32 v60, s42, v60"),
        "ARSH": ("v_ashrrev_i32_e32 v60, v46, v60", "v_ashrrev_i32_e32 v60, s42, v60"),
    }

    def alu(self, w, op, k):
        if w == "64" and op in self.INPLACE64:
            body = self.INPLACE64[op][0 if k == "R" else 1]
            if k == "R":
                self.rd("s45", 46)
            elif op in ("ADD", "SUB"):
                self.e("v_mov_b32 v47, s43")
            mode = "DST" if op == "MOV" else ("SRC0,DST" if k == "R" else "SRC1,DST")
            self.idx("s44", mode)
            self.e(*body)
            self.idx_off()
            self.next_seq()
            return
        if w == "32" and op in self.INPLACE32:
            body = self.INPLACE32[op][0 if k == "R" else 1]
            if k == "R":
                self.rd_lo("s45", 46)
            if op == "MOV":
                mode = "DST"
            elif k == "R" and op not in ("LSH", "RSH", "ARSH"):
                mode = "SRC0,DST"
            else:
                mode = "SRC1,DST"
            self.idx("s44", mode)
            self.e(body, "v_mov_b32_e32 v61, 0")      # ALU32 zero-extends
            self.idx_off()
            self.next_seq()
            return
        # MUL and 64-bit shifts: X = r[dst], Y = src / imm, X op= Y, r[dst] = X
        self.rd("s44", 44)
        if k == "R":
            self.rd("s45", 46)
        else:
            self.imm_y()
        if w == "64":
            body = {
                "MUL": ["v_mul_lo_u32 v48, v44, v47", "v_mul_lo_u32 v49, v45, v46",
                        "v_mul_hi_u32 v50, v44, v46", "v_mul_lo_u32 v44, v44, v46",
                        "v_add3_u32 v45, v48, v49, v50"],
                "LSH": ["v_lshlrev_b64 v[44:45], v46, v[44:45]"],   # shift count & 63 in hardware
                "RSH": ["v_lshrrev_b64 v[44:45], v46, v[44:45]"],
                "ARSH": ["v_ashrrev_i64 v[44:45], v46, v[44:45]"],
            }[op]
        else:
            body = {"MUL": ["v_mul_lo_u32 v44, v44, v46"]}[op] + ["v_mov_b32 v45, 0"]
        self.e(*body)
        self.wr("s44", 44)
        self.next_seq()

    def lea(self):
        """Superinstruction (loader.cpp fuse_pairs): `mov64 dst, src; add64
        dst, imm` as one dispatch, r[dst] = r[src] + imm64 (w2:3); the pair's
        second FInsn is skipped."""
        self.rd("s45", 44)
        self.e("v_lshl_add_u64 v[44:45], v[44:45], 0, s[42:43]")
        self.wr("s44", 44)
        self.next_seq(2)

    def movi_prefix(self):
        """A `mov64 r, imm32` fused in front of this jump / exit (loader.cpp
        fuse_pairs: w1 FW_MOVI, bits 3..6 = r, w7 = the imm): execute it, then
        this instruction as the pair's second (IP one slot on)."""
        skip = self.label("mvi")
        self.e("s_bitcmp1_b32 s41, 2", f"s_cbranch_scc0 {skip}",
               "s_bfe_u32 s69, s41, 0x40003", "s_lshl_b32 s69, s69, 1",
               "s_ashr_i32 s70, s47, 31")
        self.idx("s69", "DST")
        self.e(f"v_mov_b32_e32 v{R0}, s47", f"v_mov_b32_e32 v{R0 + 1}, s70")
        self.idx_off()
        self.e(f"s_add_u32 s48, s48, {INSN}", f"{skip}:")

    def neg(self, w):
        self.idx("s44", "SRC1,DST")
        if w == "64":
            self.e("v_sub_co_u32_e32 v60, vcc, 0, v60", "v_subb_co_u32_e32 v61, vcc, 0, v61, vcc")
        else:
            self.e("v_sub_u32_e32 v60, 0, v60", "v_mov_b32_e32 v61, 0")
        self.idx_off()
        self.next_seq()

    def endian(self, name):
        self.rd("s44", 44)
        body = {
            "LE16": ["v_and_b32 v44, 0xffff, v44", "v_mov_b32 v45, 0"],
            "LE32": ["v_mov_b32 v45, 0"],
            "BE16": ["s_mov_b32 s69, 0x0c0c0001", "v_perm_b32 v44, 0, v44, s69", "v_mov_b32 v45, 0"],
            "BE32": ["s_mov_b32 s69, 0x00010203", "v_perm_b32 v44, 0, v44, s69", "v_mov_b32 v45, 0"],
            "BE64": ["s_mov_b32 s69, 0x00010203", "v_perm_b32 v48, 0, v45, s69",
                     "v_perm_b32 v45, 0, v44, s69", "v_mov_b32 v44, v48"],
        }[name]
        self.e(*body)
        self.wr("s44", 44)
        self.next_seq()

    LD = {1: "flat_load_ubyte v44, v[48:49]", 2: "flat_load_ushort v44, v[48:49]",
          4: "flat_load_dword v44, v[48:49]", 8: "flat_load_dwordx2 v[44:45], v[48:49]"}
    ST = {1: "flat_store_byte v[48:49], v44", 2: "flat_store_short v[48:49], v44",
          4: "flat_store_dword v[48:49], v44", 8: "flat_store_dwordx2 v[48:49], v[44:45]"}

    def ldx(self, sz):
        stg = self.label("ls")
        glb = L(f"ldx{sz}_glb")
        self.rd("s45", 48)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        self.staged_or(sz, stg, glb)
        self.e(f"{stg}:")
        self.staged_load(sz)
        self.wr("s44", 44)
        self.next_seq()
        self.e(f"{glb}:")                 # also the staged handlers' way out (staging off)
        self.check(sz)
        self.e(self.LD[sz])
        if sz < 8:
            self.e("v_mov_b32 v45, 0")
        self.e("s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.wr("s44", 44)
        self.next_seq()

    def store(self, sz, from_reg):
        stg, unal = self.label("ss"), self.label("su")
        glb = L(("stx" if from_reg else "st") + f"{sz}_glb")
        # Z = R[dst] + off ; X = value
        self.rd("s44", 48)
        if from_reg:
            self.rd("s45", 44)
        else:
            self.imm32_x()
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        self.staged_or(sz, stg, glb)
        self.e(f"{stg}:")
        self.staged_store(sz, unal)
        self.next_seq()
        # a staged store straddling dwords: write back, end staging, store to memory
        self.e(f"{unal}:")
        self.flush_all()
        self.e("s_waitcnt vmcnt(0)", "s_mov_b32 s80, 0")
        self.e(f"{glb}:")
        self.check(sz)
        self.e(self.ST[sz])
        self.next_seq()

    # ---- map values (loader: a non-null lookup result, access inside the
    # value): no window check, never inside the staged window
    def ldx_mv(self, sz):
        ld = {1: "global_load_ubyte v44, v[48:49], off", 2: "global_load_ushort v44, v[48:49], off",
              4: "global_load_dword v44, v[48:49], off", 8: "global_load_dwordx2 v[44:45], v[48:49], off"}[sz]
        self.rd("s45", 48)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]", ld)
        if sz < 8:
            self.e("v_mov_b32 v45, 0")
        self.e("s_waitcnt vmcnt(0)")
        self.wr("s44", 44)
        self.next_seq()

    def stx_mv(self, sz):
        st = {1: "global_store_byte v[48:49], v44, off", 2: "global_store_short v[48:49], v44, off",
              4: "global_store_dword v[48:49], v44, off", 8: "global_store_dwordx2 v[48:49], v[44:45], off"}[sz]
        self.rd("s44", 48)
        self.rd("s45", 44)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]", st)
        self.next_seq()

    # ---- stack (loader: r10 + constant, in the lane's LDS stack) ----
    def ldx_stk(self, sz, base="%[stklo]"):
        """dst = the sz bytes at static offset w6 from the stack top (base
        %[r1lo]: from the lane's own LDS XDP ctx, loader.cpp *_CTX)."""
        ds = {1: "ds_read_u8", 2: "ds_read_u16", 4: "ds_read_b32", 8: "ds_read_b64"}[sz]
        self.e(f"v_add_u32 v41, s46, {base}",
               f"{ds} {'v[44:45]' if sz == 8 else 'v44'}, v41",
               "s_waitcnt lgkmcnt(0)")
        self.wr("s44", 44, hi=None if sz == 8 else "0")
        self.next_seq()

    def store_stk(self, sz, from_reg, base="%[stklo]"):
        if from_reg:
            (self.rd if sz == 8 else self.rd_lo)("s45", 44)
        else:
            self.imm32_x()
        ds = {1: "ds_write_b8", 2: "ds_write_b16", 4: "ds_write_b32", 8: "ds_write_b64"}[sz]
        self.e(f"v_add_u32 v41, s46, {base}",
               f"{ds} v41, {'v[44:45]' if sz == 8 else 'v44'}")
        self.next_seq()

    # ---- staged packet / slot accesses (link-resolved: inside the window) ----
    def fallback_addr(self):
        """Z = slot + static slot offset (w6), for the generic handlers."""
        self.e("v_add_co_u32_e32 v48, vcc, s46, v52", "v_addc_co_u32_e32 v49, vcc, 0, v53, vcc")

    def ldxs(self, name):
        fb = self.label("lfb")
        sz = int(name[4])
        self.e("s_cmp_eq_u32 s80, 0", f"s_cbranch_scc1 {fb}", "s_waitcnt vmcnt(0)")
        self.idx("s42", "SRC0")
        n = {"LDXS1": 1, "LDXS2": 1, "LDXS4": 1, "LDXS2X": 2, "LDXS4X": 2, "LDXS8A": 2, "LDXS8U": 3}[name]
        for j in range(n):
            self.e(f"v_mov_b32 v{44 + j}, v{STG + j}")
        self.idx_off()
        body = {
            "LDXS1": ["v_bfe_u32 v44, v44, s43, 8"],
            "LDXS2": ["v_bfe_u32 v44, v44, s43, 16"],
            "LDXS4": [],
            "LDXS2X": ["v_alignbit_b32 v44, v45, v44, s43", "v_and_b32 v44, 0xffff, v44"],
            "LDXS4X": ["v_alignbit_b32 v44, v45, v44, s43"],
            "LDXS8A": [],
            "LDXS8U": ["v_alignbit_b32 v44, v45, v44, s43", "v_alignbit_b32 v45, v46, v45, s43"],
        }[name]
        self.e(*body)
        self.wr("s44", 44, hi=None if sz == 8 else "0")
        self.next_seq()
        self.e(f"{fb}:")
        self.fallback_addr()
        self.e(f"s_branch {L('ldx%d_glb' % sz)}")

    def stxs(self, name):
        imm = name.startswith("STS")
        sz = int(name[-1])
        fb = self.label("sfb")
        self.e("s_cmp_eq_u32 s80, 0", f"s_cbranch_scc1 {fb}", "s_waitcnt vmcnt(0)")
        if not imm:
            (self.rd if sz == 8 else self.rd_lo)("s45", 44)
        elif sz == 8:
            self.e("v_mov_b32 v44, s45", "v_ashrrev_i32 v45, 31, v44")
        elif sz == 4:
            self.e("v_mov_b32 v44, s45")
        else:
            self.e("s_lshl_b32 s69, s45, s43", "v_mov_b32 v44, s69")
        if sz <= 2:
            if not imm:
                self.e("v_lshlrev_b32 v44, s43, v44")
            self.idx("s42", "SRC0")
            self.e(f"v_mov_b32 v46, v{STG}")
            self.idx_off()
            self.e("v_bfi_b32 v46, s47, v44, v46")
            self.idx("s42", "DST")
            self.e(f"v_mov_b32 v{STG}, v46")
            self.idx_off()
        else:
            self.idx("s42", "DST")
            self.e(f"v_mov_b32 v{STG}, v44")
            if sz == 8:
                self.e(f"v_mov_b32 v{STG + 1}, v45")
            self.idx_off()
        self.e("s_or_b32 s84, s84, s44")
        self.next_seq()
        self.e(f"{fb}:")
        self.fallback_addr()
        if imm:
            self.e("v_mov_b32 v44, s45", "v_ashrrev_i32 v45, 31, v44")
        else:
            self.rd("s45", 44)
        self.e(f"s_branch {L(('st' if imm else 'stx') + '%d_glb' % sz)}")

    def ctx_field(self, end):
        """ctx->data = slot + head; ctx->data_end = slot + head + len."""
        if end:
            self.e("v_add_u32 v46, %[head], %[ulen]")
        self.idx("s44", "DST")
        if end:
            self.e("v_add_co_u32_e32 v60, vcc, v46, v52")
        else:
            self.e("v_add_co_u32_e32 v60, vcc, %[head], v52")
        self.e("v_addc_co_u32_e32 v61, vcc, 0, v53, vcc")
        self.idx_off()
        self.next_seq()

    def call_pid(self):
        """bpf_get_current_pid_tgid (bpf_helper.cpp:330-348) of a recorded
        syscall: r0 = the u64 at slot + w7 (link_fast: KParams pid_off, the
        caller's pid_tgid in the replay record), from the unit's staged
        bytes when the window holds it (w3 = 1, w2 = its dword index), else
        a load.  r1-r5 are left as they are, as the C++ tier's helper call
        leaves them."""
        glb = self.label("pidg")
        self.e("s_cmp_eq_u32 s80, 0", f"s_cbranch_scc1 {glb}",
               "s_cmp_eq_u32 s43, 0", f"s_cbranch_scc1 {glb}",
               "s_waitcnt vmcnt(0)")
        self.idx("s42", "SRC0")
        self.e(f"v_mov_b32 v44, v{STG}", f"v_mov_b32 v45, v{STG + 1}")
        self.idx_off()
        self.e(f"v_mov_b32 v{R0}, v44", f"v_mov_b32 v{R0 + 1}, v45")
        self.next_seq()
        self.e(f"{glb}:",
               "v_add_co_u32_e32 v48, vcc, s47, v52",
               "v_addc_co_u32_e32 v49, vcc, 0, v53, vcc",
               f"global_load_dwordx2 v[{R0}:{R0 + 1}], v[48:49], off",
               "s_waitcnt vmcnt(0)")
        self.next_seq()

    def call_rec(self):
        """bpf_get_current_pid_tgid / bpf_ktime_get_ns of a thread-ordered
        callback (interp.hip k_sys_seq, loader.cpp link_fast rec_helpers):
        r0 = the u64 at slot + w7, the caller or the recorded clock the
        kernel put beside the lane's LDS ctx copy (a flat load: the slot is
        that copy).  r1-r5 are left as they are, as the C++ tier's helper
        call leaves them."""
        self.e("v_add_co_u32_e32 v48, vcc, s47, v52",
               "v_addc_co_u32_e32 v49, vcc, 0, v53, vcc",
               f"flat_load_dwordx2 v[{R0}:{R0 + 1}], v[48:49]",
               "s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.next_seq()

    def ldxk(self):
        """dst = a load from a constant address nothing in the program
        writes (loader.cpp const_loads: inside an ARRAY map's storage, e.g.
        a .rodata value), through the scalar cache: w[2:3] the address
        rounded down to 4 bytes, w7 0 (8 bytes at a 4-aligned address) or
        width << 16 | bit offset (s_bfe_u64)."""
        k = self.label("ldxk")
        self.e("s_load_dwordx2 s[52:53], s[42:43], 0x0",
               "s_waitcnt lgkmcnt(0)",
               "s_cmp_eq_u32 s47, 0", f"s_cbranch_scc1 {k}",
               "s_bfe_u64 s[52:53], s[52:53], s47",
               f"{k}:")
        self.idx("s44", "DST")
        self.e(f"v_mov_b32_e32 v{R0}, s52", f"v_mov_b32_e32 v{R0 + 1}, s53")
        self.idx_off()
        self.next_seq()

    def lddw(self):
        self.idx("s44", "DST")
        self.e("v_mov_b32_e32 v60, s42", "v_mov_b32_e32 v61, s43")
        self.idx_off()
        self.next_seq(2)

    def jcc(self, w, cc, k):
        self.movi_prefix()
        (self.rd if w == "64" else self.rd_lo)("s44", 44)
        if k == "R":
            (self.rd if w == "64" else self.rd_lo)("s45", 46)
        y64 = "v[46:47]" if k == "R" else "s[42:43]"
        y32 = "v46" if k == "R" else "s42"
        if cc == "SET":
            if w == "64":
                if k == "R":
                    self.e("v_and_b32 v44, v44, v46", "v_and_b32 v45, v45, v47")
                else:
                    self.e("v_and_b32 v44, s42, v44", "v_and_b32 v45, s43, v45")
                self.e("v_or_b32 v44, v44, v45")
            else:
                self.e(f"v_and_b32 v44, {'v46' if k == 'R' else 's42'}, v44")
            self.e("v_cmp_ne_u32_e64 vcc, 0, v44")
        elif w == "64":
            self.e(f"v_cmp_{CMP64[cc]}_e64 vcc, v[44:45], {y64}")
        else:
            self.e(f"v_cmp_{CMP32[cc]}_e64 vcc, v44, {y32}")
        # v_cmp writes 0 for inactive lanes: none taken / all taken / split
        nt = self.label("nt")
        self.e(f"s_cbranch_vccz {nt}",
               "s_cmp_eq_u64 vcc, exec", f"s_cbranch_scc0 {L('split')}")
        self.jump_taken("s42" if k == "R" else "s45")
        self.e(f"{nt}:")
        self.next_seq()

    def uniform64(self, vpair, spair):
        """spair = lane-0 value of vpair; leave unless every live lane agrees."""
        lo, hi = vpair
        slo, shi_ = spair
        self.e(f"v_readfirstlane_b32 s{slo}, v{lo}", f"v_readfirstlane_b32 s{shi_}, v{hi}",
               f"v_cmp_ne_u64 s[54:55], s[{slo}:{shi_}], v[{lo}:{hi}]",
               "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {L('slow')}")

    def call_update_stk(self):
        """bpf_map_update_elem of a HASH map, key and value on the stack
        (loader.cpp: w6 / w2 their offsets from the stack top, w7 the value's
        dwords): when every lane finds its key (the lookup's probe), the
        value is overwritten in place and r0 = 0 (fix_hash_map.cpp:34-39:
        the flags are not looked at; dev_helpers.hpp helper_update).  A new
        key, an in-flight insert, and a wave with a lane whose lookup of a
        key just missed (entry bit 8: the lookup-or-init race rule, which
        the C++ helper keeps) leave for C++ before anything is written."""
        self.e("s_bitcmp1_b32 %[entry], 8", f"s_cbranch_scc1 {L('slow')}")
        self.call_lookup(stack_key=True, update=True)

    def update_tail(self):
        """r0 = the found element's value in every lane: the value's dwords
        from the stack over it, then r0 = 0."""
        loop = self.label("upd")
        self.e("v_add_u32 v41, s42, %[stklo]",                             # the value on the stack
               f"v_mov_b32 v48, v{R0}", f"v_mov_b32 v49, v{R0 + 1}",
               "s_mov_b32 s69, s47",
               f"{loop}:",
               "ds_read_b32 v44, v41", "s_waitcnt lgkmcnt(0)",
               "global_store_dword v[48:49], v44, off",
               "v_add_u32 v41, 4, v41",
               "v_add_co_u32 v48, vcc, 4, v48", "v_addc_co_u32 v49, vcc, 0, v49, vcc",
               "s_sub_u32 s69, s69, 1", "s_cmp_lg_u32 s69, 0", f"s_cbranch_scc1 {loop}",
               "s_waitcnt vmcnt(0)",
               f"v_mov_b32 v{R0}, 0", f"v_mov_b32 v{R0 + 1}, 0")

    def call_lookup(self, stack_key=False, update=False):
        """bpf_map_lookup_elem with a wave-uniform map fd.
        ARRAY (array_map.cpp:27-40): r0 = key < max_entries ? &data[key * vsz] : 0.
        HASH with its key on the stack (stack_key: the loader proved r2 =
        stack top + w6, 4-aligned): the bpftime_hash_map probe
        (bpftime_hash_map.hpp:40-47, 127-151) per lane; a wave whose lanes
        all hit stays here, any miss or in-flight insert leaves for the C++
        helper (which also records the miss for lookup_or_try_init).
        Other map types leave for C++."""
        stg, glb, got = self.label("ks"), self.label("kg"), self.label("kd")
        self.rd_fixed(1, 44)                      # r1 = fd
        self.rd_fixed(2, 48)                      # r2 = key pointer
        self.uniform64((44, 45), (62, 63))
        self.e("s_cmp_lg_u32 s63, 0", f"s_cbranch_scc1 {L('slow')}",
               "s_cmpk_ge_u32 s62, 0x400", f"s_cbranch_scc1 {L('slow')}",  # fd >= kMaxFds
               "s_lshl_b32 s85, s62, 6",
               "s_load_dwordx4 s[72:75], %[maps], s85",                      # type, ksz, vsz, max
               "s_add_u32 s85, s85, 16",
               "s_load_dwordx2 s[76:77], %[maps], s85")                     # data
        if stack_key:
            # a hash table's words and its key, in the same round trip
            # (hash_lookup; harmless reads for the other map types): the
            # lookup index at s[52:53], DMap words 4-11 at s[64:71], the
            # stack key's four dwords at v[44:47]
            self.e("s_add_u32 s69, s85, 40",
                   "s_load_dwordx2 s[52:53], %[maps], s69",
                   "s_load_dwordx8 s[64:71], %[maps], s85",
                   "v_add_u32 v41, s46, %[stklo]",
                   "ds_read_b32 v44, v41", "ds_read_b32 v45, v41 offset:4",
                   "ds_read_b32 v46, v41 offset:8", "ds_read_b32 v47, v41 offset:12")
        self.e("s_waitcnt lgkmcnt(0)")
        if update:
            self.e("s_cmp_lg_u32 s72, 1", f"s_cbranch_scc1 {L('slow')}")       # BPF_MAP_TYPE_HASH only
            self.hash_lookup(update=True)
            return
        if stack_key:
            hsh, lpm = self.label("hash"), self.label("lpm")
            self.e("s_cmp_eq_u32 s72, 1", f"s_cbranch_scc1 {hsh}",          # BPF_MAP_TYPE_HASH
                   "s_cmp_eq_u32 s72, 11", f"s_cbranch_scc1 {lpm}")         # BPF_MAP_TYPE_LPM_TRIE
        # ARRAY: element key; PERCPU_ARRAY (per_cpu_array_map.cpp:34-48):
        # element key * ncpu + this wave's virtual cpu (%[vcpu] = cpu | ncpu
        # << 16 when the wave's lanes share one, else ~0: C++)
        parr, arr = self.label("lpc"), self.label("lar")
        self.e("s_mov_b32 s70, 1", "s_mov_b32 s71, 0",
               "s_cmp_eq_u32 s72, 6", f"s_cbranch_scc1 {parr}",
               "s_cmp_lg_u32 s72, 2", f"s_cbranch_scc1 {L('slow')}",        # not BPF_MAP_TYPE_ARRAY
               f"s_branch {arr}",
               f"{parr}:",
               "s_add_u32 s85, s85, 28",
               "s_load_dword s70, %[maps], s85",                             # DMap ncpu
               "s_lshr_b32 s69, %[vcpu], 16",
               "s_waitcnt lgkmcnt(0)",
               "s_cmp_lg_u32 s69, s70", f"s_cbranch_scc1 {L('slow')}",
               "s_and_b32 s71, %[vcpu], 0xffff",
               f"{arr}:")
        if stack_key:
            self.e("v_add_u32 v41, s46, %[stklo]", "ds_read_b32 v46, v41", "s_waitcnt lgkmcnt(0)",
                   f"s_branch {got}")
        else:
            self.staged_or(4, stg, glb)
            self.e(f"{stg}:")
            self.staged_load(4)
            self.e("v_mov_b32 v46, v44", f"s_branch {got}")
            self.e(f"{glb}:")
            self.check(4)
            self.e("flat_load_dword v46, v[48:49]", "s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.e(f"{got}:",
               "v_cmp_gt_u32 s[54:55], s75, v46",                            # key < max_entries
               "v_mov_b32 v47, s74",
               "v_mul_lo_u32 v46, v46, s70", "v_add_u32 v46, s71, v46",
               "v_mad_u64_u32 v[50:51], s[56:57], v46, v47, s[76:77]",
               f"v_cndmask_b32 v{R0}, 0, v50, s[54:55]",
               f"v_cndmask_b32 v{R0 + 1}, 0, v51, s[54:55]")
        self.next_seq()
        if stack_key:
            self.e(f"{hsh}:")
            self.hash_lookup()
            self.e(f"{lpm}:")
            self.lpm_lookup()

    def lpm_lookup(self):
        """LPM_TRIE with a 4-byte (IPv4) key on the stack whose prefixlen is
        32 in every lane: the flat table (maps.cpp LpmTrie::flat, DMap.ix):
        e = t[top 24 address bits], e = group[e][low byte] when bit 31 is
        set; r0 = e ? &value of node e - 1 in the replica : 0 -- the node the
        trie walk (dev_helpers.hpp lpm_lookup) returns.  Other keys, and
        tries without the table, leave for C++.  s85 = fd * 64 + 16."""
        grp = self.label("lg")
        self.e("s_cmp_lg_u32 s73, 8", f"s_cbranch_scc1 {L('slow')}",        # key_size 4 + 4
               "s_add_u32 s69, s85, 16",
               "s_load_dwordx4 s[64:67], %[maps], s69",                      # slot_size, key_off, val_off, ncpu
               "s_add_u32 s69, s85, 40",
               "s_load_dwordx2 s[70:71], %[maps], s69",                      # ix = the flat table
               "v_add_u32 v41, s46, %[stklo]",
               "ds_read_b32 v44, v41", "ds_read_b32 v45, v41 offset:4",     # prefixlen, address bytes
               "s_waitcnt lgkmcnt(0)",
               "s_cmp_eq_u64 s[70:71], 0", f"s_cbranch_scc1 {L('slow')}",
               "v_cmp_ne_u32 s[54:55], 32, v44", "s_and_b64 s[54:55], s[54:55], exec",
               f"s_cbranch_scc1 {L('slow')}",                                # a lane's prefixlen != 32
               "s_mov_b32 s69, 0x10203",
               "v_perm_b32 v46, v45, v45, s69",                              # the address, big endian
               "v_lshrrev_b32 v47, 8, v46", "v_lshlrev_b32 v47, 2, v47",
               "global_load_dword v50, v47, s[70:71]",
               "s_waitcnt vmcnt(0)",
               "v_cmp_gt_i32 vcc, 0, v50", "s_and_b64 vcc, vcc, exec",       # bit 31: a /24 group
               f"s_cbranch_vccz {grp}",
               "s_mov_b64 s[56:57], exec", "s_mov_b64 exec, vcc",
               "v_and_b32 v51, 0x7fffffff, v50", "v_lshlrev_b32 v51, 8, v51",
               "v_and_b32 v42, 0xff, v46", "s_mov_b32 s69, 0x1000000", "v_add3_u32 v51, v51, v42, s69",
               "v_lshlrev_b32 v51, 2, v51",
               "global_load_dword v50, v51, s[70:71]",
               "s_waitcnt vmcnt(0)",
               "s_mov_b64 exec, s[56:57]",
               f"{grp}:",
               "v_cmp_ne_u32 s[54:55], 0, v50",
               "v_add_u32 v50, -1, v50",
               "v_mov_b32 v47, s64",
               "v_mad_u64_u32 v[42:43], s[56:57], v50, v47, s[76:77]",      # data + node * slot_size
               "s_add_u32 s69, s66, 16",                                     # + 16 + val_off
               "v_add_co_u32 v42, vcc, s69, v42", "v_addc_co_u32 v43, vcc, 0, v43, vcc",
               f"v_cndmask_b32 v{R0}, 0, v42, s[54:55]",
               f"v_cndmask_b32 v{R0 + 1}, 0, v43, s[54:55]")
        self.next_seq()

    def call_lookup_ak(self):
        """ARRAY lookup, map bound at load (w[2:3] = value base, w4 =
        max_entries, w5 = value size), key at stack offset w6:
        r0 = key < max_entries ? base + key * vsz : 0 (array_map.cpp:27-40)."""
        self.e("v_add_u32 v41, s46, %[stklo]", "ds_read_b32 v46, v41", "s_waitcnt lgkmcnt(0)",
               "v_cmp_gt_u32 s[54:55], s44, v46",
               "v_mov_b32 v47, s45",
               "v_mad_u64_u32 v[50:51], s[56:57], v46, v47, s[42:43]",
               f"v_cndmask_b32 v{R0}, 0, v50, s[54:55]",
               f"v_cndmask_b32 v{R0 + 1}, 0, v51, s[54:55]")
        self.next_seq()

    def hash_mod_step(self):
        """v[50:51] = x (f64, integer < 2^48) -> v56 = x mod nb, with v[58:59]
        = nb and v[54:55] ~ 1/nb (f64).  q = trunc(x / nb) is off by at most
        one, x - q*nb is exact in one fma, then one correction each way."""
        self.e("v_mul_f64 v[42:43], v[50:51], v[54:55]",
               "v_trunc_f64 v[42:43], v[42:43]",
               "v_fma_f64 v[50:51], -v[42:43], v[58:59], v[50:51]",
               "v_cmp_gt_f64 vcc, 0, v[50:51]",
               "v_add_f64 v[42:43], v[50:51], v[58:59]",
               "v_cndmask_b32 v50, v50, v42, vcc", "v_cndmask_b32 v51, v51, v43, vcc",
               "v_cmp_le_f64 vcc, v[58:59], v[50:51]",
               "v_add_f64 v[42:43], v[50:51], -v[58:59]",
               "v_cndmask_b32 v50, v50, v42, vcc", "v_cndmask_b32 v51, v51, v43, vcc",
               "v_cvt_u32_f64 v56, v[50:51]")

    # ---- the block's hash-lookup cache (common.hpp kLcacheSets) ----
    # w4 (s44) two-way sets right below the launch constants (%[comb] - TENV -
    # 40 * sets): the ways' keys (16 B each, [way][set], the key's first kd
    # words: a way's keys of consecutive sets are consecutive 16-byte slots
    # of a bank row), then the ways' entries {u32 (slot + 1) | fd << 22}
    # ([set][way], at + 32 * sets).  The set is a mix of the key words and the fd, so a hit
    # needs neither the h*31 hash nor a memory access: the whole key is
    # compared in LDS.  Entries are written once: a lane that found its key
    # claims an empty way (0 -> -1 by compare-and-swap), writes the key, then
    # the entry; a reader reads the entries before the keys, and one CU's LDS
    # keeps every wave's accesses in order, so an entry it sees is complete.
    # Only hash lookups the loader marked FW_LCACHE use it: nothing deletes
    # during their launch (the program cannot, and vm_api.cpp / maps.cpp keep
    # every other deleting launch and host delete from overlapping it), so a
    # slot found for a key stays that key's slot.  A probe leaves v82 / v83 =
    # the key / entry address of the set's first empty way (v83 = -1: none)
    # for the fill; s49 = the map fd.
    def lcache_on(self, skip):
        self.e("s_bitcmp1_b32 s41, 1", f"s_cbranch_scc0 {skip}",
               "s_cmp_gt_u32 s66, 0x3ffffe", f"s_cbranch_scc1 {skip}")      # slot + 1 in 22 bits

    def lcache_probe(self, kd, done):
        """Lanes whose key (v44..v(43 + kd)) the cache holds get r0 and leave
        s[60:61]; the others go on to the hash with exec = s[60:61]."""
        skip = self.label("lcs")
        self.e("v_mov_b32 v83, -1")
        self.lcache_on(skip)
        mult = ["0x9e3779b1", "0x85ebca6b", "0xc2b2ae35", "0x27d4eb2f"]
        self.e("s_mul_i32 s69, s49, 0x165667b1", "v_mov_b32 v41, s69")
        for j in range(kd):
            self.e(f"s_mov_b32 s69, {mult[j]}", f"v_mul_lo_u32 v42, v{44 + j}, s69", "v_xor_b32 v41, v41, v42")
        self.e("v_lshrrev_b32 v42, 15, v41", "v_xor_b32 v41, v41, v42",
               "s_mov_b32 s69, 0x2c1b3c6d", "v_mul_lo_u32 v41, v41, s69",
               "v_mul_hi_u32 v41, v41, s44",                                       # the set (w4 sets)
               "s_mul_i32 s69, s44, 40", "s_add_u32 s69, s69, " + str(TENV),
               "s_sub_u32 s69, %[comb], s69",                                     # the cache
               "v_lshl_add_u32 v82, v41, 4, s69",                                 # its way-0 key
               "s_lshl_b32 s85, s44, 4",                                          # way 1: + sets * 16
               # (s64..s71 hold the map's words here: val_off in s70)
               "v_mul_u32_u24_e64 v83, s44, 32", "v_add_u32 v83, s69, v83",
               "v_lshl_add_u32 v83, v41, 3, v83",                                 # its entries
               "ds_read_b64 v[54:55], v83",                                       # entries first
               "v_add_u32 v41, s85, v82",
               "ds_read_b128 v[56:59], v82",
               "ds_read_b128 v[48:51], v41",
               "s_waitcnt lgkmcnt(0)",
               "s_lshl_b32 s69, s49, 22")
        for way, (ent, k0, m) in enumerate(((54, 56, "s[56:57]"), (55, 48, "s[54:55]"))):
            self.e(f"v_and_b32 v42, 0xffc00000, v{ent}", f"v_cmp_eq_u32 {m}, s69, v42",
                   f"v_cmp_ne_u32 vcc, 0, v{ent}", f"s_and_b64 {m}, {m}, vcc",
                   f"v_cmp_ne_u32 vcc, -1, v{ent}", f"s_and_b64 {m}, {m}, vcc")
            for j in range(kd):
                self.e(f"v_cmp_eq_u32 vcc, v{k0 + j}, v{44 + j}", f"s_and_b64 {m}, {m}, vcc")
        # the fill's way: the first empty one (v83 = -1: both taken)
        self.e("v_cmp_eq_u32 vcc, 0, v54",
               "v_add_u32 v42, 4, v83", "v_add_u32 v41, s85, v82",
               "v_cmp_eq_u32 s[52:53], 0, v55",
               "v_cndmask_b32 v42, -1, v42, s[52:53]",
               "v_cndmask_b32 v83, v42, v83, vcc",
               "v_cndmask_b32 v82, v41, v82, vcc",
               "v_cndmask_b32 v58, v55, v54, s[56:57]",
               "v_and_b32 v58, 0x3fffff, v58", "v_add_u32 v58, -1, v58",          # the slot
               "s_or_b64 s[56:57], s[56:57], s[54:55]", "s_and_b64 s[56:57], s[56:57], exec")
        self.lcache_count()
        self.e(f"s_cbranch_scc0 {skip}",
               "v_mov_b32 v59, s68",
               "v_mad_u64_u32 v[42:43], s[54:55], v58, v59, s[64:65]",
               "s_mov_b64 s[54:55], exec", "s_mov_b64 exec, s[56:57]",            # exec = hits
               f"v_add_co_u32 v{R0}, vcc, s70, v42", f"v_addc_co_u32 v{R0 + 1}, vcc, 0, v43, vcc",
               "s_andn2_b64 s[60:61], s[54:55], s[56:57]", "s_mov_b64 exec, s[60:61]",
               f"s_cbranch_execz {done}",
               f"{skip}:")

    def lcache_count(self):
        """BPFTIME_AMD_DBG 512 (oflags bit 3): add the probe's hits
        (s[56:57]) and misses (the other lanes of exec) to the counters at
        tenv[1] (interp.hip; read by bpftime_amd_dbg_counters).  Keeps SCC =
        (hits != 0) for the branch that follows."""
        off = self.label("lcc")
        self.e("s_bitcmp1_b32 %[oflags], 3", f"s_cbranch_scc0 {off}",
               "s_bcnt1_i32_b64 s52, s[56:57]", "s_bcnt1_i32_b64 s53, exec", "s_sub_u32 s53, s53, s52",
               "s_mov_b64 s[54:55], exec", "s_mov_b64 exec, 1",
               f"s_sub_u32 s69, %[comb], {TENV - 8}", "v_mov_b32 v41, s69",
               "ds_read_b64 v[42:43], v41",
               "v_mov_b32 v56, s52", "v_mov_b32 v57, 0",
               "s_waitcnt lgkmcnt(0)",
               "global_atomic_add_x2 v[42:43], v[56:57], off",
               "v_mov_b32 v56, s53",
               "global_atomic_add_x2 v[42:43], v[56:57], off offset:8",
               "s_mov_b64 exec, s[54:55]",
               f"{off}:",
               "s_cmp_lg_u64 s[56:57], 0")

    def dbg_lanes(self, slot, mask):
        """BPFTIME_AMD_DBG 512: add the lanes of `mask` (an SGPR pair, a
        subset of exec) to counter `slot` at tenv[1] (index-probe exits);
        uses s[52:53], s69, v[42:43], v[58:59] (the probe's entry in v56
        and key in v[48:51] stay)."""
        off, back = self.label("dlo"), self.label("dlb")
        self.e("s_bitcmp1_b32 %[oflags], 3", f"s_cbranch_scc0 {off}",
               "s_mov_b64 s[52:53], exec", f"s_and_b64 exec, exec, {mask}", f"s_cbranch_execz {back}",
               f"s_sub_u32 s69, %[comb], {TENV - 8}", "v_mov_b32 v42, s69",
               "ds_read_b64 v[42:43], v42",
               "v_mov_b32 v58, 1", "v_mov_b32 v59, 0",
               "s_waitcnt lgkmcnt(0)",
               f"global_atomic_add_x2 v[42:43], v[58:59], off offset:{8 * slot}",
               f"{back}:", "s_mov_b64 exec, s[52:53]",
               f"{off}:")

    def lcache_fill(self, vslot):
        """exec = lanes that found their key in slot v<vslot>: claim the
        probe's empty way (v83) and write the key, then the entry (a lane
        that loses the claim to another key leaves the cache as it is)."""
        skip, out = self.label("lcf"), self.label("lco")
        self.lcache_on(skip)
        self.e("s_mov_b64 s[52:53], exec",
               "v_cmp_ne_u32 vcc, -1, v83", "s_and_b64 exec, exec, vcc", f"s_cbranch_execz {out}",
               "v_mov_b32 v58, 0", "v_mov_b32 v59, -1",
               "ds_cmpst_rtn_b32 v42, v83, v58, v59",                            # claim: 0 -> -1
               "s_waitcnt lgkmcnt(0)",
               "v_cmp_eq_u32 vcc, 0, v42", "s_and_b64 exec, exec, vcc", f"s_cbranch_execz {out}",
               f"v_add_u32 v59, 1, v{vslot}", "s_lshl_b32 s69, s49, 22", "v_or_b32 v59, s69, v59",
               "ds_write_b128 v82, v[44:47]",                                     # the key, then
               "ds_write_b32 v83, v59",                                           # the entry
               f"{out}:",
               "s_mov_b64 exec, s[52:53]",
               f"{skip}:")

    def index_probe(self, kd, done, bail):
        """The map's lookup index (common.hpp ix_pos), if it has one: up to
        kIxProbes entries from ix_pos(h) until every lane has found its key
        (r0 = that slot's value).  The index is keyed (common.hpp
        ix_key_stride: the key of each entry at the same position in an
        array beside the entries), so a probe loads entry and key together
        and the bucket is never read.  The index holds exactly the keys the
        reference probe reaches, so an empty entry in any lane (a miss, or a
        line of this XCD's L2 an insert has not reached yet), an entry an
        insert holds reserved (kIxRes), or too many probes hand the whole
        wave to the C++ tier's lookup (dev_helpers.hpp hash_find_ix: coherent
        reads, the miss record the lookup-or-init race rule needs) instead of
        the reference probe's walk.  A map without an index goes to the
        reference probe that follows (h stays in v[48:49]).  A published
        entry's key was written (one store) before the entry: a key line this
        XCD's L2 holds from before can only read zero, so a hit on the
        all-zero key is confirmed in its bucket."""
        loop, fail = self.label("ixl"), self.label("ixf")
        ks = 8 if kd <= 2 else 16
        self.e("s_cmp_eq_u64 s[74:75], 0", f"s_cbranch_scc1 {fail}",
               "s_mov_b32 s85, 0x85ebca6b", "v_mul_lo_u32 v41, v49, s85", "v_xor_b32 v41, v41, v48",
               "s_mov_b32 s85, 0x9e3779b1", "v_mul_lo_u32 v41, v41, s85",
               "v_lshrrev_b32 v50, 16, v41", "v_xor_b32 v41, v41, v50", "v_and_b32 v41, s67, v41",
               "s_mov_b32 s85, 0",
               f"{loop}:",
               # the keys: 4 * (ix_mask + 1) bytes after the entries
               "s_add_u32 s52, s67, 1", "s_mov_b32 s53, 0", "s_lshl_b64 s[52:53], s[52:53], 2",
               "s_add_u32 s52, s52, s74", "s_addc_u32 s53, s53, s75",
               "v_mad_u64_u32 v[42:43], s[56:57], v41, 4, s[74:75]",
               f"v_mad_u64_u32 v[54:55], s[56:57], v41, {ks}, s[52:53]",
               "global_load_dword v56, v[42:43], off sc1",                      # bucket + 1
               "global_load_dwordx2 v[48:49], v[54:55], off sc1" if ks == 8 else
               "global_load_dwordx4 v[48:51], v[54:55], off sc1",               # its key
               "s_waitcnt vmcnt(0)",
               "v_cmp_eq_u32 s[56:57], 0, v56",                                 # empty entry
               "v_cmp_eq_u32 vcc, -1, v56", "s_or_b64 s[56:57], s[56:57], vcc")  # ... or reserved
        self.dbg_lanes(2, "s[56:57]")
        self.e("s_cmp_lg_u64 s[56:57], 0", f"s_cbranch_scc1 {bail}",
               "v_cmp_eq_u32 s[56:57], v48, v44", "v_mov_b32 v57, v44")
        for j in range(1, kd):
            self.e(f"v_cmp_eq_u32 vcc, v{48 + j}, v{44 + j}", "s_and_b64 s[56:57], s[56:57], vcc",
                   f"v_or_b32 v57, v57, v{44 + j}")
        nz = self.label("ixnz")
        self.e("v_add_u32 v50, -1, v56",
               "v_mov_b32 v51, s68",
               "v_mad_u64_u32 v[54:55], vcc, v50, v51, s[64:65]",               # slot
               # hits on the all-zero key: confirmed in the bucket (state
               # FILLED and the key, as an index without keys does)
               "v_cmp_eq_u32 vcc, 0, v57", "s_and_b64 vcc, vcc, s[56:57]", "s_and_b64 s[62:63], vcc, exec",
               f"s_cbranch_scc0 {nz}",
               "s_mov_b64 s[52:53], exec", "s_mov_b64 exec, s[62:63]",
               # (v50 = the bucket stays for the lookup cache's fill)
               "global_load_dword v57, v[54:55], off sc1",
               "global_load_dwordx2 v[58:59], v[54:55], off offset:8 sc1")
        if kd > 2:
            self.e("global_load_dwordx2 v[42:43], v[54:55], off offset:16 sc1")
        self.e("s_waitcnt vmcnt(0)",
               "v_cmp_ne_u32 vcc, 1, v57")
        for j, v in zip(range(kd), (58, 59, 42, 43)):
            self.e(f"v_cmp_ne_u32 s[62:63], v{v}, v{44 + j}", "s_or_b64 vcc, vcc, s[62:63]")
        self.e("s_and_b64 vcc, vcc, exec", "s_andn2_b64 s[56:57], s[56:57], vcc",
               "s_mov_b64 exec, s[52:53]",
               f"{nz}:",
               "s_and_saveexec_b64 s[62:63], s[56:57]",                         # exec = hits
               f"v_add_co_u32 v{R0}, vcc, s70, v54", f"v_addc_co_u32 v{R0 + 1}, vcc, 0, v55, vcc")
        self.lcache_fill(50)
        self.e("s_andn2_b64 exec, s[62:63], s[56:57]",                          # exec = other keys
               f"s_cbranch_execz {done}",
               "v_add_u32 v41, 1, v41", "v_and_b32 v41, s67, v41",
               "s_add_u32 s85, s85, 1", "s_cmp_lt_u32 s85, 8", f"s_cbranch_scc1 {loop}")
        self.dbg_lanes(3, "exec")
        self.e(f"s_branch {bail}",
               f"{fail}:", "s_mov_b64 exec, s[60:61]")

    def hash_lookup(self, update=False):
        done, bail = self.label("hdone"), self.label("hbail")
        # DMap words 4-11 (s[64:71], loaded by call_lookup): data,
        # nbuckets, ix_mask, slot_size, key_off, val_off, ncpu; words 14-15
        # (s[52:53] there): lookup index (0 = none); the key in v[44:47]
        self.e("s_mov_b64 s[74:75], s[52:53]",
               "s_mov_b64 s[60:61], exec", "s_mov_b64 s[76:77], exec",     # lanes still looking / all of them
               "s_mov_b32 s49, s62")                                          # the map fd
        for kd in (1, 2, 3, 4):
            nxt = self.label("kdn")
            self.e(f"s_cmp_lg_u32 s73, {4 * kd}", f"s_cbranch_scc1 {nxt}")
            self.lcache_probe(kd, done)
            # h = sum over key bytes of h * 31 + byte (size_t arithmetic)
            self.e("v_mov_b32 v48, 0", "v_mov_b32 v49, 0")
            for i in range(4 * kd):
                self.e("v_lshlrev_b64 v[50:51], 5, v[48:49]",
                       "v_sub_co_u32 v48, vcc, v50, v48", "v_subb_co_u32 v49, vcc, v51, v49, vcc",
                       f"v_bfe_u32 v50, v{44 + i // 4}, {8 * (i % 4)}, 8",
                       "v_add_co_u32 v48, vcc, v48, v50", "v_addc_co_u32 v49, vcc, 0, v49, vcc")
            self.index_probe(kd, done, bail)
            # idx = h % nbuckets: h = ((hi * 2^16 + lo >> 16) * 2^16 + lo & 0xffff)
            self.e("v_cvt_f64_u32 v[58:59], s66", "v_rcp_f64 v[54:55], v[58:59]",
                   "v_cvt_f64_u32 v[50:51], v49")
            self.hash_mod_step()
            for part in ("v_lshrrev_b32 v57, 16, v48", "v_and_b32 v57, 0xffff, v48"):
                self.e("v_cvt_f64_u32 v[50:51], v56", "v_ldexp_f64 v[50:51], v[50:51], 16",
                       part, "v_cvt_f64_u32 v[42:43], v57", "v_add_f64 v[50:51], v[50:51], v[42:43]")
                self.hash_mod_step()
            # linear probing from idx until every lane hits; stop at anything else
            loop = self.label("probe")
            self.e("v_mov_b32 v57, v56", "v_mov_b32 v43, s68", "s_mov_b32 s85, 0",
                   f"{loop}:",
                   "v_mad_u64_u32 v[54:55], s[56:57], v56, v43, s[64:65]",
                   "global_load_dword v58, v[54:55], off sc1",
                   "global_load_dwordx4 v[48:51], v[54:55], off offset:8 sc1",
                   "s_waitcnt vmcnt(0)",
                   "v_cmp_ne_u32 s[56:57], 1, v58",                          # not FILLED
                   "s_cmp_lg_u64 s[56:57], 0", f"s_cbranch_scc1 {bail}",
                   "v_cmp_eq_u32 s[56:57], v48, v44")
            for j in range(1, kd):
                self.e(f"v_cmp_eq_u32 vcc, v{48 + j}, v{44 + j}", "s_and_b64 s[56:57], s[56:57], vcc")
            self.e("s_and_saveexec_b64 s[62:63], s[56:57]",                   # exec = hits
                   f"v_add_co_u32 v{R0}, vcc, s70, v54", f"v_addc_co_u32 v{R0 + 1}, vcc, 0, v55, vcc")
            self.lcache_fill(56)
            self.e("s_andn2_b64 exec, s[62:63], s[56:57]",                    # exec = other keys
                   f"s_cbranch_execz {done}",
                   "v_add_u32 v56, 1, v56",
                   "v_cmp_eq_u32 vcc, s66, v56", "v_cndmask_b32 v56, v56, 0, vcc",
                   "v_cmp_eq_u32 vcc, v57, v56",                              # wrapped: a miss
                   f"s_cbranch_vccnz {bail}",
                   "s_add_u32 s85, s85, 1", "s_cmp_gt_u32 s85, 63", f"s_cbranch_scc1 {bail}",
                   f"s_branch {loop}",
                   f"{nxt}:")
        self.e(f"s_branch {L('slow')}",
               f"{bail}:", "s_mov_b64 exec, s[76:77]", f"s_branch {L('slow')}",
               f"{done}:", "s_mov_b64 exec, s[76:77]")
        if update:
            self.update_tail()
        self.next_seq()

    def counter_cache(self, sz, done):
        """A0 = s[62:63] (uniform address), V0 = s[64:65] (uniform value):
        add popcount(exec) * V0 into the per-wave delta cache (two entries,
        flushed by the C++ side); both entries taken by other addresses ->
        leave (C++ evicts one)."""
        t1, t2, t3 = (self.label(x) for x in ("t1", "t2", "t3"))
        self.e("s_bcnt1_i32_b64 s69, exec",
               "s_mul_i32 s66, s64, s69", "s_mul_hi_u32 s67, s64, s69",
               "s_mul_i32 s70, s65, s69", "s_add_u32 s67, s67, s70",
               "s_cmp_eq_u64 %[c0a], s[62:63]", f"s_cbranch_scc0 {t1}",
               f"s_cmp_eq_u32 %[c0s], {sz}", f"s_cbranch_scc0 {t1}",
               "s_add_u32 %[c0dl], %[c0dl], s66", "s_addc_u32 %[c0dh], %[c0dh], s67", f"s_branch {done}",
               f"{t1}:",
               "s_cmp_eq_u64 %[c1a], s[62:63]", f"s_cbranch_scc0 {t2}",
               f"s_cmp_eq_u32 %[c1s], {sz}", f"s_cbranch_scc0 {t2}",
               "s_add_u32 %[c1dl], %[c1dl], s66", "s_addc_u32 %[c1dh], %[c1dh], s67", f"s_branch {done}",
               f"{t2}:",
               "s_cmp_eq_u64 %[c0a], 0", f"s_cbranch_scc0 {t3}",
               "s_mov_b64 %[c0a], s[62:63]", "s_mov_b32 %[c0dl], s66", "s_mov_b32 %[c0dh], s67",
               f"s_mov_b32 %[c0s], {sz}", f"s_branch {done}",
               f"{t3}:",
               "s_cmp_eq_u64 %[c1a], 0", f"s_cbranch_scc0 {L('slow')}",      # both taken: C++ evicts
               "s_mov_b64 %[c1a], s[62:63]", "s_mov_b32 %[c1dl], s66", "s_mov_b32 %[c1dh], s67",
               f"s_mov_b32 %[c1s], {sz}",
               f"s_branch {done}")

    def rmw_value(self, k):
        if k == "R":
            self.rd("s45", 46)
        else:
            self.e("v_mov_b32 v46, s47", "v_ashrrev_i32 v47, 31, v46")

    def rmw(self, sz, k, mv=False):
        """Fused counter (loader: ldx/add/stx, register dead after).  A wave
        whose live lanes all add the same value to the same global address
        adds popcount * value into the per-wave delta cache; otherwise each
        lane adds through the LDS combining table.  mv: the base is a
        non-null map-value pointer (no staging / window checks)."""
        stg, glb = self.label("rs"), self.label("rg")
        self.rd("s44", 48)
        self.rmw_value(k)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        if not mv:
            self.staged_or(sz, stg, glb)
            self.e(f"{stg}:", f"s_branch {L('slow')}")   # a counter inside the unit's own bytes
            self.e(f"{glb}:")
            self.check(sz)
        done, lane = self.label("done"), self.label("lane")
        self.e("v_readfirstlane_b32 s62, v48", "v_readfirstlane_b32 s63, v49",
               "v_cmp_ne_u64 s[54:55], s[62:63], v[48:49]",
               "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {lane}")
        if not mv:
            self.e("s_cmp_eq_u32 s63, %[shi]", f"s_cbranch_scc1 {L('slow')}",   # LDS / scratch targets
                   "s_cmp_eq_u32 s63, %[phi]", f"s_cbranch_scc1 {L('slow')}")
        self.e("v_readfirstlane_b32 s64, v46", "v_readfirstlane_b32 s65, v47",
               "v_cmp_ne_u64 s[54:55], s[64:65], v[46:47]",
               "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {lane}")
        self.counter_cache(sz, done)
        # lanes disagree on address or value: one add per lane
        self.e(f"{lane}:")
        if not mv:
            self.check_global(sz)
        self.comb_add(sz)
        self.e(f"{done}:", "s_mov_b32 s48, s46")           # continue after the stx
        self.dispatch()

    def rmwk(self, sz, k):
        """Fused counter on a constant map-value address (lddw map_val +
        offset, bound at load: w[2:3] = the address)."""
        done, lane = self.label("done"), self.label("lane")
        if k == "I":
            self.e("s_mov_b32 s64, s47", "s_ashr_i32 s65, s47, 31")
        else:
            self.rd("s45", 46)
            self.e("v_readfirstlane_b32 s64, v46", "v_readfirstlane_b32 s65, v47",
                   "v_cmp_ne_u64 s[54:55], s[64:65], v[46:47]",
                   "s_cmp_lg_u64 s[54:55], 0", f"s_cbranch_scc1 {lane}")
        self.e("s_mov_b64 s[62:63], s[42:43]")
        self.counter_cache(sz, done)
        self.e(f"{lane}:")
        if k == "R":
            self.e("v_mov_b32 v48, s42", "v_mov_b32 v49, s43")
            self.comb_add(sz)
        self.e(f"{done}:", "s_mov_b32 s48, s46")
        self.dispatch()

    def rmwd(self, sz, k):
        """Fused counter that must reach memory now (FW_NODEFER: a later
        access of the unit may read or overwrite it, or the batch is
        ORDERED): lanes sharing an address and value fold into one device
        atomic, the rest add lane by lane, and the adds are drained before
        the next instruction.  Targets in the unit's staged bytes, LDS or
        scratch leave for the C++ tier."""
        glb = self.label("dg")
        self.rd("s44", 48)
        self.rmw_value(k)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        self.staged_or(sz, L("slow"), glb)
        self.e(f"{glb}:")
        self.check_global(sz)
        self.comb_peel(sz, direct_only=True)
        self.e("s_waitcnt vmcnt(0)", "s_mov_b32 s48, s46")   # continue after the stx
        self.dispatch()

    def atomd(self, sz):
        """BPF_ATOMIC add without fetch that must reach memory now
        (FW_NODEFER)."""
        glb = self.label("adg")
        self.rd("s44", 48)
        self.rd("s45", 46)
        if sz == 4:
            self.e("v_mov_b32 v47, 0")
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        self.staged_or(sz, L("slow"), glb)
        self.e(f"{glb}:")
        self.check_global(sz)
        self.comb_peel(sz, direct_only=True)
        self.e("s_waitcnt vmcnt(0)")
        self.next_seq()

    def atomic(self, sz, op, fetch, mv=False):
        """BPF_ATOMIC add/or/and/xor (+ BPF_FETCH) on global memory: one
        device-scope atomic per lane (array_map values, hash values).  LDS or
        scratch targets and the unit's own staged bytes leave for C++.  mv:
        the base is a non-null map-value pointer."""
        glb = self.label("ag")
        self.rd("s44", 48)
        self.rd("s45", 44)
        self.e("v_lshl_add_u64 v[48:49], v[48:49], 0, s[42:43]")
        if not mv:
            self.staged_or(sz, L("slow"), glb)
            self.e(f"{glb}:")
            self.check_global(sz)
        mn = op.lower() + ("_x2" if sz == 8 else "")
        val = "v[44:45]" if sz == 8 else "v44"
        if fetch:
            self.e(f"global_atomic_{mn} {'v[46:47]' if sz == 8 else 'v46'}, v[48:49], {val}, off sc0",
                   "s_waitcnt vmcnt(0)")
            if sz == 4:
                self.e("v_mov_b32 v47, 0")
            self.wr("s45", 46)
        elif op == "ADD":
            self.e("v_mov_b32 v46, v44", "v_mov_b32 v47, v45" if sz == 8 else "v_mov_b32 v47, 0")
            self.comb_add(sz)
        else:
            self.e(f"global_atomic_{mn} v[48:49], {val}, off")
        self.next_seq()

    def exit_(self):
        """The running lanes exit: write back their dirty bytes, store r0 as
        verdict (u32) and ret (u64); then the next pending lane group runs,
        or the block ends (every live lane has exited)."""
        nv, nr, last = self.label("nv"), self.label("nr"), self.label("last")
        self.movi_prefix()
        self.flush(clear=False)
        self.e("s_bitcmp1_b32 %[oflags], 0", f"s_cbranch_scc0 {nv}",
               f"global_store_dword %[vaddr], v{R0}, off",
               f"{nv}:",
               "s_bitcmp1_b32 %[oflags], 1", f"s_cbranch_scc0 {nr}",
               f"global_store_dwordx2 %[raddr], v[{R0}:{R0 + 1}], off",
               f"{nr}:",
               "s_cmp_eq_u32 s92, 0", f"s_cbranch_scc1 {last}",
               "s_mov_b32 s48, s86", "s_mov_b64 exec, s[88:89]")
        self.pop0()
        self.dispatch()
        self.e(f"{last}:", "s_mov_b32 s84, 0", f"s_branch {L('chain')}")

    # ---- unit chaining: the next unit starts inside the block ----
    # After a unit every lane of the wave has exited, the wave's next unit
    # (unit + ustep: %[sstep] bytes further on) runs without leaving the
    # block, while %[chain] (full iterations left, counted down here) allows:
    # the C++ side's per-unit setup and the block's entry / exit cost once
    # per chain instead of once per unit.  entry bits: 3 r1 = the slot,
    # 4 r2 = the unit length, 5 lengths from %[laddr], 6 the syscall-record
    # filter (exit / exit_group records are skipped with r0 = 0,
    # syscall_trace_attach_impl.cpp:25), 7 reset the lane's tail-call depth
    # (images), 16.. the per-unit step of the
    # virtual cpu (%[vcpu] = cpu | ncpu << 16, or ~0).
    def chain_routine(self):
        nxt, nov, nol, nos, sv, sr, nod, lw = (self.label(x) for x in ("cnext", "cnv", "cnl", "cns", "csv", "csr",
                                                                       "cnd", "clw"))
        e = self.e
        e(f"{L('chain')}:",
          "s_cmp_eq_u32 %[chain], 0", f"s_cbranch_scc1 {L('cend')}",
          f"{nxt}:",
          "s_sub_u32 %[chain], %[chain], 1",
          "s_mov_b64 exec, s[58:59]",
          "s_mov_b32 s71, 0",
          "s_mov_b32 s70, %[sstep]",
          "v_lshl_add_u64 v[52:53], v[52:53], 0, s[70:71]",
          "s_lshl_b32 s70, %[ustep], 2",
          "v_lshl_add_u64 %[vaddr], %[vaddr], 0, s[70:71]",
          "v_lshl_add_u64 %[laddr], %[laddr], 0, s[70:71]",
          "s_lshl_b32 s70, %[ustep], 3",
          "v_lshl_add_u64 %[raddr], %[raddr], 0, s[70:71]",
          # virtual cpu: + step, mod ncpu
          "s_cmp_eq_u32 %[vcpu], -1", f"s_cbranch_scc1 {nov}",
          "s_lshr_b32 s69, %[vcpu], 16",
          "s_and_b32 s70, %[vcpu], 0xffff",
          "s_lshr_b32 s71, %[entry], 16",
          "s_add_u32 s70, s70, s71",
          "s_sub_u32 s71, s70, s69",
          "s_cmp_ge_u32 s70, s69",
          "s_cselect_b32 s70, s71, s70",
          "s_lshl_b32 s69, s69, 16",
          "s_or_b32 %[vcpu], s70, s69",
          f"{nov}:",
          "s_bitcmp1_b32 %[entry], 5", f"s_cbranch_scc0 {nol}",
          "global_load_dword %[ulen], %[laddr], off",
          "s_bitcmp1_b32 %[entry], 4", f"s_cbranch_scc1 {lw}",              # r2 = the length: wait now
          "s_bitcmp1_b32 %[entry], 1", f"s_cbranch_scc1 {nol}",             # staged: waited for with its loads
          f"{lw}:", "s_waitcnt vmcnt(0)",
          f"{nol}:",
          "s_bitcmp1_b32 %[entry], 6", f"s_cbranch_scc0 {nos}",
          "s_bitcmp1_b32 %[entry], 1", f"s_cbranch_scc1 {nos}",                 # staged: filtered at fresh
          # syscall filter: nr = *(u64 *)(slot + 8) in {60, 231} -> r0 = 0
          "global_load_dwordx2 v[56:57], v[52:53], off offset:8",
          "s_movk_i32 s70, 0xe7", "s_mov_b32 s71, 0",
          "s_waitcnt vmcnt(0)",
          "v_cmp_eq_u64 s[54:55], 60, v[56:57]",
          "v_cmp_eq_u64 s[56:57], s[70:71], v[56:57]",
          "s_or_b64 s[54:55], s[54:55], s[56:57]",
          "s_and_b64 s[54:55], s[54:55], exec",
          f"s_cbranch_scc0 {nos}",
          "s_andn2_b64 s[60:61], exec, s[54:55]",
          "s_mov_b64 exec, s[54:55]",
          "v_mov_b32 v56, 0", "v_mov_b32 v57, 0",
          "s_bitcmp1_b32 %[oflags], 0", f"s_cbranch_scc0 {sv}",
          "global_store_dword %[vaddr], v56, off",
          f"{sv}:",
          "s_bitcmp1_b32 %[oflags], 1", f"s_cbranch_scc0 {sr}",
          "global_store_dwordx2 %[raddr], v[56:57], off",
          f"{sr}:",
          "s_mov_b64 exec, s[60:61]",
          f"s_cbranch_execnz {nos}",
          "s_cmp_eq_u32 %[chain], 0", f"s_cbranch_scc0 {nxt}",
          f"s_branch {L('cend')}",
          f"{nos}:",
          # images: the lane's tail-call depth back to 0 (R slot 12, lo word)
          "s_bitcmp1_b32 %[entry], 7", f"s_cbranch_scc0 {nod}",
          "v_mov_b32 v56, 0",
          f"ds_write_b32 v40, v56 offset:{self.depth_off}",
          f"{nod}:",
          "s_mov_b32 %[steps], 0",
          "s_mov_b32 s48, 0",
          f"s_branch {L('fresh')}",
          f"{L('cend')}:",
          "s_mov_b64 exec, 0", "s_mov_b32 s68, 2", f"s_branch {L('done')}")

    # ---- bpf_tail_call in a linked image (XDP entry form) ----
    # The C++ path (interp.hip, kTailHelper / kRetHelper) restated for the
    # common case: every lane's ctx argument is its own LDS ctx (48 bytes
    # copied).  Frames have the C++ layout ([depth][word][lane] u64: r1..r10,
    # ctx address, return pc | ctx bytes << 32, ctx bytes from word 12, stack
    # bytes from word 20), so either tier pops what the other pushed.  The
    # launch constants sit in LDS 32 bytes below the combining table
    # (common.hpp dyn_lds_for; frames 0: tail calls in C++): frames
    # base, entry table, word stride, depth stride, stack words; a lane's depth
    # and grid lane index in its R[12] slot (v40 + 12 * 2048).
    def rgb(self):
        """s[52:53] = the launch constant tenv[4] (greg: the block's global
        r0 column minus the LDS address of the lane columns, so that v40 +
        r * 2048 addresses r's copy).  With no lane in exec nothing is
        stored or loaded through it.  (A VALU write of an SGPR that a VMEM
        instruction reads as its address needs 5 wait states: s_nop 4.)"""
        self.e(f"s_sub_u32 s52, %[comb], {TENV - 32}", "v_mov_b32 v41, s52",
               "ds_read_b64 v[42:43], v41", "s_waitcnt lgkmcnt(0)",
               "v_readfirstlane_b32 s52, v42", "v_readfirstlane_b32 s53, v43", "s_nop 4")

    def call_rbout(self):
        """bpf_ringbuf_output(ring, data, size, flags) (bpf_helper.cpp:451-467)
        on the block's ring staging (dev_helpers.hpp rb_reserve's staged path
        and rb_submit), the data being the unit's staged bytes from window
        dword w2 (loader.cpp link_staged: data = the packet at a constant
        offset): with the unit staged, the block's staging holding a promise
        from ring w6 (RbLds.fd), size (r3) wave-uniform, a multiple of 4 and
        at most 16, the first lane claims the wave's records in the block's
        budget with a compare-and-swap on RbLds.used and takes their record
        indices from RbLds.nrec; each lane writes its record (final: the
        block publishes its records when it ends, rb_publish) and its offset,
        r0 = 0.  Anything else -- no staging, an undecided or other ring, a
        closed or spent budget -- leaves for the C++ tier before any state
        changes (bail: exec restored first)."""
        slow = L("slow")
        loop, bail, d0, d1, d2, d3, dd = (self.label(x) for x in ("rbl", "rbb", "rb0", "rb1", "rb2", "rb3", "rbd"))
        e = self.e
        e("s_cmp_eq_u32 s80, 0", f"s_cbranch_scc1 {slow}",                 # the unit's staging
          f"s_sub_u32 s69, %[comb], {TENV - RB_TENV}", "v_mov_b32 v41, s69",
          "ds_read_b64 v[42:43], v41", "ds_read_b32 v44, v41 offset:8",
          f"v_mov_b32 v45, v{R0 + 6}", f"v_mov_b32 v46, v{R0 + 7}",          # r3 = size
          "s_waitcnt lgkmcnt(0)",
          "v_readfirstlane_b32 s52, v42", "v_readfirstlane_b32 s53, v43",  # the block's staging area
          "v_readfirstlane_b32 s70, v44",                                  # its RbLds
          "v_readfirstlane_b32 s44, v45",
          "s_cmp_eq_u64 s[52:53], 0", f"s_cbranch_scc1 {slow}",
          "v_cmp_ne_u32 s[54:55], s44, v45", "v_cmp_ne_u32 vcc, 0, v46",
          "s_or_b64 vcc, vcc, s[54:55]", "s_and_b64 vcc, vcc, exec", f"s_cbranch_vccnz {slow}",
          "s_and_b32 s69, s44, 3", "s_cmp_lg_u32 s69, 0", f"s_cbranch_scc1 {slow}",
          "s_cmp_gt_u32 s44, 16", f"s_cbranch_scc1 {slow}",
          "v_mov_b32 v41, s70",
          "ds_read_b32 v45, v41 offset:8",                                 # RbLds.fd
          "s_waitcnt lgkmcnt(0)", "v_readfirstlane_b32 s71, v45",
          "s_cmp_lg_u32 s71, s46", f"s_cbranch_scc1 {slow}",
          # the wave's bytes: lanes x total, total = (size + 8 + 7) & ~7
          "s_add_u32 s45, s44, 15", "s_and_b32 s45, s45, -8",
          "s_bcnt1_i32_b64 s69, exec", "s_mul_i32 s71, s69, s45",
          "s_mov_b64 s[54:55], exec",
          "s_ff1_i32_b64 s72, exec", "s_lshl_b64 exec, 1, s72",              # the first lane claims
          f"{loop}:",
          "ds_read_b32 v46, v41",                                          # RbLds.used
          "s_waitcnt lgkmcnt(0)", "v_readfirstlane_b32 s72, v46",
          "s_bitcmp1_b32 s72, 31", f"s_cbranch_scc1 {bail}",               # closed
          "s_add_u32 s73, s72, s71", f"s_cmp_gt_u32 s73, {RB_STAGE_REC}", f"s_cbranch_scc1 {bail}",
          "v_mov_b32 v46, s72", "v_mov_b32 v47, s73",
          "ds_cmpst_rtn_b32 v48, v41, v46, v47",
          "s_waitcnt lgkmcnt(0)", "v_readfirstlane_b32 s74, v48",
          "s_cmp_lg_u32 s74, s72", f"s_cbranch_scc1 {loop}",
          "v_mov_b32 v46, s69",
          "ds_add_rtn_u32 v48, v41, v46 offset:4",                          # RbLds.nrec
          "s_waitcnt lgkmcnt(0)", "v_readfirstlane_b32 s73, v48",
          "s_mov_b64 exec, s[54:55]",
          # each lane's record at base + rank * total: the header, then the data
          "v_mbcnt_lo_u32_b32 v46, s54, 0", "v_mbcnt_hi_u32_b32 v46, s55, v46",
          "v_mul_lo_u32 v47, v46, s45", "v_add_u32 v47, s72, v47",
          "v_add_co_u32 v48, vcc, s52, v47", "v_mov_b32 v49, s53", "v_addc_co_u32 v49, vcc, 0, v49, vcc",
          "v_mov_b32 v50, s44", "v_mov_b32 v51, s46",
          "global_store_dwordx2 v[48:49], v[50:51], off")
        self.idx("s42", "SRC0")
        e(f"v_mov_b32 v42, v{STG}", f"v_mov_b32 v43, v{STG + 1}", f"v_mov_b32 v44, v{STG + 2}",
          f"v_mov_b32 v45, v{STG + 3}")
        self.idx_off()
        e("s_cmp_eq_u32 s44, 4", f"s_cbranch_scc1 {d1}",
          "s_cmp_eq_u32 s44, 8", f"s_cbranch_scc1 {d2}",
          "s_cmp_eq_u32 s44, 12", f"s_cbranch_scc1 {d3}",
          "s_cmp_eq_u32 s44, 16", f"s_cbranch_scc0 {dd}",
          "global_store_dwordx4 v[48:49], v[42:45], off offset:8", f"s_branch {dd}",
          f"{d3}:", "global_store_dwordx3 v[48:49], v[42:44], off offset:8", f"s_branch {dd}",
          f"{d2}:", "global_store_dwordx2 v[48:49], v[42:43], off offset:8", f"s_branch {dd}",
          f"{d1}:", "global_store_dword v[48:49], v42, off offset:8",
          f"{dd}:",
          # the record's offset at the block's table (after the budget)
          "v_add_u32 v46, s73, v46", "v_lshlrev_b32 v46, 2, v46",
          f"v_add_u32 v46, {RB_STAGE_REC}, v46",
          "v_add_co_u32 v50, vcc, s52, v46", "v_mov_b32 v51, s53", "v_addc_co_u32 v51, vcc, 0, v51, vcc",
          "global_store_dword v[50:51], v47, off",
          f"v_mov_b32 v{R0}, 0", f"v_mov_b32 v{R0 + 1}, 0")
        self.next_seq()
        e(f"{bail}:", "s_mov_b64 exec, s[54:55]", f"s_branch {slow}")
        del d0

    def tail_env(self, slots=False):
        """The launch constants of tail calls; s46 / s47 = the LDS frames'
        offset from v40 and depths | words << 8 (FInsn w6 / w7 are not
        needed by TAIL / TRET); slots: also s[70:71] = the image's slot ->
        entry table (tenv[7]), read in the same LDS round trip."""
        self.e(f"s_sub_u32 s69, %[comb], {TENV}", "v_mov_b32 v41, s69",
               "ds_read_b128 v[42:45], v41", "ds_read_b128 v[46:49], v41 offset:16",
               f"ds_read_b64 v[58:59], v41 offset:{LF_TENV}",
               f"ds_read_b64 v[54:55], v40 offset:{self.depth_off}")          # depth, grid lane
        if slots:
            self.e("ds_read_b64 v[56:57], v41 offset:56")
        self.e("s_waitcnt lgkmcnt(0)",
               "v_readfirstlane_b32 s46, v58", "v_readfirstlane_b32 s47, v59",  # LDS frames
               "v_readfirstlane_b32 s72, v42", "v_readfirstlane_b32 s73, v43",  # frames
               "v_readfirstlane_b32 s74, v44", "v_readfirstlane_b32 s75, v45",  # entry table
               "v_readfirstlane_b32 s76, v46", "v_readfirstlane_b32 s77, v47",  # word / depth stride
               "v_readfirstlane_b32 s85, v48",                 # stack save mask | stack bytes << 16
               "v_readfirstlane_b32 s68, v49",                 # ctx save mask (s68: free until an exit)
               "s_cmp_eq_u64 s[72:73], 0", f"s_cbranch_scc1 {L('slow')}")
        if slots:
            self.e("v_readfirstlane_b32 s70, v56", "v_readfirstlane_b32 s71, v57", "s_nop 4")

    def lds_frame_ptr(self, v="v41"):
        """v = the LDS address of this lane's word 0 at depth v54 (an LDS
        frame: v40 + s46 + depth * words * 2048)."""
        self.e("s_lshr_b32 s69, s47, 8", "s_lshl_b32 s69, s69, 11",
               f"v_mul_lo_u32 {v}, v54, s69", f"v_add3_u32 {v}, {v}, v40, s46")

    def lds_stack_words(self, store, mask):
        """The stack words of the SGPR `mask` to (store) or from the LDS
        frame words at v48 on (v48 advances a word each)."""
        loop, done = self.label("tll"), self.label("tld")
        self.e("s_lshr_b32 s69, s85, 16", "v_subrev_u32 v43, s69, %[stklo]",   # the stack bottom
               f"s_mov_b32 s70, {mask}",
               f"{loop}:", "s_cmp_eq_u32 s70, 0", f"s_cbranch_scc1 {done}",
               "s_ff1_i32_b32 s69, s70", "s_bitset0_b32 s70, s69",
               "s_lshl_b32 s71, s69, 3", "v_add_u32 v49, s71, v43")
        if store:
            self.e("ds_read_b64 v[44:45], v49", "s_waitcnt lgkmcnt(0)", "ds_write_b64 v48, v[44:45]")
        else:
            self.e("ds_read_b64 v[44:45], v48", "s_waitcnt lgkmcnt(0)", "ds_write_b64 v49, v[44:45]")
        self.e("v_add_u32 v48, 0x800, v48", f"s_branch {loop}", f"{done}:")

    def frame_ptr(self):
        """v[56:57] = this lane's word 0 at depth v54."""
        self.e("v_mad_u64_u32 v[56:57], s[62:63], v55, 8, s[72:73]",
               "v_mad_u64_u32 v[56:57], s[62:63], v54, s77, v[56:57]")

    def fnext(self, n=1):
        for _ in range(n):
            self.e("v_add_co_u32 v56, vcc, s76, v56", "v_addc_co_u32 v57, vcc, 0, v57, vcc")

    def word_addr(self, w):
        """v[58:59] = the address of frame word w of this lane's frame."""
        if w == 0:
            self.e("v_mov_b32 v58, v56", "v_mov_b32 v59, v57")
        else:
            self.e(f"v_mad_u64_u32 v[58:59], s[62:63], {w}, s76, v[56:57]")

    def stack_words(self, store, mask=None):
        """The stack words of the save mask (s85 & 0xffff, or the SGPR
        `mask`; stack bytes s85 >> 16) to (store) or from the frame (words
        20..)."""
        loop, done = self.label("tsl"), self.label("tsd")
        self.e("s_lshr_b32 s69, s85, 16", "v_subrev_u32 v41, s69, %[stklo]",   # the stack bottom
               f"s_mov_b32 s70, {mask}" if mask else "s_and_b32 s70, s85, 0xffff",
               f"{loop}:", "s_cmp_eq_u32 s70, 0", f"s_cbranch_scc1 {done}",
               "s_ff1_i32_b32 s69, s70", "s_bitset0_b32 s70, s69",
               "s_lshl_b32 s71, s69, 3", "v_add_u32 v43, s71, v41",
               "s_add_u32 s71, s69, 20", "s_mul_i32 s71, s71, s76",
               "v_add_co_u32 v58, vcc, s71, v56", "v_addc_co_u32 v59, vcc, 0, v57, vcc")
        if store:
            self.e("ds_read_b64 v[44:45], v43", "s_waitcnt lgkmcnt(0)",
                   "global_store_dwordx2 v[58:59], v[44:45], off")
        else:
            self.e("global_load_dwordx2 v[44:45], v[58:59], off", "s_waitcnt vmcnt(0)",
                   "ds_write_b64 v43, v[44:45]")
        self.e(f"s_branch {loop}", f"{done}:")

    def go_groups(self):
        """Every running lane continues at its own IP (v50, bytes): the first
        lane's group runs, the others are parked as pending groups; more
        groups than the list holds hand every lane's pc to the C++ side."""
        single, over = self.label("g1"), self.label("gov")
        self.e("s_mov_b64 s[60:61], exec",
               "v_readfirstlane_b32 s69, v50",
               "v_cmp_eq_u32 s[62:63], s69, v50",
               "s_mov_b32 s48, s69", "s_mov_b64 s[72:73], s[62:63]",           # the running group
               "s_andn2_b64 s[74:75], s[60:61], s[62:63]")                     # lanes left
        for _ in range(KP):
            self.e("s_cmp_eq_u64 s[74:75], 0", f"s_cbranch_scc1 {single}",
                   f"s_cmp_ge_u32 s92, {KP}", f"s_cbranch_scc1 {over}",
                   "s_mov_b64 exec, s[74:75]",
                   "v_readfirstlane_b32 s69, v50",
                   "v_cmp_eq_u32 s[62:63], s69, v50",
                   "s_andn2_b64 s[74:75], s[74:75], s[62:63]")
            self.push()
        self.e("s_cmp_eq_u64 s[74:75], 0", f"s_cbranch_scc0 {over}",
               f"{single}:", "s_mov_b64 exec, s[72:73]")
        self.dispatch()
        # too many groups: every lane of this instruction takes its pc from
        # v50, the pending groups theirs (some may be this instruction's)
        self.e(f"{over}:",
               "s_mov_b64 exec, s[60:61]",
               "v_lshrrev_b32 %[lpc], 5, v50")
        self.materialize_pending()
        self.e("s_mov_b64 exec, s[60:61]", "s_mov_b32 s92, 0", "s_mov_b32 s68, 3", f"s_branch {L('spill')}")

    def tail_call(self):
        """bpf_tail_call(ctx, prog_array, index) (bpf_helper.cpp:568-650):
        index in range, a prog fd in the slot that is linked into the image,
        depth below 32 -> push a frame, r0 = r3..r9 = 0, r2 = 64, enter the
        target; else r0 = -1 and go on.  The map must be wave-uniform and a
        PROG_ARRAY, and every lane that can call must pass its own ctx;
        anything else leaves for C++ before changing state."""
        noval, ni = self.label("tnv"), self.label("tni")
        self.rd_fixed(2, 44)
        self.uniform64((44, 45), (62, 63))
        self.e("s_cmp_lg_u32 s63, 0", f"s_cbranch_scc1 {L('slow')}",
               "s_cmpk_ge_u32 s62, 0x400", f"s_cbranch_scc1 {L('slow')}",
               "s_lshl_b32 s69, s62, 6",
               "s_load_dwordx4 s[64:67], %[maps], s69")                      # type, ksz, vsz, max
        # the launch constants, and the image's slot -> entry pc table
        # (tenv[7], vm_api.cpp d_tail_slots: one load per lane instead of the
        # slot's prog fd and then that fd's entry), under the map's load
        self.tail_env(slots=True)
        self.e("s_cmp_lg_u32 s64, 3", f"s_cbranch_scc1 {L('slow')}",         # BPF_MAP_TYPE_PROG_ARRAY
               "s_cmp_eq_u64 s[70:71], 0", f"s_cbranch_scc1 {L('slow')}",
               "s_lshl_b32 s69, s62, 2",
               "s_load_dword s69, s[70:71], s69",                            # the array's offset
               "s_waitcnt lgkmcnt(0)",
               "s_cmp_lt_i32 s69, 0", f"s_cbranch_scc1 {L('slow')}",         # not in the image
               f"v_mov_b32 v46, v{R0 + 6}",                                  # `int idx = index`
               "v_cmp_gt_u32 s[54:55], s67, v46",                            # 0 <= idx < max_entries
               "v_cndmask_b32 v46, 0, v46, s[54:55]",
               "v_add_u32 v47, s69, v46",
               "v_mad_u64_u32 v[48:49], s[56:57], v47, 4, s[70:71]",
               "global_load_dword v50, v[48:49], off",
               "s_waitcnt vmcnt(0)",
               "v_cmp_le_i32 s[56:57], 0, v50", "s_and_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_gt_u32 s[56:57], 32, v54", "s_and_b64 s[54:55], s[54:55], s[56:57]",   # depth
               "s_and_b64 s[54:55], s[54:55], exec",
               # callers passing anything but their own ctx go to C++
               f"v_cmp_eq_u32 s[56:57], %[r1lo], v{R0 + 2}",
               f"v_cmp_eq_u32 vcc, %[r1hi], v{R0 + 3}", "s_and_b64 s[56:57], s[56:57], vcc",
               "s_andn2_b64 s[56:57], s[54:55], s[56:57]", f"s_cbranch_scc1 {L('slow')}",
               "s_lshr_b32 s49, s48, 5", "s_add_u32 s49, s49, 1",           # return pc
               "s_mov_b64 s[60:61], exec",
               "s_and_b64 exec, exec, s[54:55]", f"s_cbranch_execz {noval}")
        # ---- push (a masked frame, common.hpp kFrameMasked): the caller's
        # live registers (FInsn imm), the header, the ctx / stack words the
        # image's targets may write (tenv masks); the lanes at a depth below
        # s47 & 0xff into their LDS frame (common.hpp kTailLdsMax), the others
        # into global memory ----
        nog, nol = self.label("tng"), self.label("tnl")
        self.e("s_lshl_b32 s69, s42, 8", "s_or_b32 s69, s69, 0x100",              # masked | live << 8
               "v_mov_b32 v44, s49", "v_mov_b32 v45, s69",
               "s_and_b32 s69, s47, 0xff",
               "v_cmp_gt_u32 s[64:65], s69, v54", "s_and_b64 s[64:65], s[64:65], exec",
               "s_andn2_b64 s[66:67], exec, s[64:65]",
               "s_mov_b64 exec, s[66:67]", f"s_cbranch_execz {nog}")
        self.frame_ptr()
        for r in range(1, 10):
            skip = self.label("tpr")
            self.e(f"s_bitcmp1_b32 s42, {r}", f"s_cbranch_scc0 {skip}")
            self.word_addr(r - 1)
            self.e(f"global_store_dwordx2 v[58:59], v[{R0 + 2 * r}:{R0 + 2 * r + 1}], off", f"{skip}:")
        self.word_addr(11)
        self.e("global_store_dwordx2 v[58:59], v[44:45], off")
        for k in range(6):
            skip = self.label("tpc")
            self.e(f"s_bitcmp1_b32 s68, {k}", f"s_cbranch_scc0 {skip}",
                   f"ds_read_b64 v[42:43], v{R0 + 2} offset:{8 * k}", "s_waitcnt lgkmcnt(0)")
            self.word_addr(12 + k)
            self.e("global_store_dwordx2 v[58:59], v[42:43], off", f"{skip}:")
        self.stack_words(store=True)
        self.e(f"{nog}:", "s_mov_b64 exec, s[64:65]", f"s_cbranch_execz {nol}")
        self.lds_frame_ptr()
        self.e("ds_write_b64 v41, v[44:45]", "v_add_u32 v48, 0x800, v41")
        # the live registers (s42 bits 1..9), then the ctx words of the mask
        # (s68 bits 0..5), one loop trip per word
        lr, ld, lc, lcd = self.label("tlr"), self.label("tlrd"), self.label("tlc"), self.label("tlcd")
        self.e("s_and_b32 s70, s42, 0x3fe",
               f"{lr}:", "s_cmp_eq_u32 s70, 0", f"s_cbranch_scc1 {ld}",
               "s_ff1_i32_b32 s69, s70", "s_bitset0_b32 s70, s69", "s_lshl_b32 s71, s69, 1")
        self.rd("s71", 42)
        self.e("ds_write_b64 v48, v[42:43]", "v_add_u32 v48, 0x800, v48", f"s_branch {lr}",
               f"{ld}:",
               "s_and_b32 s70, s68, 0x3f",
               f"{lc}:", "s_cmp_eq_u32 s70, 0", f"s_cbranch_scc1 {lcd}",
               "s_ff1_i32_b32 s69, s70", "s_bitset0_b32 s70, s69", "s_lshl_b32 s71, s69, 3",
               f"v_add_u32 v49, s71, v{R0 + 2}",
               "ds_read_b64 v[42:43], v49", "s_waitcnt lgkmcnt(0)",
               "ds_write_b64 v48, v[42:43]", "v_add_u32 v48, 0x800, v48", f"s_branch {lc}",
               f"{lcd}:")
        self.e("s_and_b32 s71, s85, 0xffff")
        self.lds_stack_words(store=True, mask="s71")
        self.e(f"{nol}:", "s_mov_b64 exec, s[54:55]")
        self.e("v_add_u32 v54, 1, v54", f"ds_write_b32 v40, v54 offset:{self.depth_off}",
               f"v_mov_b32 v{R0}, 0", f"v_mov_b32 v{R0 + 1}, 0",
               f"v_mov_b32 v{R0 + 4}, 64", f"v_mov_b32 v{R0 + 5}, 0",
               f"v_mov_b32 v{R0 + 20}, %[r10lo]", f"v_mov_b32 v{R0 + 21}, %[r10hi]")
        for r in range(3, 10):
            self.e(f"v_mov_b32 v{R0 + 2 * r}, 0", f"v_mov_b32 v{R0 + 2 * r + 1}, 0")
        self.e("v_lshlrev_b32 v50, 5, v50",                                 # target IP
               f"{noval}:",
               "s_andn2_b64 exec, s[60:61], s[54:55]", f"s_cbranch_execz {ni}",
               f"v_mov_b32 v{R0}, -1", f"v_mov_b32 v{R0 + 1}, -1",
               "s_lshl_b32 s69, s49, 5", "v_mov_b32 v50, s69",
               f"{ni}:", "s_mov_b64 exec, s[60:61]")
        self.go_groups()

    def tail_ret(self):
        """A linked target's exit (kRetHelper): pop a masked frame (the live
        registers its header names, the image's ctx / stack words), r10 =
        the stack top, r0 stays the target's result, continue after the
        tail call.  Full frames (pushed by C++) leave for C++."""
        self.tail_env()
        self.e("s_bitcmp1_b32 s68, 31", f"s_cbranch_scc1 {L('slow')}",
               "v_cmp_eq_u32 s[54:55], 0, v54", "s_and_b64 s[54:55], s[54:55], exec",
               f"s_cbranch_scc1 {L('slow')}",                                # no frame: C++ fails the lane
               "v_add_u32 v54, -1, v54",
               # s[52:53]: lanes whose frame is in LDS (depth < s47 & 0xff;
               # its header 0: a full frame in global memory, left for C++),
               # s[56:57]: the others
               "s_and_b32 s69, s47, 0xff",
               "v_cmp_gt_u32 s[52:53], s69, v54", "s_and_b64 s[52:53], s[52:53], exec",
               "s_andn2_b64 s[56:57], exec, s[52:53]")
        h1, h2 = self.label("trh1"), self.label("trh2")
        self.e("s_mov_b64 exec, s[52:53]", f"s_cbranch_execz {h1}")
        self.lds_frame_ptr()
        self.e("ds_read_b64 v[46:47], v41",
               f"{h1}:", "s_mov_b64 exec, s[56:57]", f"s_cbranch_execz {h2}",
               "s_waitcnt vmcnt(0)")
        self.frame_ptr()
        self.word_addr(11)
        self.e("global_load_dwordx2 v[46:47], v[58:59], off",                 # return pc | flags
               f"{h2}:", "s_or_b64 exec, s[52:53], s[56:57]",
               "s_waitcnt vmcnt(0) lgkmcnt(0)",
               "v_and_b32 v49, 0x100, v47", "v_cmp_ne_u32 vcc, 0, v49",
               "s_andn2_b64 s[54:55], exec, vcc", f"s_cbranch_scc1 {L('slow')}",
               f"ds_write_b32 v40, v54 offset:{self.depth_off}",
               "v_lshlrev_b32 v50, 5, v46")                                  # return IP
        # ---- global frames: the live registers the header names, the
        # image's ctx / stack words ----
        ng = self.label("trng")
        self.e("s_mov_b64 exec, s[56:57]", f"s_cbranch_execz {ng}", "s_mov_b64 s[60:61], exec")
        for r in range(1, 10):
            skip = self.label("trr")
            self.e("s_mov_b64 exec, s[60:61]",
                   f"v_and_b32 v49, {1 << (8 + r)}, v47", "v_cmp_ne_u32 vcc, 0, v49",
                   "s_and_b64 exec, s[60:61], vcc", f"s_cbranch_execz {skip}")
            self.word_addr(r - 1)
            self.e(f"global_load_dwordx2 v[{R0 + 2 * r}:{R0 + 2 * r + 1}], v[58:59], off", f"{skip}:")
        self.e("s_mov_b64 exec, s[60:61]")
        # the first saved ctx word and the first saved stack word load with
        # the registers (one memory round trip for the usual frame: a live
        # register, a ctx field, a stack word); the others one at a time.
        # s64 / s66: ctx / stack words left; s65: the first ctx word's byte
        # offset, s67: the first stack word's index (-1: none)
        c0, s0, cw, sw = self.label("trc0"), self.label("trs0"), self.label("trcw"), self.label("trsw")
        self.e("s_and_b32 s64, s68, 0x3f", "s_mov_b32 s65, -1",
               "s_cmp_eq_u32 s64, 0", f"s_cbranch_scc1 {c0}",
               "s_ff1_i32_b32 s69, s64", "s_bitset0_b32 s64, s69",
               "s_lshl_b32 s65, s69, 3",
               "s_add_u32 s69, s69, 12", "s_mul_i32 s69, s69, s76",
               "v_add_co_u32 v58, vcc, s69, v56", "v_addc_co_u32 v59, vcc, 0, v57, vcc",
               "global_load_dwordx2 v[42:43], v[58:59], off",
               f"{c0}:",
               "s_and_b32 s66, s85, 0xffff", "s_mov_b32 s67, -1",
               "s_cmp_eq_u32 s66, 0", f"s_cbranch_scc1 {s0}",
               "s_ff1_i32_b32 s67, s66", "s_bitset0_b32 s66, s67",
               "s_add_u32 s69, s67, 20", "s_mul_i32 s69, s69, s76",
               "v_add_co_u32 v58, vcc, s69, v56", "v_addc_co_u32 v59, vcc, 0, v57, vcc",
               "global_load_dwordx2 v[44:45], v[58:59], off",
               f"{s0}:",
               "s_waitcnt vmcnt(0)",
               "s_cmp_lt_i32 s65, 0", f"s_cbranch_scc1 {cw}",
               "v_add_u32 v41, s65, %[r1lo]", "ds_write_b64 v41, v[42:43]",
               f"{cw}:",
               "s_cmp_lt_i32 s67, 0", f"s_cbranch_scc1 {sw}",
               "s_lshr_b32 s69, s85, 16", "v_subrev_u32 v41, s69, %[stklo]",  # the stack bottom
               "s_lshl_b32 s69, s67, 3", "v_add_u32 v41, s69, v41",
               "ds_write_b64 v41, v[44:45]",
               f"{sw}:")
        loop, done = self.label("trcl"), self.label("trcd")
        self.e(f"{loop}:", "s_cmp_eq_u32 s64, 0", f"s_cbranch_scc1 {done}",
               "s_ff1_i32_b32 s69, s64", "s_bitset0_b32 s64, s69",
               "s_lshl_b32 s65, s69, 3",
               "s_add_u32 s69, s69, 12", "s_mul_i32 s69, s69, s76",
               "v_add_co_u32 v58, vcc, s69, v56", "v_addc_co_u32 v59, vcc, 0, v57, vcc",
               "global_load_dwordx2 v[42:43], v[58:59], off", "s_waitcnt vmcnt(0)",
               "v_add_u32 v41, s65, %[r1lo]", "ds_write_b64 v41, v[42:43]",
               f"s_branch {loop}", f"{done}:")
        self.stack_words(store=False, mask="s66")
        self.e("s_waitcnt vmcnt(0) lgkmcnt(0)")
        # ---- LDS frames: the same words in order from word 1 ----
        nl = self.label("trnl")
        self.e(f"{ng}:", "s_mov_b64 exec, s[52:53]", f"s_cbranch_execz {nl}",
               "v_add_u32 v48, 0x800, v41")
        # the live registers the header names: one loop trip each when every
        # lane's header is the same (one call site), else per register
        gen_, uni, ur, urd, regs_done = (self.label(x) for x in ("tlg", "tlu", "tlur", "tlurd", "tlrd"))
        self.e("v_readfirstlane_b32 s70, v47", "v_cmp_ne_u32 vcc, s70, v47", "s_and_b64 vcc, vcc, exec",
               f"s_cbranch_vccnz {gen_}",
               f"{uni}:", "s_lshr_b32 s70, s70, 8", "s_and_b32 s70, s70, 0x3fe",
               f"{ur}:", "s_cmp_eq_u32 s70, 0", f"s_cbranch_scc1 {urd}",
               "s_ff1_i32_b32 s69, s70", "s_bitset0_b32 s70, s69", "s_lshl_b32 s71, s69, 1",
               "ds_read_b64 v[42:43], v48", "v_add_u32 v48, 0x800, v48", "s_waitcnt lgkmcnt(0)")
        self.wr("s71", 42)
        self.e(f"s_branch {ur}", f"{urd}:", f"s_branch {regs_done}", f"{gen_}:")
        for r in range(1, 10):
            skip = self.label("tlr")
            self.e("s_mov_b64 exec, s[52:53]",
                   f"v_and_b32 v49, {1 << (8 + r)}, v47", "v_cmp_ne_u32 vcc, 0, v49",
                   "s_and_b64 exec, s[52:53], vcc", f"s_cbranch_execz {skip}",
                   f"ds_read_b64 v[{R0 + 2 * r}:{R0 + 2 * r + 1}], v48", "v_add_u32 v48, 0x800, v48", f"{skip}:")
        lc, lcd = self.label("tlc"), self.label("tlcd")
        self.e(f"{regs_done}:", "s_mov_b64 exec, s[52:53]",
               "s_and_b32 s70, s68, 0x3f",
               f"{lc}:", "s_cmp_eq_u32 s70, 0", f"s_cbranch_scc1 {lcd}",
               "s_ff1_i32_b32 s69, s70", "s_bitset0_b32 s70, s69", "s_lshl_b32 s71, s69, 3",
               "ds_read_b64 v[42:43], v48", "v_add_u32 v48, 0x800, v48",
               "v_add_u32 v49, s71, %[r1lo]", "s_waitcnt lgkmcnt(0)",
               "ds_write_b64 v49, v[42:43]", f"s_branch {lc}",
               f"{lcd}:")
        self.e("s_and_b32 s71, s85, 0xffff")
        self.lds_stack_words(store=False, mask="s71")
        self.e("s_waitcnt lgkmcnt(0)",
               f"{nl}:", "s_or_b64 exec, s[52:53], s[56:57]",
               f"v_mov_b32 v{R0 + 20}, %[r10lo]", f"v_mov_b32 v{R0 + 21}, %[r10hi]")
        # registers that held the lane's own ctx pointer at the call
        # (header bits 50 + r, common.hpp kFrameRematShift): set again
        nr = self.label("trnr")
        self.e("v_and_b32 v49, 0x0ff80000, v47", "v_cmp_ne_u32 vcc, 0, v49", "s_and_b64 vcc, vcc, exec",
               f"s_cbranch_vccz {nr}", "s_mov_b64 s[60:61], exec")
        for r in range(1, 10):
            self.e("s_mov_b64 exec, s[60:61]",
                   f"v_and_b32 v49, {1 << (18 + r)}, v47", "v_cmp_ne_u32 vcc, 0, v49", "s_and_b64 exec, s[60:61], vcc",
                   f"v_mov_b32 v{R0 + 2 * r}, %[r1lo]", f"v_mov_b32 v{R0 + 2 * r + 1}, %[r1hi]")
        self.e("s_mov_b64 exec, s[60:61]", f"{nr}:")
        self.go_groups()

    # ---- divergence: min-pc scheduling of lane groups ----
    # A split branch leaves the wave as the running group (IP, exec) plus up
    # to three pending groups (PIP = IPs, PM = lane masks, s92 = count),
    # sorted by IP.  The running group always has the lowest
    # pc; while any group is pending, dispatch goes through the divergent
    # table, whose entries compare IP with the first pending IP: equal -> the
    # groups merge (reconvergence), greater -> the running group is parked
    # and the pending one runs.  A fourth pending group, or any instruction
    # the asm does not run, hands every group's pc to the C++ divergent loop
    # (exit reason 3).
    def set_table(self, divergent):
        """Dispatch into the handlers' divergent stubs (8 bytes in front of
        each handler) or straight into the handlers."""
        if divergent:
            self.e("s_sub_u32 s50, s50, 8", "s_subb_u32 s51, s51, 0")
        else:
            self.e("s_add_u32 s50, s50, 8", "s_addc_u32 s51, s51, 0")

    def pop0(self):
        keep = self.label("keep")
        for i in range(KP - 1):
            self.e(f"s_mov_b32 {PIP[i]}, {PIP[i + 1]}", f"s_mov_b64 {PM[i]}, {PM[i + 1]}")
        self.e(f"s_mov_b32 {PIP[KP - 1]}, -1",
               "s_sub_u32 s92, s92, 1", "s_cmp_eq_u32 s92, 0", f"s_cbranch_scc0 {keep}")
        self.set_table(False)
        self.e(f"{keep}:")

    def push(self):
        """Park group (s69 = IP, s[62:63] = lanes): merged into a pending
        group at the same IP, else inserted in IP order (s49 / s[56:57]
        scratch); a full list leaves for C++ (overflow)."""
        done, ins, first = self.label("pd"), self.label("pi"), self.label("pf")
        for i in range(KP):
            nx = self.label("pm")
            self.e(f"s_cmp_gt_u32 s92, {i}", f"s_cbranch_scc0 {ins}",
                   f"s_cmp_eq_u32 s69, {PIP[i]}", f"s_cbranch_scc0 {nx}",
                   f"s_or_b64 {PM[i]}, {PM[i]}, s[62:63]", f"s_branch {done}", f"{nx}:")
        self.e(f"{ins}:", f"s_cmp_ge_u32 s92, {KP}", f"s_cbranch_scc1 {L('overflow')}",
               "s_cmp_eq_u32 s92, 0", f"s_cbranch_scc0 {first}")
        self.set_table(True)
        self.e(f"{first}:")
        for n in range(KP):  # append at index n = count, then bubble towards the front
            nx = self.label("pa")
            self.e(f"s_cmp_eq_u32 s92, {n}", f"s_cbranch_scc0 {nx}",
                   f"s_mov_b32 {PIP[n]}, s69", f"s_mov_b64 {PM[n]}, s[62:63]", f"s_add_u32 s92, s92, 1")
            for j in range(n, 0, -1):
                self.e(f"s_cmp_lt_u32 {PIP[j]}, {PIP[j - 1]}", f"s_cbranch_scc0 {done}",
                       f"s_mov_b32 s49, {PIP[j]}", f"s_mov_b32 {PIP[j]}, {PIP[j - 1]}", f"s_mov_b32 {PIP[j - 1]}, s49",
                       f"s_mov_b64 s[56:57], {PM[j]}", f"s_mov_b64 {PM[j]}, {PM[j - 1]}",
                       f"s_mov_b64 {PM[j - 1]}, s[56:57]")
            self.e(f"s_branch {done}", f"{nx}:")
        self.e(f"{done}:")

    def materialize(self, extra):
        """Every group's pc (FInsn index) into the lpc output of its lanes,
        exec = all of them; exit reason 3."""
        self.e("s_lshr_b32 s52, s48, 5", "v_mov_b32 %[lpc], s52",
               "s_mov_b64 s[60:61], exec")
        if extra:
            self.e("s_mov_b64 exec, s[62:63]", "s_lshr_b32 s52, s69, 5",
                   "v_mov_b32 %[lpc], s52", "s_or_b64 s[60:61], s[60:61], exec")
        self.materialize_pending()
        self.e("s_mov_b64 exec, s[60:61]", "s_mov_b32 s68, 3", f"s_branch {L('spill')}")

    def materialize_pending(self):
        """lpc of the pending groups' lanes; s[60:61] |= their masks."""
        for i in range(KP):
            skip = self.label("mz")
            self.e(f"s_cmp_ge_u32 s92, {i + 1}", f"s_cbranch_scc0 {skip}",
                   f"s_mov_b64 exec, {PM[i]}", f"s_lshr_b32 s52, {PIP[i]}, 5",
                   "v_mov_b32 %[lpc], s52", "s_or_b64 s[60:61], s[60:61], exec", f"{skip}:")

    def divergence_routines(self):
        back, spush, ahead = self.label("sback"), self.label("spush"), self.label("dahead")
        # split branch: vcc = taken lanes, W = the branch
        self.e(f"{L('split')}:",
               "s_bitcmp1_b32 %[entry], 2", f"s_cbranch_scc0 {L('slow')}",
               "s_andn2_b64 s[56:57], exec, vcc",
               f"s_add_u32 s48, s48, {INSN}",
               "s_cmp_lt_u32 s46, s48", f"s_cbranch_scc1 {back}",
               # forward: not-taken lanes run on, taken lanes wait at the target
               "s_mov_b32 s69, s46", "s_mov_b64 s[62:63], vcc", "s_mov_b64 exec, s[56:57]",
               f"s_branch {spush}",
               # backward (loop): taken lanes run on, the others wait after the branch
               f"{back}:",
               "s_mov_b32 s69, s48", "s_mov_b64 s[62:63], s[56:57]", "s_mov_b64 exec, vcc",
               "s_mov_b32 s48, s46",
               "s_add_u32 %[steps], %[steps], 1",
               "s_cmp_gt_u32 %[steps], %[limit]", f"s_cbranch_scc1 {L('steps')}",
               f"{spush}:")
        self.push()
        self.dispatch()
        # divergent dispatch (build: the divergent table's per-handler
        # stubs): the running group reached the first pending IP
        self.e(f"{L('dswitch')}:",
               "s_waitcnt lgkmcnt(0)",       # the fall-through fetch lands before another
               "s_cmp_eq_u32 s48, s86", f"s_cbranch_scc0 {ahead}",
               "s_or_b64 exec, exec, s[88:89]")                # reconvergence
        self.pop0()
        self.dispatch()
        self.e(f"{ahead}:",
               "s_mov_b32 s69, s48", "s_mov_b64 s[62:63], exec",
               "s_mov_b32 s48, s86", "s_mov_b64 exec, s[88:89]")
        self.pop0()
        self.push()
        self.dispatch()
        self.e(f"{L('overflow')}:")
        self.materialize(extra=True)

    def build(self):
        ids = handler_ids()
        e = self.e
        fresh, loaded = L("fresh"), self.label("loaded")
        # ---- entry ----
        # (M0: s_set_gpr_idx_on writes it; the compiler's value is kept in an
        # operand register and restored at the exit, so M0 is no clobber)
        e("s_mov_b32 %[m0s], m0",
          "s_mov_b64 s[78:79], %[prog]",
          "v_mov_b32 v40, %[rb]",
          "s_lshl_b32 s48, %[pc], 5",
          "s_mov_b64 s[58:59], exec", "s_mov_b64 exec, %[alive]")
        # the host linker's query (entry = ~0, which no unit's entry is: its
        # RAW and SYSCALL bits exclude each other): every handler's offset
        # from the handler base, u32 per id at the vaddr operand
        # (vm_api.cpp fast_xlat), then out
        nq = self.label("nq")
        e("s_cmp_eq_u32 %[entry], -1", f"s_cbranch_scc0 {nq}")
        for i, name in enumerate(handler_ids()):
            e(f"v_mov_b32 v56, ({L('d_' + name)} - {L('hbase')})",
              f"global_store_dword %[vaddr], v56, off offset:{4 * i}")
        e("s_mov_b32 s48, 0", "s_mov_b32 s68, 0", f"s_branch {L('done')}", f"{nq}:")
        e("s_mov_b32 s80, 0", "s_mov_b32 s81, 0", "s_mov_b32 s84, 0", "s_mov_b32 s92, 0",
          "s_mov_b32 s86, -1", "s_mov_b32 s87, -1", "s_mov_b32 s93, -1",
          "v_mov_b32 v52, %[slotlo]", "v_mov_b32 v53, %[slothi]",
          "s_bitcmp1_b32 %[entry], 0", f"s_cbranch_scc1 {fresh}")
        # re-entry: registers from the C++ side's LDS copy, no staging
        if self.greg:
            self.rgb()
        for r in range(NREG):
            if self.greg:
                e(f"v_add_u32 v41, {r * 2048}, v40",
                  f"global_load_dwordx2 v[{R0 + 2 * r}:{R0 + 2 * r + 1}], v41, s[52:53]")
            else:
                e(f"ds_read_b64 v[{R0 + 2 * r}:{R0 + 2 * r + 1}], v40 offset:{r * 2048}")
        e("s_waitcnt vmcnt(0) lgkmcnt(0)", f"s_branch {loaded}")
        # fresh unit: r1, r2, r10 from operands, the rest zero; stage the slot
        e(f"{fresh}:")
        for r in range(NREG):
            if r == 1:
                e(f"v_mov_b32 v{R0 + 2}, %[r1lo]", f"v_mov_b32 v{R0 + 3}, %[r1hi]")
            elif r == 2:
                e(f"v_mov_b32 v{R0 + 4}, %[r2lo]", f"v_mov_b32 v{R0 + 5}, 0")
            elif r == 10:
                e(f"v_mov_b32 v{R0 + 20}, %[r10lo]", f"v_mov_b32 v{R0 + 21}, %[r10hi]")
            else:
                e(f"v_mov_b32 v{R0 + 2 * r}, 0", f"v_mov_b32 v{R0 + 2 * r + 1}, 0")
        # raw / syscall units: r1 = the slot, r2 = the length (chained units)
        n1, n2 = self.label("nr1"), self.label("nr2")
        e("s_bitcmp1_b32 %[entry], 3", f"s_cbranch_scc0 {n1}",
          f"v_mov_b32 v{R0 + 2}, v52", f"v_mov_b32 v{R0 + 3}, v53",
          f"{n1}:",
          "s_bitcmp1_b32 %[entry], 4", f"s_cbranch_scc0 {n2}",
          f"v_mov_b32 v{R0 + 4}, %[ulen]",
          f"{n2}:")
        filt, fsv, fsr = self.label("filt"), self.label("fsv"), self.label("fsr")
        e("s_bitcmp1_b32 %[entry], 1", f"s_cbranch_scc0 {loaded}",
          "s_mov_b32 s80, %[stage]",
          f"global_load_dwordx4 v[{STG}:{STG + 3}], v[52:53], off" + SLOT_POLICY)
        for c in range(1, 4):
            e(f"s_cmp_lt_u32 %[stage], {16 * (c + 1)}", f"s_cbranch_scc1 {filt}",
              f"global_load_dwordx4 v[{STG + 4 * c}:{STG + 4 * c + 3}], v[52:53], off offset:{16 * c}"
              + SLOT_POLICY)
        # syscall records (entry bit 6) of a staged unit: exit / exit_group
        # lanes (nr = bytes 8..15, syscall_trace_attach_impl.cpp:25) finish
        # with r0 = 0 here, from the staged bytes, instead of a separate load
        # of nr before the staging loads (chain_routine: unstaged units)
        fchk = self.label("fchk")
        e(f"{filt}:",
          # a chained unit's length load (chain_routine) completes with the
          # staging loads: one memory round trip per unit instead of two
          "s_bitcmp1_b32 %[entry], 5", f"s_cbranch_scc0 {fchk}",
          "s_waitcnt vmcnt(0)",
          f"{fchk}:",
          "s_bitcmp1_b32 %[entry], 6", f"s_cbranch_scc0 {loaded}",
          "s_waitcnt vmcnt(0)",
          f"v_cmp_eq_u64 s[54:55], 60, v[{STG + 2}:{STG + 3}]",
          "s_movk_i32 s70, 0xe7", "s_mov_b32 s71, 0",
          f"v_cmp_eq_u64 s[56:57], s[70:71], v[{STG + 2}:{STG + 3}]",
          "s_or_b64 s[54:55], s[54:55], s[56:57]",
          "s_and_b64 s[54:55], s[54:55], exec",
          f"s_cbranch_scc0 {loaded}",
          "s_andn2_b64 s[60:61], exec, s[54:55]",
          "s_mov_b64 exec, s[54:55]",
          "v_mov_b32 v56, 0", "v_mov_b32 v57, 0",
          "s_bitcmp1_b32 %[oflags], 0", f"s_cbranch_scc0 {fsv}",
          "global_store_dword %[vaddr], v56, off",
          f"{fsv}:",
          "s_bitcmp1_b32 %[oflags], 1", f"s_cbranch_scc0 {fsr}",
          "global_store_dwordx2 %[raddr], v[56:57], off",
          f"{fsr}:",
          "s_mov_b64 exec, s[60:61]",
          f"s_cbranch_execnz {loaded}",
          "s_mov_b32 s84, 0", f"s_branch {L('chain')}")                  # every lane an exit record
        # Direct dispatch: an FInsn's handler offset (and the next one's, in
        # w1) is its handler's divergent stub's distance from the 64-aligned
        # handler base (the host linker learns the distances from the asm
        # itself: the query above); each stub is 8 bytes in front of its
        # handler, so s[50:51] = base + 8 jumps straight into handlers and
        # base + 0 (set_table, while lane groups are pending) into the stubs.
        here = self.label("here")
        e(f"{loaded}:",
          "s_getpc_b64 s[50:51]",
          f"{here}:",
          f"s_add_u32 s50, s50, ({L('hbase')} - {here} + 8)",
          "s_addc_u32 s51, s51, 0",
          f"s_branch {L('start')}")
        e(f"{L('start')}:")
        self.dispatch()
        # ---- handlers, each behind its divergent stub: the running group
        # has reached the first pending group's IP (s86) -> dswitch, else on
        # into the handler ----
        e(".p2align 6", f"{L('hbase')}:")
        for name in ids:
            if HANDLER_ALIGN:
                e(f".p2align {HANDLER_ALIGN}")
            e(f"{L('d_' + name)}:", "s_cmp_ge_u32 s48, s86", f"s_cbranch_scc1 {L('dswitch')}")
            e(f"{L('h_' + name)}:", "s_waitcnt lgkmcnt(0)")  # W of a fall-through fetch
            if name == "SLOW":
                e(f"s_branch {L('slow')}")
            elif name == "ATOMMV8_ADD2":
                self.atomic_pair()
            elif name.startswith("ATOMD"):
                self.atomd(int(name[5]))
            elif name.startswith("ATOMMV"):
                self.atomic(int(name[6]), "ADD", False, mv=True)
            elif name.startswith("ATOM"):
                parts = name.split("_")
                self.atomic(int(parts[0][4:]), parts[1], len(parts) == 3)
            elif name in ("A64_NEG", "A32_NEG"):
                self.neg(name[1:3])
            elif name[0] == "A":
                w, op, k = name[1:3], name.split("_")[1], name.split("_")[2]
                self.alu(w, op, k)
            elif name in ("LE16", "LE32", "BE16", "BE32", "BE64"):
                self.endian(name)
            elif name == "NOP":
                self.next_seq()
            elif name == "LEA":
                self.lea()
            elif name in ("LDX_CTXDATA", "LDX_CTXEND"):
                self.ctx_field(name == "LDX_CTXEND")
            elif name in STAGED_LD:
                self.ldxs(name)
            elif name in STAGED_ST:
                self.stxs(name)
            elif (name.endswith("_STK") or name.endswith("_CTX")) and not name.startswith("CALL"):
                op = name.split("_")[0]
                base = "%[r1lo]" if name.endswith("_CTX") else "%[stklo]"
                if op.startswith("LDX"):
                    self.ldx_stk(int(op[3:]), base)
                elif op.startswith("STX"):
                    self.store_stk(int(op[3:]), True, base)
                else:
                    self.store_stk(int(op[2:]), False, base)
            elif name.endswith("_MV"):
                op = name.split("_")[0]
                if op.startswith("LDX"):
                    self.ldx_mv(int(op[3:]))
                else:
                    self.stx_mv(int(op[3:]))
            elif name.startswith("LDX"):
                self.ldx(int(name[3:]))
            elif name.startswith("STX"):
                self.store(int(name[3:]), True)
            elif name.startswith("ST"):
                self.store(int(name[2:]), False)
            elif name == "LDDW":
                self.lddw()
            elif name == "JA":
                self.jump_taken("s42")
            elif name == "CALL_LOOKUP":
                self.call_lookup()
            elif name in ("CALL_LOOKUP_STK3", "CALL_LOOKUP_AK3"):
                # r1 = the map fd (w7), r2 = r10 + the key's stack offset (w6),
                # then the lookup; the next FInsn is 5 slots on
                self.e(f"v_mov_b32 v{R0 + 2}, s47", f"v_mov_b32 v{R0 + 3}, 0",
                       "s_ashr_i32 s69, s46, 31",
                       f"v_add_co_u32 v{R0 + 4}, vcc, s46, v{R0 + 20}",
                       f"v_mov_b32 v{R0 + 5}, s69",
                       f"v_addc_co_u32 v{R0 + 5}, vcc, v{R0 + 5}, v{R0 + 21}, vcc")
                self.span = 5
                if name == "CALL_LOOKUP_AK3":
                    self.call_lookup_ak()
                else:
                    self.call_lookup(stack_key=True)
                self.span = 1
            elif name == "CALL_LOOKUP_STK":
                self.call_lookup(stack_key=True)
            elif name == "CALL_LOOKUP_AK":
                self.call_lookup_ak()
            elif name == "CALL_RBOUT":
                self.call_rbout()
            elif name == "EXIT":
                self.exit_()
            elif name == "TAIL":
                self.tail_call()
            elif name == "TRET":
                self.tail_ret()
            elif name == "CALL_PID":
                self.call_pid()
            elif name == "CALL_REC":
                self.call_rec()
            elif name == "CALL_UPDATE_STK":
                self.call_update_stk()
            elif name == "KLDX":
                self.ldxk()
            elif name.startswith("RMWD"):
                self.rmwd(int(name[4]), name[6])
            elif name.startswith("RMWMV"):
                self.rmw(int(name[5]), name[7], mv=True)
            elif name.startswith("RMWK"):
                self.rmwk(int(name[4]), name[6])
            elif name.startswith("RMW"):
                self.rmw(int(name[3]), name[5])
            elif name[0] == "J":
                w, cc, k = name[1:3], name.split("_")[1], name.split("_")[2]
                self.jcc(w, cc, k)
            else:
                raise ValueError(name)
        self.divergence_routines()
        self.chain_routine()
        # ---- exits: the instruction at pc was not executed; write back
        # staging, spill registers
        e(f"{L('steps')}:", "s_mov_b32 s68, 1")
        self.union_exec()
        e(f"s_branch {L('spill')}")
        e(f"{L('slow')}:", "s_mov_b32 s68, 0",
          "s_cmp_eq_u32 s92, 0", f"s_cbranch_scc1 {L('spill')}")
        self.materialize(extra=False)
        e(f"{L('spill')}:")
        self.flush()
        if self.greg:
            self.rgb()
        for r in range(NREG):
            if self.greg:
                e(f"v_add_u32 v41, {r * 2048}, v40",
                  f"global_store_dwordx2 v41, v[{R0 + 2 * r}:{R0 + 2 * r + 1}], s[52:53]")
            else:
                e(f"ds_write_b64 v40, v[{R0 + 2 * r}:{R0 + 2 * r + 1}] offset:{r * 2048}")
        e(f"{L('done')}:",
          "s_waitcnt vmcnt(0) lgkmcnt(0)",
          "s_mov_b64 %[aliveout], exec",
          "s_mov_b64 exec, s[58:59]",
          "s_lshr_b32 s52, s48, 5",
          "s_mov_b32 %[pc], s52", "s_mov_b32 %[why], s68",
          "s_mov_b32 m0, %[m0s]", "s_nop 0")
        return ids


def vmap(n):
    """Handlers are written against v40..v101; the block is placed at the top
    of a 128-VGPR budget (v66..v127, an even shift so register pairs stay
    aligned) so that the compiler's own values stay below it and the kernel
    keeps 4 waves per SIMD."""
    assert 40 <= n <= 101, n
    return n + 26


def relocate(line):
    line = re.sub(r"v\[(\d+):(\d+)\]", lambda m: f"v[{vmap(int(m.group(1)))}:{vmap(int(m.group(2)))}]", line)
    return re.sub(r"\bv(\d+)\b", lambda m: f"v{vmap(int(m.group(1)))}", line)


def inc_blocks(path):
    """The asm lines of each BPFTIME_AMD_FAST_ASM* macro of a written
    fast_asm.inc (what the kernel compiles)."""
    blocks, cur = {}, None
    for line in open(path):
        m = re.match(r"#define (BPFTIME_AMD_FAST_ASM\w*) \\$", line)
        if m:
            cur = blocks.setdefault(m.group(1), [])
            continue
        m = re.match(r'\s*"(.*)\\n" \\$', line)
        if m and cur is not None:
            cur.append(m.group(1))
        elif not line.startswith("  "):
            cur = None
    return blocks


def check_hazards(blocks):
    """hazards.py over each block; exits non-zero on a violation."""
    import hazards
    bad = []
    for name, lines in blocks.items():
        bad += [f"{name}: {v}" for v in hazards.check(lines)]
    if bad:
        raise SystemExit("wait-state hazards in the fast path:\n  " + "\n  ".join(bad))


def main():
    import sys
    if "--check" in sys.argv:  # (make: the committed fast_asm.inc, every build)
        blocks = inc_blocks(os.path.join(HERE, "fast_asm.inc"))
        assert len(blocks) == 2, sorted(blocks)
        check_hazards(blocks)
        print("fast_asm.inc: no wait-state hazards (%d lines)" % sum(len(b) for b in blocks.values()))
        return
    # v126/v127 (v100/v101 before relocation) are read, never written, by
    # staged loads near the window end
    clob = [f"s{i}" for i in range(40, 96)] + [f"v{vmap(i)}" for i in range(40, 102)]
    gens = {}
    for suffix, greg in (("", False), ("_G", True)):
        g = Gen(greg)
        ids = g.build()
        g.out = [relocate(x) for x in g.out]
        gens[suffix] = g
    check_hazards({"BPFTIME_AMD_FAST_ASM" + k: g.out for k, g in gens.items()})
    with open(os.path.join(HERE, "fast_asm.inc"), "w") as f:
        f.write("// Generated by gen_fast.py; do not edit.\n")
        # register spill copy in LDS, and (_G) in global memory
        for suffix, g in gens.items():
            f.write("#define BPFTIME_AMD_FAST_ASM%s \\\n" % suffix)
            for line in g.out:
                f.write('  "%s\\n" \\\n' % line)
            f.write('  ""\n')
        f.write("#define BPFTIME_AMD_FAST_CLOBBERS %s\n" %
                ", ".join('"%s"' % c for c in clob + ["vcc", "scc", "memory"]))
    with open(os.path.join(HERE, "fast_ops.hpp"), "w") as f:
        f.write("// Generated by gen_fast.py; do not edit.\n#pragma once\n#include <stdint.h>\n\n")
        f.write("namespace bpftime_amd {\n\n// handler ids of the threaded fast path (FInsn::hoff = 4 + 4 * id)\nenum FOp : uint32_t {\n")
        for i, name in enumerate(ids):
            f.write(f"  F_{name} = {i},\n")
        f.write(f"  F_COUNT = {len(ids)}\n}};\n\n")
        f.write("// their names (BPFTIME_AMD_DUMP_FAST: vm_api.cpp prints a linked form)\n"
                "inline const char *fop_name(uint32_t id) {\n  static const char *const k[] = {\n")
        for name in ids:
            f.write(f'      "{name}",\n')
        f.write("  };\n  return id < F_COUNT ? k[id] : \"?\";\n}\n\n")
        f.write("// 32-byte threaded instruction (gen_fast.py register map, word for word):\n"
                "//   dst_x2 / src_x2 are eBPF register numbers times two (VGPR pair index);\n"
                "//   the staged / map-bound handlers reuse the fields as documented there\n"
                "struct FInsn {\n  uint32_t hoff;\n  uint32_t w1;\n  int64_t imm;\n  uint32_t dst_x2;\n"
                "  uint32_t src_x2;\n  uint32_t target;\n  int32_t aux;\n};\n"
                "static_assert(sizeof(FInsn) == 32, \"FInsn must be 32 bytes\");\n\n"
                f"constexpr uint32_t kFastInsnBytes = {INSN};\n"
                "constexpr uint32_t kFastStageBytes = 64;  // max staged bytes per unit\n\n"
                "}  // namespace bpftime_amd\n")


if __name__ == "__main__":
    main()
