"""Generates the gfx950 threaded-code fast path of the interpreter.

    python gen_fast.py  ->  fast_asm.inc, fast_ops.hpp   (run by the Makefile)

The uniform interpreter loop (every live lane of the wave at one pc) is one
inline-asm block.  Each eBPF instruction is pre-decoded by the loader into a
32-byte FInsn whose first word is the byte offset of its handler's entry in
a table of `s_branch` instructions; dispatch is

    s_load_dwordx8 W, IP          ; fetch (scalar cache)
    s_add_u32/s_addc_u32 T, TB, W0
    s_setpc_b64 T                 ; -> table entry -> handler

instead of a compare tree.  The handlers cover ALU64/ALU32 (reg and imm),
byte swaps, loads/stores of every size with the batch/arena/LDS window check,
lddw, ja and every conditional jump whose outcome is wave-uniform.  Anything
else (helper calls, exit, fused counters, atomics, div/mod, a split branch,
an access failing the window check) leaves the block at that pc, and the C++
interpreter executes that one instruction (interp.hip, run_loop<true, true>).

exec = the wave's live lanes inside the block, so compare results and
stores need no per-lane predication.

Register file: r0..r10 stay in LDS, lane-major (8 B per lane, 2 KiB per
register), so the C++ path and the asm path share one representation.

Fixed registers (declared as clobbers; the compiler keeps nothing live in
them across the block):
  s[40:47] W   current FInsn: w0 handler offset, w1 dst*2048, w[2:3] imm64,
               w4 src*2048, w5 jump target (byte offset from PROG), w[6:7] off64
  s[48:49] IP  address of the current FInsn     s[50:51] TB  table base - 4
  s[52:53] T   scratch / dispatch target        s[54:55], s[56:57], s[76:77] masks
  s[58:59] saved exec                            s[60:61] PROG (FInsn base)
  s[62:63]/s[64:65] batch window lo/hi           s[66:67]/s[68:69] map arena lo/hi
  s70 LDS aperture (address bits 63:32)          s71 scratch aperture
  s72 steps  s73 step limit  s74 exit reason  s75 scratch
  v40 lane's R[0] LDS address  v41/v42 register addresses
  v[44:45] X  v[46:47] Y  v[48:49] Z (address)  v[50:51] E (address end)
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

ALU_OPS = ["ADD", "SUB", "MUL", "OR", "AND", "XOR", "MOV", "LSH", "RSH", "ARSH"]
JCC = ["EQ", "GT", "GE", "SET", "NE", "SGT", "SGE", "LT", "LE", "SLT", "SLE"]
CMP64 = {"EQ": "eq_u64", "GT": "gt_u64", "GE": "ge_u64", "NE": "ne_u64", "SGT": "gt_i64",
         "SGE": "ge_i64", "LT": "lt_u64", "LE": "le_u64", "SLT": "lt_i64", "SLE": "le_i64"}
CMP32 = {k: v.replace("64", "32") for k, v in CMP64.items()}


def handler_ids():
    ids = ["SLOW"]
    for w in ("64", "32"):
        for op in ALU_OPS:
            for k in ("R", "I"):
                ids.append(f"A{w}_{op}_{k}")
        ids.append(f"A{w}_NEG")
    ids += ["LE16", "LE32", "BE16", "BE32", "BE64", "NOP"]
    for sz in (1, 2, 4, 8):
        ids += [f"LDX{sz}", f"STX{sz}", f"ST{sz}"]
    ids += ["LDDW", "JA"]
    for w in ("64", "32"):
        for cc in JCC:
            for k in ("R", "I"):
                ids.append(f"J{w}_{cc}_{k}")
    return ids


def L(name):
    return f".Lf%=_{name}"


class Gen:
    def __init__(self):
        self.out = []

    def e(self, *lines):
        self.out.extend(lines)

    # ---- building blocks ----
    def dispatch(self):
        """IP points at the next FInsn: fetch it and jump to its handler."""
        self.e("s_load_dwordx8 s[40:47], s[48:49], 0x0",
               "s_add_u32 s72, s72, 1",
               "s_waitcnt lgkmcnt(0)",
               "s_add_u32 s52, s50, s40",
               "s_addc_u32 s53, s51, 0",
               "s_setpc_b64 s[52:53]")

    def next_seq(self, slots=1):
        self.e(f"s_add_u32 s48, s48, {32 * slots}", "s_addc_u32 s49, s49, 0")
        self.dispatch()

    def jump_taken(self):
        self.e("s_add_u32 s48, s60, s45", "s_addc_u32 s49, s61, 0",
               "s_cmp_gt_u32 s72, s73", f"s_cbranch_scc1 {L('steps')}")
        self.dispatch()

    def read_dst(self):  # X = R[dst], v41 = &R[dst]
        self.e("v_add_u32 v41, s41, v40", "ds_read_b64 v[44:45], v41")

    def read_src(self):  # Y = R[src]
        self.e("v_add_u32 v42, s44, v40", "ds_read_b64 v[46:47], v42")

    def imm_y(self):     # Y = imm (sign-extended by the loader)
        self.e("v_mov_b32 v46, s42", "v_mov_b32 v47, s43")

    def write_dst(self):
        self.e("ds_write_b64 v41, v[44:45]")

    def check(self, sz):
        """Every live lane's [Z, Z+sz) inside the batch window, the map arena,
        or the LDS / scratch aperture; else leave for the C++ path (which
        fails the offending lanes)."""
        self.e(f"v_lshl_add_u64 v[50:51], v[48:49], 0, {sz}",
               "v_cmp_le_u64 s[54:55], s[62:63], v[48:49]",
               "v_cmp_ge_u64 s[56:57], s[64:65], v[50:51]",
               "s_and_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_le_u64 s[56:57], s[66:67], v[48:49]",
               "v_cmp_ge_u64 s[76:77], s[68:69], v[50:51]",
               "s_and_b64 s[56:57], s[56:57], s[76:77]",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_eq_u32 s[56:57], s70, v49",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "v_cmp_eq_u32 s[56:57], s71, v49",
               "s_or_b64 s[54:55], s[54:55], s[56:57]",
               "s_andn2_b64 s[54:55], exec, s[54:55]",
               f"s_cbranch_scc1 {L('slow')}")

    # ---- handlers ----
    def alu(self, w, op, k):
        if op != "MOV":
            self.read_dst()
        else:
            self.e("v_add_u32 v41, s41, v40")
        if k == "R":
            self.read_src()
        else:
            self.imm_y()
        self.e("s_waitcnt lgkmcnt(0)")
        if w == "64":
            body = {
                "ADD": ["v_lshl_add_u64 v[44:45], v[44:45], 0, v[46:47]"],
                "SUB": ["v_sub_co_u32 v44, vcc, v44, v46", "v_subb_co_u32 v45, vcc, v45, v47, vcc"],
                "MUL": ["v_mul_lo_u32 v48, v44, v47", "v_mul_lo_u32 v49, v45, v46",
                        "v_mul_hi_u32 v50, v44, v46", "v_mul_lo_u32 v44, v44, v46",
                        "v_add3_u32 v45, v48, v49, v50"],
                "OR": ["v_or_b32 v44, v44, v46", "v_or_b32 v45, v45, v47"],
                "AND": ["v_and_b32 v44, v44, v46", "v_and_b32 v45, v45, v47"],
                "XOR": ["v_xor_b32 v44, v44, v46", "v_xor_b32 v45, v45, v47"],
                "MOV": ["v_mov_b32 v44, v46", "v_mov_b32 v45, v47"],
                "LSH": ["v_lshlrev_b64 v[44:45], v46, v[44:45]"],   # shift count & 63 in hardware
                "RSH": ["v_lshrrev_b64 v[44:45], v46, v[44:45]"],
                "ARSH": ["v_ashrrev_i64 v[44:45], v46, v[44:45]"],
            }[op]
        else:
            body = {
                "ADD": ["v_add_u32 v44, v44, v46"],
                "SUB": ["v_sub_u32 v44, v44, v46"],
                "MUL": ["v_mul_lo_u32 v44, v44, v46"],
                "OR": ["v_or_b32 v44, v44, v46"],
                "AND": ["v_and_b32 v44, v44, v46"],
                "XOR": ["v_xor_b32 v44, v44, v46"],
                "MOV": ["v_mov_b32 v44, v46"],
                "LSH": ["v_lshlrev_b32 v44, v46, v44"],             # & 31 in hardware
                "RSH": ["v_lshrrev_b32 v44, v46, v44"],
                "ARSH": ["v_ashrrev_i32 v44, v46, v44"],
            }[op] + ["v_mov_b32 v45, 0"]                          # ALU32 zero-extends
        self.e(*body)
        self.write_dst()
        self.next_seq()

    def neg(self, w):
        self.read_dst()
        self.e("s_waitcnt lgkmcnt(0)")
        if w == "64":
            self.e("v_sub_co_u32 v44, vcc, 0, v44", "v_subb_co_u32 v45, vcc, 0, v45, vcc")
        else:
            self.e("v_sub_u32 v44, 0, v44", "v_mov_b32 v45, 0")
        self.write_dst()
        self.next_seq()

    def endian(self, name):
        self.read_dst()
        self.e("s_waitcnt lgkmcnt(0)")
        body = {
            "LE16": ["v_and_b32 v44, 0xffff, v44", "v_mov_b32 v45, 0"],
            "LE32": ["v_mov_b32 v45, 0"],
            "BE16": ["s_mov_b32 s75, 0x0c0c0001", "v_perm_b32 v44, 0, v44, s75", "v_mov_b32 v45, 0"],
            "BE32": ["s_mov_b32 s75, 0x00010203", "v_perm_b32 v44, 0, v44, s75", "v_mov_b32 v45, 0"],
            "BE64": ["s_mov_b32 s75, 0x00010203", "v_perm_b32 v48, 0, v45, s75",
                     "v_perm_b32 v45, 0, v44, s75", "v_mov_b32 v44, v48"],
        }[name]
        self.e(*body)
        self.write_dst()
        self.next_seq()

    def ldx(self, sz):
        self.read_src_as_addr()
        self.check(sz)
        ld = {1: "flat_load_ubyte v44, v[48:49]", 2: "flat_load_ushort v44, v[48:49]",
              4: "flat_load_dword v44, v[48:49]", 8: "flat_load_dwordx2 v[44:45], v[48:49]"}[sz]
        self.e(ld)
        if sz < 8:
            self.e("v_mov_b32 v45, 0")
        self.e("v_add_u32 v41, s41, v40", "s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.write_dst()
        self.next_seq()

    def read_src_as_addr(self):
        # Z = R[src] + off
        self.e("v_add_u32 v42, s44, v40", "ds_read_b64 v[48:49], v42", "s_waitcnt lgkmcnt(0)",
               "v_lshl_add_u64 v[48:49], v[48:49], 0, s[46:47]")

    def store(self, sz, from_reg):
        # Z = R[dst] + off ; value = R[src] or imm
        self.e("v_add_u32 v41, s41, v40", "ds_read_b64 v[48:49], v41")
        if from_reg:
            self.e("v_add_u32 v42, s44, v40", "ds_read_b64 v[44:45], v42")
        else:
            self.e("v_mov_b32 v44, s42", "v_mov_b32 v45, s43")
        self.e("s_waitcnt lgkmcnt(0)", "v_lshl_add_u64 v[48:49], v[48:49], 0, s[46:47]")
        self.check(sz)
        st = {1: "flat_store_byte v[48:49], v44", 2: "flat_store_short v[48:49], v44",
              4: "flat_store_dword v[48:49], v44", 8: "flat_store_dwordx2 v[48:49], v[44:45]"}[sz]
        self.e(st)
        self.next_seq()

    def lddw(self):
        self.e("v_add_u32 v41, s41, v40", "v_mov_b32 v44, s42", "v_mov_b32 v45, s43")
        self.write_dst()
        self.next_seq(2)

    def jcc(self, w, cc, k):
        self.read_dst()
        if k == "R":
            self.read_src()
        self.e("s_waitcnt lgkmcnt(0)")
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
            self.e("v_cmp_ne_u32 s[54:55], 0, v44")
        elif w == "64":
            self.e(f"v_cmp_{CMP64[cc]} s[54:55], v[44:45], {y64}")
        else:
            self.e(f"v_cmp_{CMP32[cc]} s[54:55], v44, {y32}")
        # v_cmp writes 0 for inactive lanes: none taken / all taken / split
        nt = L(f"nt_{w}_{cc}_{k}")
        self.e("s_cmp_eq_u64 s[54:55], 0", f"s_cbranch_scc1 {nt}",
               "s_cmp_eq_u64 s[54:55], exec", f"s_cbranch_scc0 {L('slow')}")
        self.jump_taken()
        self.e(f"{nt}:")
        self.next_seq()

    def build(self):
        ids = handler_ids()
        e = self.e
        # ---- entry: inputs into fixed registers ----
        e("s_mov_b64 s[60:61], %[prog]", "s_mov_b64 s[62:63], %[dlo]", "s_mov_b64 s[64:65], %[dhi]",
          "s_mov_b64 s[66:67], %[alo]", "s_mov_b64 s[68:69], %[ahi]", "s_mov_b32 s70, %[shi]",
          "s_mov_b32 s71, %[phi]", "s_mov_b32 s72, %[steps]", "s_mov_b32 s73, %[limit]",
          "v_mov_b32 v40, %[rb]",
          "s_lshl_b32 s52, %[pc], 5", "s_add_u32 s48, s60, s52", "s_addc_u32 s49, s61, 0",
          "s_mov_b64 s[58:59], exec", "s_mov_b64 exec, %[alive]",
          "s_getpc_b64 s[50:51]",          # = address of the s_branch below
          f"s_branch {L('start')}")
        for name in ids:                   # table: entry i at TB + 4 + 4*i
            e(f"s_branch {L('h_' + name)}")
        e(f"{L('start')}:")
        self.dispatch()
        # ---- handlers ----
        for name in ids:
            e(f"{L('h_' + name)}:")
            if name == "SLOW":
                e(f"s_branch {L('slow')}")
            elif name in ("A64_NEG", "A32_NEG"):
                self.neg(name[1:3])
            elif name[0] == "A":
                w, op, k = name[1:3], name.split("_")[1], name.split("_")[2]
                self.alu(w, op, k)
            elif name in ("LE16", "LE32", "BE16", "BE32", "BE64"):
                self.endian(name)
            elif name == "NOP":
                self.next_seq()
            elif name.startswith("LDX"):
                self.ldx(int(name[3:]))
            elif name.startswith("STX"):
                self.store(int(name[3:]), True)
            elif name.startswith("ST"):
                self.store(int(name[2:]), False)
            elif name == "LDDW":
                self.lddw()
            elif name == "JA":
                self.jump_taken()
            elif name[0] == "J":
                w, cc, k = name[1:3], name.split("_")[1], name.split("_")[2]
                self.jcc(w, cc, k)
            else:
                raise ValueError(name)
        # ---- exits: the instruction was not executed; one step was counted
        e(f"{L('steps')}:", "s_mov_b32 s74, 1", f"s_branch {L('exit')}")
        e(f"{L('slow')}:", "s_mov_b32 s74, 0", "s_sub_u32 s72, s72, 1")
        e(f"{L('exit')}:",
          "s_waitcnt vmcnt(0) lgkmcnt(0)",
          "s_mov_b64 exec, s[58:59]",
          "s_sub_u32 s52, s48, s60", "s_lshr_b32 s52, s52, 5",
          "s_mov_b32 %[pc], s52", "s_mov_b32 %[steps], s72", "s_mov_b32 %[why], s74")
        return ids


def main():
    g = Gen()
    ids = g.build()
    clob = [f"s{i}" for i in range(40, 78)] + [f"v{i}" for i in range(40, 52)]
    with open(os.path.join(HERE, "fast_asm.inc"), "w") as f:
        f.write("// Generated by gen_fast.py; do not edit.\n")
        f.write("#define BPFTIME_AMD_FAST_ASM \\\n")
        for line in g.out:
            f.write('  "%s\\n" \\\n' % line)
        f.write('  ""\n')
        f.write("#define BPFTIME_AMD_FAST_CLOBBERS %s\n" % ", ".join('"%s"' % c for c in clob + ["vcc", "scc", "memory"]))
    with open(os.path.join(HERE, "fast_ops.hpp"), "w") as f:
        f.write("// Generated by gen_fast.py; do not edit.\n#pragma once\n#include <stdint.h>\n\n")
        f.write("namespace bpftime_amd {\n\n// handler ids of the threaded fast path (FInsn::hoff = 4 + 4 * id)\nenum FOp : uint32_t {\n")
        for i, name in enumerate(ids):
            f.write(f"  F_{name} = {i},\n")
        f.write(f"  F_COUNT = {len(ids)}\n}};\n\n")
        f.write("// 32-byte threaded instruction (gen_fast.py register map, word for word)\n"
                "struct FInsn {\n  uint32_t hoff;\n  uint32_t dst_off;\n  int64_t imm;\n  uint32_t src_off;\n"
                "  uint32_t target;\n  int64_t off;\n};\n"
                "static_assert(sizeof(FInsn) == 32, \"FInsn must be 32 bytes\");\n\n}  // namespace bpftime_amd\n")


if __name__ == "__main__":
    main()
