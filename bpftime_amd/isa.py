"""eBPF instruction set: encoding, a label-aware assembler and a disassembler.

There is no BPF-target clang in this image, so every program the
tests and the bench run is assembled here.  Opcode values follow the table in
the reference's ``vm/compat/include/ebpf_inst.h:22-200`` (struct ebpf_inst at
:22-28: u8 code, u4 dst, u4 src, s16 off, s32 imm; little-endian, 8 bytes).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Union

# --- classes / fields (ebpf_inst.h:45-67) -----------------------------------
CLS_LD, CLS_LDX, CLS_ST, CLS_STX, CLS_ALU, CLS_JMP, CLS_JMP32, CLS_ALU64 = range(8)
SRC_IMM, SRC_REG = 0x00, 0x08
SIZE_W, SIZE_H, SIZE_B, SIZE_DW = 0x00, 0x08, 0x10, 0x18
MODE_IMM, MODE_MEM, MODE_ATOMIC = 0x00, 0x60, 0xC0

ALU_OPS = {
    "add": 0x00, "sub": 0x10, "mul": 0x20, "div": 0x30, "or": 0x40, "and": 0x50,
    "lsh": 0x60, "rsh": 0x70, "neg": 0x80, "mod": 0x90, "xor": 0xA0, "mov": 0xB0,
    "arsh": 0xC0,
}
JMP_OPS = {
    "ja": 0x00, "jeq": 0x10, "jgt": 0x20, "jge": 0x30, "jset": 0x40, "jne": 0x50,
    "jsgt": 0x60, "jsge": 0x70, "call": 0x80, "exit": 0x90, "jlt": 0xA0,
    "jle": 0xB0, "jslt": 0xC0, "jsle": 0xD0,
}
SIZES = {1: SIZE_B, 2: SIZE_H, 4: SIZE_W, 8: SIZE_DW}
SIZE_NAMES = {SIZE_B: "b", SIZE_H: "h", SIZE_W: "w", SIZE_DW: "dw"}
SIZE_BYTES = {SIZE_B: 1, SIZE_H: 2, SIZE_W: 4, SIZE_DW: 8}

# atomic op types in imm (ebpf_inst.h:29-42)
ATOMIC_ADD, ATOMIC_OR, ATOMIC_AND, ATOMIC_XOR = 0x00, 0x40, 0x50, 0xA0
ATOMIC_FETCH = 0x01
ATOMIC_XCHG = 0xE0 | ATOMIC_FETCH
ATOMIC_CMPXCHG = 0xF0 | ATOMIC_FETCH

OP_LDDW = CLS_LD | MODE_IMM | SIZE_DW  # 0x18
OP_CALL = CLS_JMP | 0x80  # 0x85
OP_EXIT = CLS_JMP | 0x90  # 0x95
OP_LE = CLS_ALU | SRC_IMM | 0xD0  # 0xd4
OP_BE = CLS_ALU | SRC_REG | 0xD0  # 0xdc

# lddw pseudo sources (compat_ubpf.cpp:113-185)
PSEUDO_MAP_FD, PSEUDO_MAP_VALUE, PSEUDO_VAR_ADDR, PSEUDO_CODE_ADDR = 1, 2, 3, 4
PSEUDO_MAP_IDX, PSEUDO_MAP_IDX_VALUE = 5, 6

# XDP verdicts (third_party/vmlinux/x86/vmlinux_601.h:29920-29924)
XDP_ABORTED, XDP_DROP, XDP_PASS, XDP_TX, XDP_REDIRECT = range(5)

# helper ids (runtime/src/bpf_helper.cpp:901-1114)
BPF_FUNC_map_lookup_elem = 1
BPF_FUNC_map_update_elem = 2
BPF_FUNC_map_delete_elem = 3
BPF_FUNC_ktime_get_ns = 5
BPF_FUNC_trace_printk = 6
BPF_FUNC_get_prandom_u32 = 7
BPF_FUNC_get_smp_processor_id = 8
BPF_FUNC_tail_call = 12
BPF_FUNC_get_current_pid_tgid = 14
BPF_FUNC_override_return = 58
BPF_FUNC_set_retval = 187
BPF_FUNC_csum_diff = 28
BPF_FUNC_xdp_adjust_head = 44
BPF_FUNC_xdp_adjust_tail = 65
BPF_FUNC_ringbuf_output = 130
BPF_FUNC_ringbuf_reserve = 131
BPF_FUNC_ringbuf_submit = 132
BPF_FUNC_ringbuf_discard = 133
BPF_FUNC_xdp_load_bytes = 189

# map types (linux/bpf.h)
BPF_MAP_TYPE_HASH = 1
BPF_MAP_TYPE_ARRAY = 2
BPF_MAP_TYPE_PROG_ARRAY = 3
BPF_MAP_TYPE_PERCPU_HASH = 5
BPF_MAP_TYPE_PERCPU_ARRAY = 6
BPF_MAP_TYPE_LRU_HASH = 9
BPF_MAP_TYPE_LPM_TRIE = 11
BPF_MAP_TYPE_RINGBUF = 27
BPF_ANY, BPF_NOEXIST, BPF_EXIST = 0, 1, 2
BPF_F_MMAPABLE = 1 << 10


@dataclass
class Insn:
    code: int
    dst: int = 0
    src: int = 0
    off: int = 0
    imm: int = 0

    def encode(self) -> bytes:
        return struct.pack("<BBhi", self.code & 0xFF, (self.dst & 0xF) | ((self.src & 0xF) << 4),
                           _s16(self.off), _s32(self.imm))


def _s16(v: int) -> int:
    v &= 0xFFFF
    return v - 0x10000 if v & 0x8000 else v


def _s32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - 0x100000000 if v & 0x80000000 else v


def decode(code: bytes) -> List[Insn]:
    if len(code) % 8:
        raise ValueError("code length must be a multiple of 8")
    out = []
    for i in range(0, len(code), 8):
        c, regs, off, imm = struct.unpack_from("<BBhi", code, i)
        out.append(Insn(c, regs & 0xF, regs >> 4, off, imm))
    return out


def _reg(r: Union[str, int]) -> int:
    if isinstance(r, int):
        return r
    r = r.strip().lower()
    if r == "fp":
        return 10
    if not r.startswith("r"):
        raise ValueError(f"bad register {r!r}")
    return int(r[1:])


class Asm:
    """Label-aware eBPF assembler.

    Jumps take either a relative int offset or a label name; labels are
    resolved at :meth:`assemble`.  Each method appends one instruction (``lddw``
    appends two slots).
    """

    def __init__(self) -> None:
        self.insns: List[Insn] = []
        self.labels: Dict[str, int] = {}
        self.fixups: List[tuple] = []

    # -- bookkeeping --
    def label(self, name: str) -> "Asm":
        if name in self.labels:
            raise ValueError(f"duplicate label {name}")
        self.labels[name] = len(self.insns)
        return self

    def raw(self, code: int, dst=0, src=0, off=0, imm=0) -> "Asm":
        self.insns.append(Insn(code, _reg(dst), _reg(src), off, imm))
        return self

    @property
    def pc(self) -> int:
        return len(self.insns)

    # -- ALU --
    def _alu(self, cls: int, op: str, dst, src_or_imm) -> "Asm":
        code = cls | ALU_OPS[op]
        if isinstance(src_or_imm, str):
            return self.raw(code | SRC_REG, dst, _reg(src_or_imm))
        return self.raw(code | SRC_IMM, dst, 0, 0, src_or_imm)

    def alu64(self, op: str, dst, v) -> "Asm":
        return self._alu(CLS_ALU64, op, dst, v)

    def alu32(self, op: str, dst, v) -> "Asm":
        return self._alu(CLS_ALU, op, dst, v)

    def mov64(self, dst, v) -> "Asm":
        return self.alu64("mov", dst, v)

    def mov32(self, dst, v) -> "Asm":
        return self.alu32("mov", dst, v)

    def add64(self, dst, v) -> "Asm":
        return self.alu64("add", dst, v)

    def neg64(self, dst) -> "Asm":
        return self.raw(CLS_ALU64 | ALU_OPS["neg"], dst)

    def neg32(self, dst) -> "Asm":
        return self.raw(CLS_ALU | ALU_OPS["neg"], dst)

    def be(self, dst, bits: int) -> "Asm":
        return self.raw(OP_BE, dst, 0, 0, bits)

    def le(self, dst, bits: int) -> "Asm":
        return self.raw(OP_LE, dst, 0, 0, bits)

    # -- memory --
    def ldx(self, size: int, dst, src, off: int = 0) -> "Asm":
        return self.raw(CLS_LDX | MODE_MEM | SIZES[size], dst, src, off)

    def stx(self, size: int, dst, off: int, src) -> "Asm":
        return self.raw(CLS_STX | MODE_MEM | SIZES[size], dst, src, off)

    def st(self, size: int, dst, off: int, imm: int) -> "Asm":
        return self.raw(CLS_ST | MODE_MEM | SIZES[size], dst, 0, off, imm)

    def atomic(self, size: int, aop: int, dst, off: int, src) -> "Asm":
        assert size in (4, 8)
        return self.raw(CLS_STX | MODE_ATOMIC | SIZES[size], dst, src, off, aop)

    def lddw(self, dst, imm64: int, src: int = 0, next_imm: Optional[int] = None) -> "Asm":
        lo = imm64 & 0xFFFFFFFF
        hi = (imm64 >> 32) & 0xFFFFFFFF if next_imm is None else next_imm
        self.raw(OP_LDDW, dst, src, 0, lo)
        self.raw(0, 0, 0, 0, hi)
        return self

    def ld_map_fd(self, dst, fd: int) -> "Asm":
        """lddw src=1 (BPF_PSEUDO_MAP_FD) as libbpf relocates it."""
        return self.lddw(dst, fd, src=PSEUDO_MAP_FD, next_imm=0)

    def ld_map_value(self, dst, fd: int, off: int = 0) -> "Asm":
        """lddw src=2 (BPF_PSEUDO_MAP_VALUE): imm=fd, next.imm=offset."""
        return self.lddw(dst, fd, src=PSEUDO_MAP_VALUE, next_imm=off)

    # -- control flow --
    def _jmp(self, cls: int, op: str, dst, v, target) -> "Asm":
        code = cls | JMP_OPS[op]
        if isinstance(v, str):
            code |= SRC_REG
            src, imm = _reg(v), 0
        else:
            src, imm = 0, v
        self.raw(code, dst, src, 0, imm)
        self._target(target)
        return self

    def _target(self, target) -> None:
        if isinstance(target, str):
            self.fixups.append((len(self.insns) - 1, target))
        else:
            self.insns[-1].off = target

    def jmp(self, op: str, dst, v, target) -> "Asm":
        return self._jmp(CLS_JMP, op, dst, v, target)

    def jmp32(self, op: str, dst, v, target) -> "Asm":
        return self._jmp(CLS_JMP32, op, dst, v, target)

    def ja(self, target) -> "Asm":
        self.raw(CLS_JMP | JMP_OPS["ja"])
        self._target(target)
        return self

    def call(self, helper: int) -> "Asm":
        return self.raw(OP_CALL, 0, 0, 0, helper)

    def exit(self) -> "Asm":
        return self.raw(OP_EXIT)

    # -- output --
    def assemble(self) -> bytes:
        for idx, name in self.fixups:
            if name not in self.labels:
                raise ValueError(f"undefined label {name}")
            self.insns[idx].off = self.labels[name] - idx - 1
        return b"".join(i.encode() for i in self.insns)


_ALU_NAMES = {v: k for k, v in ALU_OPS.items()}
_JMP_NAMES = {v: k for k, v in JMP_OPS.items()}


def disasm(code: bytes) -> List[str]:
    """Human-readable listing (one line per 8-byte slot)."""
    ins = decode(code)
    out = []
    i = 0
    while i < len(ins):
        d = ins[i]
        cls = d.code & 7
        if d.code == OP_LDDW and i + 1 < len(ins):
            imm = (d.imm & 0xFFFFFFFF) | ((ins[i + 1].imm & 0xFFFFFFFF) << 32)
            out.append(f"{i:4d}: lddw r{d.dst}, {imm:#x}" + (f" (src={d.src})" if d.src else ""))
            out.append(f"{i + 1:4d}:   (lddw hi)")
            i += 2
            continue
        if cls in (CLS_ALU, CLS_ALU64):
            op = d.code & 0xF0
            sfx = "64" if cls == CLS_ALU64 else "32"
            if op == 0xD0:
                txt = f"{'be' if d.code & SRC_REG else 'le'}{d.imm} r{d.dst}"
            elif op == 0x80:
                txt = f"neg{sfx} r{d.dst}"
            else:
                v = f"r{d.src}" if d.code & SRC_REG else str(d.imm)
                txt = f"{_ALU_NAMES.get(op, '?')}{sfx} r{d.dst}, {v}"
        elif cls in (CLS_JMP, CLS_JMP32):
            op = d.code & 0xF0
            if d.code == OP_CALL:
                txt = f"call {d.imm}"
            elif d.code == OP_EXIT:
                txt = "exit"
            elif op == 0:
                txt = f"ja {d.off:+d} (-> {i + 1 + d.off})"
            else:
                v = f"r{d.src}" if d.code & SRC_REG else str(d.imm)
                sfx = "32" if cls == CLS_JMP32 else ""
                txt = f"{_JMP_NAMES.get(op, '?')}{sfx} r{d.dst}, {v}, {d.off:+d} (-> {i + 1 + d.off})"
        elif cls == CLS_LDX:
            txt = f"ldx{SIZE_NAMES[d.code & 0x18]} r{d.dst}, [r{d.src}{d.off:+d}]"
        elif cls == CLS_STX and (d.code & 0xE0) == MODE_ATOMIC:
            txt = f"atomic{SIZE_BYTES[d.code & 0x18] * 8} op={d.imm:#x} [r{d.dst}{d.off:+d}], r{d.src}"
        elif cls == CLS_STX:
            txt = f"stx{SIZE_NAMES[d.code & 0x18]} [r{d.dst}{d.off:+d}], r{d.src}"
        elif cls == CLS_ST:
            txt = f"st{SIZE_NAMES[d.code & 0x18]} [r{d.dst}{d.off:+d}], {d.imm}"
        else:
            txt = f".raw {d.code:#04x} {d.dst} {d.src} {d.off} {d.imm}"
        out.append(f"{i:4d}: {txt}")
        i += 1
    return out
