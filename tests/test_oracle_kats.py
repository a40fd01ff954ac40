"""Oracle known-answer tests (CPU).

The interpreter arithmetic of the reference lives in the absent ubpf
submodule, so the oracle is pinned here by (a) the analytic
KATs the reference carries as bytecode + comments (vm/example/bpf_progs.h,
.github/assets/sum.bpf.o semantics) and (b) the eBPF ISA definition of every
opcode in vm/compat/include/ebpf_inst.h, evaluated independently in Python.
"""
import struct

import numpy as np
import pytest

from bpftime_amd import isa, programs
from bpftime_amd.isa import Asm

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1


def sx32(v):
    v &= M32
    return v - (1 << 32) if v >> 31 else v


def sx64(v):
    v &= M64
    return v - (1 << 64) if v >> 63 else v


def spec_alu(op, a, b, w32):
    """eBPF ISA (kernel Documentation/bpf/standardization) restated."""
    if w32:
        a &= M32
        b &= M32
        sh = b & 31
        r = {
            "add": a + b, "sub": a - b, "mul": a * b, "or": a | b, "and": a & b, "xor": a ^ b,
            "mov": b, "div": (a // b) if b else 0, "mod": (a % b) if b else a,
            "lsh": a << sh, "rsh": a >> sh, "arsh": sx32(a) >> sh, "neg": -a,
        }[op]
        return r & M32
    sh = b & 63
    r = {
        "add": a + b, "sub": a - b, "mul": a * b, "or": a | b, "and": a & b, "xor": a ^ b,
        "mov": b, "div": (a // b) if b else 0, "mod": (a % b) if b else a,
        "lsh": a << sh, "rsh": a >> sh, "arsh": sx64(a) >> sh, "neg": -a,
    }[op]
    return r & M64


def spec_jmp(op, a, b, w32):
    if w32:
        a, b = a & M32, b & M32
        sa, sb = sx32(a), sx32(b)
    else:
        sa, sb = sx64(a), sx64(b)
    return {
        "jeq": a == b, "jne": a != b, "jgt": a > b, "jge": a >= b, "jlt": a < b, "jle": a <= b,
        "jset": (a & b) != 0, "jsgt": sa > sb, "jsge": sa >= sb, "jslt": sa < sb, "jsle": sa <= sb,
    }[op]


VALUES = [0, 1, 2, 3, 7, 31, 32, 33, 63, 64, 65, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF, 0x100000000,
          0x123456789ABCDEF0, 0x7FFFFFFFFFFFFFFF, 0x8000000000000000, 0xFFFFFFFFFFFFFFFF,
          0xFFFFFFFF00000000, 0xDEADBEEF]


def alu_prog(op, a, b, w32, imm=None):
    p = Asm()
    p.lddw(0, a)
    if imm is None:
        p.lddw(1, b)
        (p.alu32 if w32 else p.alu64)(op, 0, "r1") if op != "neg" else (p.neg32(0) if w32 else p.neg64(0))
    else:
        (p.alu32 if w32 else p.alu64)(op, 0, imm)
    p.exit()
    return p.assemble()


def run(code, mem=b""):
    from oracle import pyoracle as po
    vm = po.OracleVM()
    vm.load(code)
    rc, r = vm.exec(bytearray(mem))
    assert rc == 0
    return r


@pytest.mark.parametrize("w32", [False, True])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "or", "and", "xor", "mov", "div", "mod", "lsh",
                                "rsh", "arsh", "neg"])
def test_alu_reg(fresh_oracle, op, w32):
    for a in VALUES:
        for b in VALUES[::3]:
            assert run(alu_prog(op, a, b, w32)) == spec_alu(op, a, b, w32), (op, hex(a), hex(b))


@pytest.mark.parametrize("w32", [False, True])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "or", "and", "xor", "mov", "div", "mod", "lsh",
                                "rsh", "arsh"])
def test_alu_imm(fresh_oracle, op, w32):
    for a in VALUES[::2]:
        for imm in [0, 1, 5, 31, 63, -1, -7, 0x7FFFFFFF, -0x80000000]:
            # immediates are sign-extended to 64 bits
            assert run(alu_prog(op, a, 0, w32, imm)) == spec_alu(op, a, imm & M64, w32), (op, a, imm)


@pytest.mark.parametrize("w32", [False, True])
@pytest.mark.parametrize("op", ["jeq", "jne", "jgt", "jge", "jlt", "jle", "jset", "jsgt", "jsge", "jslt",
                                "jsle"])
def test_jmp(fresh_oracle, op, w32):
    for a in VALUES[::2]:
        for b in VALUES[1::3]:
            p = Asm()
            p.lddw(1, a).lddw(2, b).mov64(0, 0)
            (p.jmp32 if w32 else p.jmp)(op, 1, "r2", "t")
            p.exit().label("t").mov64(0, 1).exit()
            assert run(p.assemble()) == int(spec_jmp(op, a, b, w32)), (op, hex(a), hex(b))


def test_endian(fresh_oracle):
    v = 0x0102030405060708
    for bits, exp_be, exp_le in [(16, 0x0807, 0x0708), (32, 0x08070605, 0x05060708),
                                 (64, 0x0807060504030201, v)]:
        assert run(Asm().lddw(0, v).be(0, bits).exit().assemble()) == exp_be
        assert run(Asm().lddw(0, v).le(0, bits).exit().assemble()) == exp_le


def test_memory_sizes_and_sign(fresh_oracle):
    mem = bytearray(range(1, 33))
    p = Asm()
    p.ldx(1, 2, 1, 3).ldx(2, 3, 1, 4).ldx(4, 4, 1, 8).ldx(8, 5, 1, 16)
    p.stx(8, 10, -8, "r5").st(4, 10, -12, -2).ldx(4, 6, 10, -12).ldx(8, 7, 10, -8)
    p.mov64(0, "r2").add64(0, "r3").add64(0, "r4").add64(0, "r5").add64(0, "r6").alu64("xor", 0, "r7")
    p.exit()
    b, h, w, dw = 4, 0x0605, 0x0C0B0A09, struct.unpack("<Q", bytes(range(17, 25)))[0]
    exp = ((b + h + w + dw + 0xFFFFFFFE) & M64) ^ dw
    assert run(p.assemble(), mem) == exp


def test_atomics(fresh_oracle):
    p = Asm()
    p.st(8, 10, -8, 10)
    p.mov64(1, 5).atomic(8, isa.ATOMIC_ADD | isa.ATOMIC_FETCH, 10, -8, "r1")   # r1 = 10, mem 15
    p.mov64(2, 3).atomic(8, isa.ATOMIC_OR, 10, -8, "r2")                      # mem 15
    p.mov64(3, 0xFF).atomic(8, isa.ATOMIC_XCHG, 10, -8, "r3")                 # r3 = 15, mem 255
    p.mov64(0, 255).mov64(4, 7).atomic(8, isa.ATOMIC_CMPXCHG, 10, -8, "r4")   # r0 = 255, mem 7
    p.ldx(8, 5, 10, -8)
    p.alu64("lsh", 1, 8).add64(0, "r1").alu64("lsh", 3, 16).add64(0, "r3").alu64("lsh", 5, 32).add64(0, "r5")
    p.exit()
    assert run(p.assemble()) == 255 + (10 << 8) + (15 << 16) + (7 << 32)


def test_kat_bpf_progs_h(fresh_oracle):
    # vm/example/bpf_progs.h:6-11 / :44-57: d->a + d->b
    mem = struct.pack("<II", 40, 2)
    assert run(programs.kat_add_mem(), mem) == 42
    assert run(programs.kat_add_mem_stack(), mem) == 42
    assert run(programs.kat_mul()) == 2  # bpf_progs.h:66-77


def test_kat_sum(fresh_oracle):
    # .github/assets/sum.bpf.o: test(int *arr) = sum(arr[1..arr[0]])
    arr = [5, 1, -2, 30, 4, -100, 999]
    mem = struct.pack("<7i", *arr)
    assert run(programs.kat_sum(), mem) == (sum(arr[1:6]) & M64)
    assert run(programs.kat_sum(), struct.pack("<2i", 0, 77)) == 0


def test_ubpf_conventions(fresh_oracle):
    # r1 = mem, r2 = len, r10 = stack top (ebpf-vm.h:47-49)
    assert run(Asm().mov64(0, "r2").exit().assemble(), b"x" * 37) == 37
    p = Asm().mov64(0, "r10").alu64("sub", 0, "r1").exit().assemble()
    assert run(p, b"y") != 0


def test_helper_call_keeps_r1_r5(fresh_oracle):
    from oracle import pyoracle as po
    m = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)
    p = Asm()
    p.st(4, 10, -4, 9).ld_map_fd(1, m.fd).mov64(2, "r10").add64(2, -4).mov64(3, 77).call(1)
    p.mov64(0, "r3").exit()
    assert run(p.assemble()) == 77  # ubpf leaves r1-r5 untouched


def test_load_errors_match_compat_ubpf(fresh_oracle):
    from oracle import pyoracle as po
    vm = po.OracleVM()
    assert vm.try_load(b"\x95" + b"\0" * 6)[1] == "Length of code must be a multiple of 8"
    vm = po.OracleVM()
    rc, msg = vm.try_load(Asm().call(99).exit().assemble())
    assert rc < 0 and msg == "invalid call immediate at PC 0"
    vm = po.OracleVM()
    rc, msg = vm.try_load(Asm().mov64(0, 0).call(60).exit().assemble())
    assert rc < 0 and msg == "call to nonexistent function 60 at PC 1"
    vm = po.OracleVM()
    rc, msg = vm.try_load(Asm().lddw(0, 1, src=3).exit().assemble())
    assert msg == "Unable to patch lddw instruction at 0, var_addr not defined"
    vm = po.OracleVM()
    code = Asm().mov64(0, 0).exit().assemble() + bytes([0x18, 0, 0, 0, 0, 0, 0, 0])
    rc, msg = vm.try_load(code)
    assert msg == "Unable to patch lddw instructions at 2, it's the last instruction"
