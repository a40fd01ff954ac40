"""eBPF ELF object loader (csrc/object.cpp) without a
GPU: parsing, libbpf-style map / global-data relocation and CO-RE against
the xdp_md layout of runtime/extension/userspace_xdp.h:6-17, checked
instruction by instruction and, through the oracle, against the
hand-assembled xdp-counter of SURVEY.md Appendix A on the config-1 pcap."""
import os
import struct

import numpy as np
import pytest

from bpftime_amd import isa, programs
from bpftime_amd.object import BpfObject, ObjectError

import _elf
from _helpers import make_maps

BASE_BTF = "/root/reference/example/xdp-counter/base.btf"  # present only in the build container


def decode(code: bytes):
    out = []
    for i in range(0, len(code), 8):
        op, regs, off, imm = struct.unpack_from("<BBhi", code, i)
        out.append((op, regs & 15, regs >> 4, off, imm))
    return out


def test_parse_xdp_counter_object():
    o = BpfObject.from_bytes(_elf.xdp_counter_object(), "xdp-counter")
    progs = o.programs()
    assert [(p.name, p.secname, p.prog_type, p.insn_cnt) for p in progs] == [("xdp_pass", "xdp", 6, 37)]
    maps = o.maps()
    assert [(m.name, m.type, m.key_size, m.value_size, m.max_entries) for m in maps] == [
        ("ctl_array", isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2),
        ("xdp_coun.bss", isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)]   # libbpf internal_map_name()
    assert maps[1].flags == 0x400  # BPF_F_MMAPABLE
    assert o.license() == "GPL"


@pytest.mark.parametrize("variant", ["builtin", "target_btf", "legacy_maps"])
def test_relocated_instructions(variant):
    obj = _elf.xdp_counter_object(legacy_maps=variant == "legacy_maps")
    btf = _elf.target_btf_xdp_md() if variant == "target_btf" else None
    o = BpfObject.from_bytes(obj, "xdp-counter", btf=btf)
    ins = decode(o.insns(0, [5, 9]))
    # CO-RE: u32 loads of the kernel xdp_md become u64 loads at 8 / 0
    assert ins[0] == (0x79, 7, 1, 8, 0) and ins[1] == (0x79, 6, 1, 0, 0)
    # lddw of the map -> BPF_PSEUDO_MAP_FD, of the global -> BPF_PSEUDO_MAP_VALUE
    assert ins[6][:3] == (0x18, 1, 1) and ins[6][4] == 5 and ins[7][4] == 0
    assert ins[14][:3] == (0x18, 1, 2) and ins[14][4] == 9 and ins[15][4] == 0
    raw = decode(_elf.xdp_counter_program())
    for i in set(range(len(ins))) - {0, 1, 6, 7, 14, 15}:
        assert ins[i] == raw[i], i


@pytest.mark.skipif(not os.path.exists(BASE_BTF), reason="reference tree not mounted (GPU box)")
def test_reference_base_btf_gives_builtin_layout():
    """The reference example's base.btf (its xdp_md: u64 data / data_end)
    relocates exactly like the built-in target."""
    o1 = BpfObject.from_bytes(_elf.xdp_counter_object(), "xdp-counter")
    o2 = BpfObject.from_bytes(_elf.xdp_counter_object(), "xdp-counter", btf=open(BASE_BTF, "rb").read())
    assert o1.insns(0, [3, 4]) == o2.insns(0, [3, 4])


def test_object_matches_appendix_a_on_oracle(fresh_oracle):
    """Config 1 (1000-frame pcap, ctl 0 then 1) through the oracle: the
    object's relocated program and the hand-assembled Appendix A program
    give the same verdicts, packet bytes and counters."""
    from bpftime_amd import gen
    po = fresh_oracle
    o = BpfObject.from_bytes(_elf.xdp_counter_object(), "xdp-counter")
    for flag in (0, 1):
        res = []
        for code_of in (lambda c, b: o.insns(0, [c, b]), programs.xdp_counter):
            po.reset()
            (octl, obss), _ = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2), (isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)],
                                        po, None)
            if flag:
                octl.update(struct.pack("<I", 0), struct.pack("<I", 1))
            vm = po.OracleVM()
            vm.load(code_of(octl.fd, obss.fd))
            pk, lens = gen.frames_to_slots(gen.config1_frames(), stride=64)
            v = vm.run_xdp(pk, lens=lens)
            res.append((v, pk, obss.lookup(b"\0\0\0\0")))
        (v1, p1, c1), (v2, p2, c2) = res
        np.testing.assert_array_equal(v1, v2)
        np.testing.assert_array_equal(p1, p2)
        assert c1 == c2
        assert struct.unpack_from("<Q", c1)[0] == (1000 if flag == 0 else 0)


def test_bpf_to_bpf_call_rejected():
    e = _elf.Elf()
    code = _elf.Asm().call(1).mov64(0, 0).exit().assemble()
    e.section("xdp", code, flags=_elf.SHF_ALLOC | _elf.SHF_EXECINSTR)
    e.section(".text", _elf.Asm().mov64(0, 1).exit().assemble(), flags=_elf.SHF_ALLOC | _elf.SHF_EXECINSTR)
    e.symbol("prog", "xdp", 0, len(code), type_=_elf.STT_FUNC)
    e.symbol("sub", ".text", 0, 16, type_=_elf.STT_FUNC)
    e.reloc("xdp", 0, "sub", _elf.R_BPF_64_32)
    with pytest.raises(ObjectError, match="BPF-to-BPF call"):
        BpfObject.from_bytes(e.encode(), "calls")


def test_not_an_object():
    with pytest.raises(ObjectError, match="not an ELF"):
        BpfObject.from_bytes(b"\0" * 128, "junk")


def test_missing_target_field_poisons_insn():
    """A CO-RE field the target lacks: libbpf's poison (call 0xbad2310)."""
    b = _elf.Btf()
    u32 = b.int_("unsigned int", 4)
    t = b.struct_("xdp_md", 8, [("data", u32, 0), ("no_such_field", u32, 32)])
    code = _elf.Asm().ldx(4, 0, 1, 4).exit().assemble()
    ext = _elf.btf_ext(b, [("xdp", 0, t, "0:1", 0)])  # adds its strings to .BTF first
    e = _elf.Elf()
    e.section("xdp", code, flags=_elf.SHF_ALLOC | _elf.SHF_EXECINSTR)
    e.section(".BTF", b.encode(), align=4)
    e.section(".BTF.ext", ext, align=4)
    e.symbol("prog", "xdp", 0, len(code), type_=_elf.STT_FUNC)
    o = BpfObject.from_bytes(e.encode(), "poison")
    ins = decode(o.insns(0, []))
    assert ins[0] == (0x85, 0, 0, 0, 0xBAD2310)
