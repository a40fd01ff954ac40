"""Test infrastructure: writes eBPF ELF objects the way clang -target bpf
(+ libbpf's bpf_helpers.h conventions) lays them out, since no BPF-capable
clang exists in this image.  Formats: ELF64 (elf.h), BTF / BTF.ext
(linux/btf.h, the kernel's Documentation/bpf/btf.rst): program sections,
.maps with BTF-defined map variables, legacy "maps", .bss/.data/.rodata,
.rel<sec> R_BPF_64_64 relocations, .BTF.ext CO-RE field relocations.

`xdp_counter_object()` is example/xdp-counter/xdp-counter.bpf.c as clang
would emit it (kernel xdp_md layout, u32 ctx loads carrying CO-RE relocs),
the instruction stream semantically equal to SURVEY.md Appendix A."""
import struct
from typing import Dict, List, Optional, Tuple

from bpftime_amd.isa import Asm

# BTF kinds
INT, PTR, ARRAY, STRUCT, UNION, ENUM, FWD, TYPEDEF, VOLATILE, CONST, RESTRICT, FUNC, FUNC_PROTO, VAR, \
    DATASEC = range(1, 16)


class Btf:
    def __init__(self):
        self.types: List[bytes] = []
        self.strs = bytearray(b"\0")
        self.names: Dict[str, int] = {"": 0}

    def s(self, name: str) -> int:
        if name not in self.names:
            self.names[name] = len(self.strs)
            self.strs += name.encode() + b"\0"
        return self.names[name]

    def _add(self, name, kind, vlen, su, extra=b"", kflag=0) -> int:
        info = (kflag << 31) | (kind << 24) | vlen
        self.types.append(struct.pack("<III", self.s(name), info, su) + extra)
        return len(self.types)

    def int_(self, name, size, signed=False):
        return self._add(name, INT, 0, size, struct.pack("<I", ((1 if signed else 0) << 24) | size * 8))

    def ptr(self, t):
        return self._add("", PTR, 0, t)

    def array(self, elem, index, n):
        return self._add("", ARRAY, 0, 0, struct.pack("<III", elem, index, n))

    def struct_(self, name, size, members: List[Tuple[str, int, int]]):
        extra = b"".join(struct.pack("<III", self.s(m), t, off) for m, t, off in members)
        return self._add(name, STRUCT, len(members), size, extra)

    def typedef(self, name, t):
        return self._add(name, TYPEDEF, 0, t)

    def var(self, name, t, linkage=1):
        return self._add(name, VAR, 0, t, struct.pack("<I", linkage))

    def datasec(self, name, size, vars_: List[Tuple[int, int, int]]):
        extra = b"".join(struct.pack("<III", v, off, sz) for v, off, sz in vars_)
        return self._add(name, DATASEC, len(vars_), size, extra)

    def func_proto(self, ret, params: List[Tuple[str, int]]):
        extra = b"".join(struct.pack("<II", self.s(n), t) for n, t in params)
        return self._add("", FUNC_PROTO, len(params), ret, extra)

    def func(self, name, proto, linkage=1):
        return self._add(name, FUNC, linkage, proto)

    def encode(self) -> bytes:
        tb = b"".join(self.types)
        hdr = struct.pack("<HBBIIIII", 0xEB9F, 1, 0, 24, 0, len(tb), len(tb), len(self.strs))
        return hdr + tb + bytes(self.strs)


def btf_ext(btf: Btf, core: List[Tuple[str, int, int, str, int]]) -> bytes:
    """core: (section, insn byte offset, type id, access string, kind)."""
    func_info = struct.pack("<I", 8)
    line_info = struct.pack("<I", 16)
    by_sec: Dict[str, list] = {}
    for sec, off, tid, acc, kind in core:
        by_sec.setdefault(sec, []).append(struct.pack("<IIII", off, tid, btf.s(acc), kind))
    cr = struct.pack("<I", 16) + b"".join(struct.pack("<II", btf.s(sec), len(r)) + b"".join(r)
                                          for sec, r in by_sec.items())
    hdr_len = 32
    body = func_info + line_info + cr
    hdr = struct.pack("<HBBIIIIIII", 0xEB9F, 1, 0, hdr_len, 0, len(func_info), len(func_info), len(line_info),
                      len(func_info) + len(line_info), len(cr))
    return hdr + body


# ELF
SHT_PROGBITS, SHT_SYMTAB, SHT_STRTAB, SHT_NOBITS, SHT_REL = 1, 2, 3, 8, 9
SHF_WRITE, SHF_ALLOC, SHF_EXECINSTR = 1, 2, 4
STB_LOCAL, STB_GLOBAL = 0, 1
STT_NOTYPE, STT_OBJECT, STT_FUNC, STT_SECTION = 0, 1, 2, 3
R_BPF_64_64, R_BPF_64_32 = 1, 10


class Elf:
    def __init__(self):
        self.secs: List[dict] = []   # name, type, flags, data, size, align, link, info, entsize
        self.syms: List[tuple] = []  # name, value, size, bind, type, sec name
        self.rels: Dict[str, List[Tuple[int, str, int]]] = {}

    def section(self, name, data=b"", type_=SHT_PROGBITS, flags=0, align=8, size=None):
        self.secs.append(dict(name=name, type=type_, flags=flags, data=data,
                              size=len(data) if size is None else size, align=align))

    def symbol(self, name, sec, value=0, size=0, bind=STB_GLOBAL, type_=STT_OBJECT):
        self.syms.append((name, value, size, bind, type_, sec))

    def reloc(self, sec, offset, sym, type_=R_BPF_64_64):
        self.rels.setdefault(sec, []).append((offset, sym, type_))

    def encode(self) -> bytes:
        secs = [dict(name="", type=0, flags=0, data=b"", size=0, align=0)] + list(self.secs)
        idx = {s["name"]: i for i, s in enumerate(secs)}
        for name in self.rels:
            secs.append(dict(name=".rel" + name, type=SHT_REL, flags=0, data=b"", size=0, align=8, target=name))
        secs.append(dict(name=".symtab", type=SHT_SYMTAB, flags=0, data=b"", size=0, align=8))
        secs.append(dict(name=".strtab", type=SHT_STRTAB, flags=0, data=b"", size=0, align=1))
        idx = {s["name"]: i for i, s in enumerate(secs)}
        strtab = bytearray(b"\0")
        soff: Dict[str, int] = {}

        def sname(n):
            if n not in soff:
                soff[n] = len(strtab)
                strtab.extend(n.encode() + b"\0")
            return soff[n]

        for s in secs:
            s["name_off"] = sname(s["name"]) if s["name"] else 0
        # symbols: null, section symbols (local), then globals
        syms = [(0, 0, 0, 0, 0, 0)]
        sym_index = {}
        for s in self.secs:
            if s["type"] in (SHT_PROGBITS, SHT_NOBITS) and s["flags"] & SHF_ALLOC:
                syms.append((0, (STB_LOCAL << 4) | STT_SECTION, 0, idx[s["name"]], 0, 0))
        first_global = len(syms)
        for name, value, size, bind, type_, sec in self.syms:
            sym_index[name] = len(syms)
            syms.append((sname(name), (bind << 4) | type_, 0, idx[sec], value, size))
        symtab = b"".join(struct.pack("<IBBHQQ", *s) for s in syms)
        for s in secs:
            if s["type"] == SHT_SYMTAB:
                s.update(data=symtab, size=len(symtab), link=idx[".strtab"], info=first_global, entsize=24)
            elif s["type"] == SHT_REL:
                rel = b"".join(struct.pack("<QQ", off, (sym_index[sym] << 32) | t)
                               for off, sym, t in self.rels[s["target"]])
                s.update(data=rel, size=len(rel), link=idx[".symtab"], info=idx[s["target"]], entsize=16)
        secs[idx[".strtab"]].update(data=bytes(strtab), size=len(strtab))
        out = bytearray(64)
        for s in secs[1:]:
            if s["type"] == SHT_NOBITS:
                s["offset"] = len(out)
                continue
            al = max(1, s["align"])
            out.extend(b"\0" * ((-len(out)) % al))
            s["offset"] = len(out)
            out.extend(s["data"])
        out.extend(b"\0" * ((-len(out)) % 8))
        shoff = len(out)
        secs[0]["offset"] = 0
        for s in secs:
            out.extend(struct.pack("<IIQQQQIIQQ", s["name_off"], s["type"], s["flags"], 0, s["offset"], s["size"],
                                   s.get("link", 0), s.get("info", 0), s["align"], s.get("entsize", 0)))
        ident = b"\x7fELF" + bytes([2, 1, 1, 0]) + b"\0" * 8
        eh = ident + struct.pack("<HHIQQQIHHHHHH", 1, 247, 1, 0, 0, shoff, 0, 64, 0, 0, 64, len(secs),
                                 idx[".strtab"])
        out[:64] = eh
        return bytes(out)


def xdp_counter_program() -> bytes:
    """xdp_pass as clang -O2 emits it before libbpf: u32 ctx loads (CO-RE
    relocated at insns 0 and 1), lddw 6 -> ctl_array, lddw 14 -> cntrs_array."""
    a = Asm()
    a.ldx(4, 7, 1, 4)               # 0  data_end = ctx->data_end   (CO-RE xdp_md 0:1)
    a.ldx(4, 6, 1, 0)               # 1  data     = ctx->data       (CO-RE xdp_md 0:0)
    a.mov64(1, 0)                   # 2
    a.stx(4, 10, -4, "r1")          # 3  ctl_flag_pos = 0
    a.mov64(2, "r10").add64(2, -4)  # 4, 5
    a.lddw(1, 0)                    # 6  r1 = &ctl_array  (R_BPF_64_64)
    a.call(1)                       # 8  bpf_map_lookup_elem
    a.mov64(1, "r0").mov64(0, 2)    # 9, 10
    a.jmp("jeq", 1, 0, "out")       # 11
    a.ldx(4, 1, 1, 0)               # 12
    a.jmp("jne", 1, 0, "out")       # 13
    a.lddw(1, 0)                    # 14 r1 = &cntrs_array[0] (R_BPF_64_64)
    a.ldx(8, 2, 1, 0).add64(2, 1).stx(8, 1, 0, "r2")   # 16-18 cntrs_array[0]++
    a.mov64(1, "r6").add64(1, 14)   # 19, 20
    a.mov64(0, 1)                   # 21 XDP_DROP
    a.jmp("jgt", 1, "r7", "out")    # 22
    a.ldx(2, 1, 6, 0).ldx(2, 2, 6, 6).stx(2, 6, 0, "r2")       # swap_src_dst_mac
    a.ldx(2, 2, 6, 2).ldx(2, 3, 6, 8).stx(2, 6, 2, "r3")
    a.ldx(2, 3, 6, 4).ldx(2, 4, 6, 10).stx(2, 6, 4, "r4")
    a.stx(2, 6, 6, "r1").stx(2, 6, 8, "r2").stx(2, 6, 10, "r3")
    a.mov64(0, 3)                   # XDP_TX
    a.label("out").exit()
    return a.assemble()


def xdp_counter_object(legacy_maps: bool = False, with_core: bool = True) -> bytes:
    code = xdp_counter_program()
    b = Btf()
    u32 = b.int_("unsigned int", 4)
    t_u32 = b.typedef("__u32", u32)
    i32 = b.int_("int", 4, signed=True)
    arr2 = b.array(i32, i32, 2)          # __uint(type, BPF_MAP_TYPE_ARRAY) / __uint(max_entries, 2)
    p_arr2 = b.ptr(arr2)
    p_u32 = b.ptr(t_u32)
    mdef = b.struct_("", 32, [("type", p_arr2, 0), ("key", p_u32, 64), ("value", p_u32, 128),
                             ("max_entries", p_arr2, 192)])
    v_ctl = b.var("ctl_array", mdef)
    u64 = b.int_("long long unsigned int", 8)
    t_u64 = b.typedef("__u64", u64)
    a512 = b.array(t_u64, i32, 512)
    v_cnt = b.var("cntrs_array", a512)
    xdp_md = b.struct_("xdp_md", 24, [("data", t_u32, 0), ("data_end", t_u32, 32), ("data_meta", t_u32, 64),
                                      ("ingress_ifindex", t_u32, 96), ("rx_queue_index", t_u32, 128),
                                      ("egress_ifindex", t_u32, 160)])
    proto = b.func_proto(i32, [("ctx", b.ptr(xdp_md))])
    b.func("xdp_pass", proto)
    if not legacy_maps:
        b.datasec(".maps", 32, [(v_ctl, 0, 32)])
    b.datasec(".bss", 4096, [(v_cnt, 0, 4096)])
    core = [("xdp", 0, xdp_md, "0:1", 0), ("xdp", 8, xdp_md, "0:0", 0)] if with_core else []
    ext = btf_ext(b, core)
    e = Elf()
    e.section("xdp", code, flags=SHF_ALLOC | SHF_EXECINSTR)
    if legacy_maps:
        e.section("maps", struct.pack("<IIIII", 2, 4, 4, 2, 0), flags=SHF_ALLOC | SHF_WRITE, align=4)
        e.symbol("ctl_array", "maps", 0, 20)
    else:
        e.section(".maps", bytes(32), flags=SHF_ALLOC | SHF_WRITE)
        e.symbol("ctl_array", ".maps", 0, 32)
    e.section(".bss", type_=SHT_NOBITS, flags=SHF_ALLOC | SHF_WRITE, size=4096)
    e.section("license", b"GPL\0", flags=SHF_ALLOC | SHF_WRITE, align=1)
    e.section(".BTF", b.encode(), align=4)
    e.section(".BTF.ext", ext, align=4)
    e.symbol("xdp_pass", "xdp", 0, len(code), type_=STT_FUNC)
    e.symbol("cntrs_array", ".bss", 0, 4096)
    e.symbol("_license", "license", 0, 4)
    e.reloc("xdp", 6 * 8, "ctl_array")
    e.reloc("xdp", 14 * 8, "cntrs_array")
    return e.encode()


def target_btf_xdp_md() -> bytes:
    """A target BTF with xdp_md as the runtime lays it out (u64 data /
    data_end, like example/xdp-counter/base.btf)."""
    b = Btf()
    u32 = b.typedef("__u32", b.int_("unsigned int", 4))
    u64 = b.typedef("__u64", b.int_("long long unsigned int", 8))
    b.struct_("xdp_md", 32, [("data", u64, 0), ("data_end", u64, 64), ("data_meta", u32, 128),
                             ("ingress_ifindex", u32, 160), ("rx_queue_index", u32, 192),
                             ("egress_ifindex", u32, 224)])
    return b.encode()
