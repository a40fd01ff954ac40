"""eBPF ELF objects (host mirror of runtime/object/bpftime_object.hpp over the
C ABI of csrc/object.cpp): open + CO-RE + relocation on the host, load to
device maps and prog records.

    obj = BpfObject.open("xdp-counter.bpf.o", btf="base.btf")
    obj.load()
    vm = prog_instantiate(obj.program_fd("xdp_pass"))
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional

from ._lib import BpfMapAttr, lib


class ObjectError(RuntimeError):
    pass


@dataclass
class ObjMap:
    name: str
    type: int
    key_size: int
    value_size: int
    max_entries: int
    flags: int


@dataclass
class ObjProg:
    name: str
    secname: str
    prog_type: int
    insn_cnt: int


class BpfObject:
    def __init__(self, handle: int):
        self.h = C.c_void_p(handle)
        err = lib().bpftime_object_error(self.h)
        if err:
            msg = err.decode()
            self.close()
            raise ObjectError(msg)

    @classmethod
    def open(cls, path: str, btf: Optional[str] = None) -> "BpfObject":
        h = lib().bpftime_object_open(path.encode())
        if not h:
            raise ObjectError(f"cannot read {path}")
        o = cls(h)
        if btf is not None:
            o.relocate_btf(btf)
        return o

    @classmethod
    def from_bytes(cls, data: bytes, name: str = "obj", btf: Optional[bytes] = None) -> "BpfObject":
        h = lib().bpftime_object_open_mem(data, len(data), name.encode())
        o = cls(h)
        if btf is not None:
            if lib().bpftime_object_load_relocate_btf_mem(o.h, btf, len(btf)) < 0:
                raise ObjectError(o.error())
        return o

    def error(self) -> str:
        return lib().bpftime_object_error(self.h).decode()

    def relocate_btf(self, path: str) -> None:
        if lib().bpftime_object_load_relocate_btf(self.h, path.encode()) < 0:
            raise ObjectError(self.error())

    def maps(self) -> List[ObjMap]:
        out = []
        for i in range(lib().bpftime_object_map_count(self.h)):
            name = C.c_char_p()
            a = BpfMapAttr()
            lib().bpftime_object_map_info(self.h, i, C.byref(name), C.byref(a))
            out.append(ObjMap(name.value.decode(), a.type, a.key_size, a.value_size, a.max_ents, a.flags))
        return out

    def programs(self) -> List[ObjProg]:
        out = []
        for i in range(lib().bpftime_object_program_count(self.h)):
            name, sec = C.c_char_p(), C.c_char_p()
            t, n = C.c_int(), C.c_size_t()
            lib().bpftime_object_program_info(self.h, i, C.byref(name), C.byref(sec), C.byref(t), C.byref(n))
            out.append(ObjProg(name.value.decode(), sec.value.decode(), t.value, n.value))
        return out

    def insns(self, idx: int, map_fds: List[int]) -> bytes:
        """Relocated instructions of program idx for the given map fds."""
        progs = self.programs()
        fds = (C.c_int * max(1, len(map_fds)))(*map_fds)
        buf = C.create_string_buffer(8 * progs[idx].insn_cnt)
        n = lib().bpftime_object_program_insns(self.h, idx, fds, buf, progs[idx].insn_cnt)
        if n < 0:
            raise ObjectError("relocation failed")
        return buf.raw[:8 * n]

    def load(self) -> None:
        if lib().bpftime_object_load(self.h) < 0:
            raise ObjectError(self.error())

    def program_fd(self, name: str) -> int:
        return lib().bpftime_object_find_program_by_name(self.h, name.encode())

    def program_fd_by_secname(self, sec: str) -> int:
        return lib().bpftime_object_find_program_by_secname(self.h, sec.encode())

    def map_fd(self, name: str) -> int:
        return lib().bpftime_object_find_map_fd_by_name(self.h, name.encode())

    def license(self) -> str:
        return lib().bpftime_object_license(self.h).decode()

    def close(self) -> None:
        if self.h:
            lib().bpftime_object_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
