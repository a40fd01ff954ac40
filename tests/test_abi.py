"""C-ABI checks that need no GPU: libbpftime_amd.so loads and exports every
function include/*.h declares; VM-level error paths that run before any
device work behave like the reference (compat_ubpf.cpp:61-200,
ebpf-vm.cpp:6-98)."""
import ctypes as C
import errno
import os
import re

import pytest

from bpftime_amd import _lib, isa
from bpftime_amd.isa import Asm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("ebpf-vm.h", "bpftime_amd.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^(?!typedef)[a-z][\w\s\*]*?\b(\w+)\s*\(", txt, flags=re.M):
            name = m.group(1)
            if name not in ("sizeof",):
                names.add(name)
    return names


def test_library_exports_every_declared_symbol():
    l = _lib.lib()
    names = declared_functions()
    assert len(names) > 60
    missing = [n for n in sorted(names) if not hasattr(l, n)]
    assert not missing, missing
    bound = {s[0] for s in _lib.SIGNATURES}
    assert names <= bound, sorted(names - bound)


def test_create_unknown_vm_returns_null():
    l = _lib.lib()
    assert not l.ebpf_create(b"ubpf")
    assert not l.ebpf_create(b"")
    vm = l.ebpf_create(b"mi355x")
    assert vm
    assert l.ebpf_get_vm_name(C.c_void_p(vm)) == b""  # ebpf-vm.cpp:13-16 never sets it
    l.ebpf_destroy(C.c_void_p(vm))


def _load(code, register=True):
    from bpftime_amd.vm import VM
    vm = VM(default_helpers=register)
    return vm.try_load(code)


def test_load_errors_before_device_work():
    assert _load(b"\x95" + b"\0" * 6) == (-1, "Length of code must be a multiple of 8")
    rc, msg = _load(Asm().call(99).exit().assemble())
    assert rc == -22 and msg == "invalid call immediate at PC 0"
    rc, msg = _load(Asm().mov64(0, 0).call(1).exit().assemble(), register=False)
    assert rc == -22 and msg == "call to nonexistent function 1 at PC 1"
    rc, msg = _load(Asm().lddw(0, 1, src=4).exit().assemble())
    assert msg == "Unable to patch lddw instruction at 0, code_addr not defined"
    rc, msg = _load(Asm().lddw(0, 1, src=9).exit().assemble())
    assert msg == "Unable to patch lddw instruction at 0, unsupported src_reg 9"
    rc, msg = _load(Asm().raw(0x8e).exit().assemble())
    assert msg == "unknown opcode 0x8e at PC 0"
    rc, msg = _load(Asm().mov64(10, 1).exit().assemble())
    assert msg == "invalid destination register at PC 0"
    rc, msg = _load(Asm().jmp("jeq", 1, 0, -5).exit().assemble())
    assert msg == "jump out of bounds at PC 0"


def test_host_only_helper_rejected_at_load():
    from bpftime_amd.vm import VM
    vm = VM()
    vm.register(6, "bpf_trace_printk")
    rc, msg = vm.try_load(Asm().call(6).exit().assemble())
    assert rc == -22 and "has no device implementation" in msg


def test_compile_and_aot_unsupported():
    l = _lib.lib()
    vm = l.ebpf_create(b"mi355x")
    err = C.c_void_p()
    assert not l.ebpf_compile(C.c_void_p(vm), C.byref(err))
    assert b"interpreter" in C.string_at(err.value)
    assert not l.ebpf_load_aot_object(C.c_void_p(vm), None, 0)
    l.ebpf_destroy(C.c_void_p(vm))


def test_sysbpf_errors_before_device_work():
    """bpf(2) commands the data path does not serve, and element ops on an
    fd that is no map (syscall_context.cpp:490-514: ENOENT)."""
    import struct
    from bpftime_amd import vm
    r, e = vm.sys_bpf(99, bytearray(128))
    assert r == -1 and e == errno.ENOTSUP
    key = bytearray(4)
    kb = (C.c_char * 4).from_buffer(key)
    val = bytearray(8)
    vb = (C.c_char * 8).from_buffer(val)
    r, e = vm.sys_bpf(vm.BPF_MAP_LOOKUP_ELEM, vm.attr_map_elem(777, C.addressof(kb), C.addressof(vb)))
    assert r == -1 and e == errno.ENOENT
    assert vm.sys_bpf(vm.BPF_MAP_FREEZE, bytearray(128))[0] == 0
    assert _lib.lib().bpftime_amd_handle_sysbpf(vm.BPF_MAP_CREATE, None, 0) == -1
    assert struct.calcsize("<IIQQQ") == 32


def test_lds_sizing_of_launch_shapes():
    """The LDS a block asks for (bpftime_amd_lds_bytes: common.hpp
    dyn_lds_for + the kernel's static LDS, restated without a device): the
    override shape that failed in round 4 (flow-hash with
    BPFTIME_AMD_COMB_ENTRIES=2000 BPFTIME_AMD_LCACHE_SETS=2048, 1024-lane
    blocks) exceeds the CU's 160 KiB and is refused by name before a launch
    (vm_api.cpp lds_fit_error); the default flow-hash and headline shapes
    fit."""
    l = _lib.lib()
    cu = 160 * 1024
    xdp, syscall = 1, 2
    # kind, big_stack, stack, comb entries, lcache sets, ctx in LDS, gregs, block
    bad = l.bpftime_amd_lds_bytes(xdp, False, 32, 2000, 2048, False, True, 1024)
    assert bad > cu
    flow = l.bpftime_amd_lds_bytes(xdp, False, 32, 2800, 1024, False, True, 1024)
    assert flow <= cu
    head = l.bpftime_amd_lds_bytes(xdp, False, 8, 0, 0, False, False, 256)
    assert head <= cu // 4           # four headline blocks per CU
    # the parts add up: each 8 entries of the combining table 8 tags + a
    # 144-B delta row (common.hpp kCombRowBytes), each lookup set 40 B, each
    # lane's stack its bytes at a stride of 8 x an odd number (lane_stride:
    # with BPFTIME_AMD_LANE_PAD=1: 32 and 40 -> 40, 48 -> 56; unpadded by default)
    assert l.bpftime_amd_lds_bytes(xdp, False, 32, 2008, 2048, False, True, 1024) - bad == 8 * 4 + 144
    assert l.bpftime_amd_lds_bytes(xdp, False, 32, 2000, 2049, False, True, 1024) - bad == 40
    pad = os.environ.get("BPFTIME_AMD_LANE_PAD", "0") not in ("", "0")
    assert l.bpftime_amd_lds_bytes(xdp, False, 40, 2000, 2048, False, True, 1024) - bad == (0 if pad else 8 * 1024)
    assert l.bpftime_amd_lds_bytes(xdp, False, 48, 2000, 2048, False, True, 1024) - bad == (16 if pad else 16) * 1024
    assert l.bpftime_amd_lds_bytes(syscall, False, 32, 512, 2048, True, True, 1024) < cu
