"""Thin Python host layer over the C ABI (test / bench convenience).

Mirrors the reference's embedder usage of the VM C ABI
(vm/example/main.c:25-51, benchmark/test_embed.c:155-168) and of the shm map
API (runtime/include/bpftime_shm.hpp:303-345).  Everything here calls
libbpftime_amd.so; nothing executes eBPF on the CPU.
"""
from __future__ import annotations

import ctypes as C
import struct
from typing import Optional

import numpy as np

from . import isa
from ._lib import BpfLinkCreateArgs, BpfMapAttr, EbpfBatch, SysRecords, lib

CTX_RAW, CTX_XDP, CTX_SYSCALL, CTX_SYSCALL_EXIT = 0, 1, 2, 3
SYSCALL_RECORD, SYSCALL_RECORD_FULL, SYSCALL_RECORD_TIMED = 64, 96, 128  # include/bpftime_amd.h replay records
DISPATCH_THREADS, DISPATCH_PROGRAMS = 0x100, 0x200  # dispatch plans (include/bpftime_amd.h)
BATCH_SYNC, BATCH_ORDERED, BATCH_UNCHECKED, BATCH_SYS_NR, BATCH_TIMED = 0x1, 0x2, 0x4, 0x8, 0x10


class EbpfError(RuntimeError):
    pass


def _err() -> str:
    e = lib().bpftime_amd_last_error()
    return e.decode() if e else ""


# ---------------------------------------------------------------------------
# device memory
# ---------------------------------------------------------------------------
class DeviceBuffer:
    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = lib().bpftime_amd_dev_alloc(max(self.nbytes, 1))
        if not self.ptr:
            raise EbpfError(f"device alloc of {nbytes} bytes failed")

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(a)
        if lib().bpftime_amd_memcpy_htod(C.c_void_p(self.ptr + offset), a.ctypes.data, a.nbytes):
            raise EbpfError("htod failed")

    def download(self, dtype=np.uint8, count: Optional[int] = None, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        n = (self.nbytes - offset) // dt.itemsize if count is None else count
        out = np.empty(n, dtype=dt)
        if n and lib().bpftime_amd_memcpy_dtoh(out.ctypes.data, C.c_void_p(self.ptr + offset), out.nbytes):
            raise EbpfError("dtoh failed")
        return out

    def zero(self) -> None:
        lib().bpftime_amd_memset(C.c_void_p(self.ptr), 0, self.nbytes)

    def free(self) -> None:
        if self.ptr:
            lib().bpftime_amd_dev_free(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# maps
# ---------------------------------------------------------------------------
class Map:
    def __init__(self, type_: int, key_size: int, value_size: int, max_entries: int, flags: int = 0,
                 name: str = "", fd: int = -1):
        attr = BpfMapAttr(type=type_, key_size=key_size, value_size=value_size, max_ents=max_entries,
                          flags=flags)
        self.fd = lib().bpftime_maps_create(fd, name.encode(), attr)
        if self.fd < 0:
            raise EbpfError(f"map create failed: {_err()}")
        self.type, self.key_size, self.value_size, self.max_entries = type_, key_size, value_size, max_entries

    @classmethod
    def from_fd(cls, fd: int) -> "Map":
        """Wrap a map record created elsewhere (e.g. by BpfObject.load)."""
        if not lib().bpftime_is_map_fd(fd):
            raise EbpfError(f"fd {fd} is not a map")
        m = cls.__new__(cls)
        m.fd = fd
        a = BpfMapAttr()
        if lib().bpftime_map_get_info(fd, C.byref(a), None, None) < 0:
            raise EbpfError(f"fd {fd}: no map info")
        m.type, m.key_size, m.value_size, m.max_entries = a.type, a.key_size, a.value_size, a.max_ents
        return m

    def ringbuf_fetch(self, cap: int = 1 << 24) -> list:
        """Consume committed ring-buffer records (BPF_MAP_TYPE_RINGBUF)."""
        buf = C.create_string_buffer(cap)
        used = C.c_uint64(0)
        n = lib().bpftime_amd_ringbuf_fetch(self.fd, buf, cap, C.byref(used))
        if n < 0:
            raise EbpfError(f"ringbuf fetch failed: {_err()}")
        raw, out, off = buf.raw[:used.value], [], 0
        for _ in range(n):
            ln = int.from_bytes(raw[off:off + 4], "little")
            out.append(raw[off + 4:off + 4 + ln])
            off += 4 + ln
        return out

    @property
    def user_value_size(self) -> int:
        return lib().bpftime_map_value_size_from_syscall(self.fd)

    def lookup(self, key: bytes) -> Optional[bytes]:
        k = C.create_string_buffer(bytes(key), len(key))
        p = lib().bpftime_map_lookup_elem(self.fd, k)
        if not p:
            return None
        return C.string_at(p, self.user_value_size)

    def update(self, key: bytes, value: bytes, flags: int = 0) -> int:
        k = C.create_string_buffer(bytes(key), len(key))
        v = C.create_string_buffer(bytes(value), len(value))
        return lib().bpftime_map_update_elem(self.fd, k, v, flags)

    def delete(self, key: bytes) -> int:
        k = C.create_string_buffer(bytes(key), len(key))
        return lib().bpftime_map_delete_elem(self.fd, k)

    def next_key(self, key: Optional[bytes]) -> Optional[bytes]:
        out = C.create_string_buffer(self.key_size)
        kb = C.create_string_buffer(bytes(key), len(key)) if key is not None else None
        if lib().bpftime_map_get_next_key(self.fd, kb, out) < 0:
            return None
        return out.raw

    def storage_bytes(self) -> int:
        n = C.c_uint64(0)
        lib().bpftime_amd_map_device_ptr(self.fd, C.byref(n))
        return n.value

    def device_ptr(self) -> int:
        return lib().bpftime_amd_map_device_ptr(self.fd, None)

    def snapshot(self) -> np.ndarray:
        n = self.storage_bytes()
        out = np.empty(n, dtype=np.uint8)
        if lib().bpftime_amd_map_snapshot(self.fd, out.ctypes.data, n):
            raise EbpfError("snapshot failed")
        return out

    def restore(self, raw: np.ndarray) -> None:
        raw = np.ascontiguousarray(raw, dtype=np.uint8)
        if lib().bpftime_amd_map_restore(self.fd, raw.ctypes.data, raw.nbytes):
            raise EbpfError("restore failed")

    def geometry(self):
        nb, ss, ko, vo, nc = C.c_uint64(), C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        lib().bpftime_amd_map_geometry(self.fd, C.byref(nb), C.byref(ss), C.byref(ko), C.byref(vo), C.byref(nc))
        return nb.value, ss.value, ko.value, vo.value, nc.value

    def hash_items(self) -> dict:
        """Decode a (per-CPU) hash map snapshot into {key: value-bytes}."""
        nb, ss, ko, vo, nc = self.geometry()
        raw = self.snapshot().reshape(nb, ss)
        vs = self.value_size * (nc if self.type == isa.BPF_MAP_TYPE_PERCPU_HASH else 1)
        filled = raw[:, :4].view(np.uint32)[:, 0] == 1
        out = {}
        for row in raw[filled]:
            out[bytes(row[ko:ko + self.key_size])] = bytes(row[vo:vo + vs])
        return out

    def count(self) -> int:
        return lib().bpftime_amd_map_count(self.fd)

    def close(self) -> None:
        lib().bpftime_close(self.fd)


def close_fd(fd: int) -> None:
    """bpftime_close: a map, prog or link record (a closed prog leaves the
    prog arrays that name it, prog_array.cpp:127-131)."""
    lib().bpftime_close(fd)


def reset_runtime() -> None:
    lib().bpftime_amd_reset()


def set_ncpu(n: int) -> None:
    lib().bpftime_amd_set_ncpu(n)


# ---------------------------------------------------------------------------
# VM
# ---------------------------------------------------------------------------
class VM:
    def __init__(self, name: str = "mi355x", default_helpers: bool = True):
        self.h = lib().ebpf_create(name.encode())
        if not self.h:
            raise EbpfError(f"ebpf_create({name!r}) failed")
        if default_helpers:
            lib().bpftime_amd_register_default_helpers(C.c_void_p(self.h))

    def register(self, index: int, name: str) -> int:
        return lib().ebpf_register(C.c_void_p(self.h), index, name.encode(), None)

    def set_unwind(self, idx: int) -> int:
        """ebpf_set_unwind_function_index (idx = the ubpf id a helper was
        registered under: the order of registration, from 1)."""
        return lib().ebpf_set_unwind_function_index(C.c_void_p(self.h), idx)

    def load(self, code: bytes) -> None:
        err = C.c_void_p()
        buf = C.create_string_buffer(code, len(code))
        rc = lib().ebpf_load(C.c_void_p(self.h), buf, len(code), C.byref(err))
        if rc < 0:
            msg = C.string_at(err.value).decode() if err.value else "?"
            raise EbpfError(msg)

    def try_load(self, code: bytes):
        """(rc, errmsg) like ebpf_load."""
        err = C.c_void_p()
        buf = C.create_string_buffer(code, len(code))
        rc = lib().ebpf_load(C.c_void_p(self.h), buf, len(code), C.byref(err))
        return rc, (C.string_at(err.value).decode() if err.value else "")

    def unload(self) -> None:
        lib().ebpf_unload_code(C.c_void_p(self.h))

    def set_ctx_kind(self, kind: int) -> None:
        lib().ebpf_set_ctx_kind(C.c_void_p(self.h), kind)

    def exec(self, mem: bytearray) -> tuple:
        """ebpf_exec on a host buffer (copied to the GPU and back)."""
        buf = (C.c_uint8 * len(mem)).from_buffer(mem) if len(mem) else None
        ret = C.c_uint64(0)
        rc = lib().ebpf_exec(C.c_void_p(self.h), buf, len(mem), C.byref(ret))
        return rc, ret.value

    def info(self) -> dict:
        ss, big, fused, n = C.c_uint32(), C.c_int(), C.c_uint32(), C.c_uint32()
        lib().bpftime_amd_vm_info(C.c_void_p(self.h), C.byref(ss), C.byref(big), C.byref(fused), C.byref(n))
        return {"stack_size": ss.value, "big_stack": bool(big.value), "fused_rmw": fused.value,
                "n_insns": n.value}

    def fast_specialized(self, kind: int) -> int:
        n = C.c_uint32()
        if lib().bpftime_amd_vm_fast_info(C.c_void_p(self.h), kind, C.byref(n)):
            raise EbpfError("vm_fast_info failed")
        return n.value

    def counter_info(self, kind: int) -> tuple:
        """(deferred, direct) counter-add sites for the entry form of `kind`."""
        d, n = C.c_uint32(), C.c_uint32()
        if lib().bpftime_amd_vm_counter_info(C.c_void_p(self.h), kind, C.byref(d), C.byref(n)):
            raise EbpfError("vm_counter_info failed")
        return d.value, n.value

    def set_step_limit(self, n: int) -> None:
        lib().bpftime_amd_set_step_limit(C.c_void_p(self.h), n)

    def last_batch_ms(self) -> float:
        """Kernel time of this VM's last BATCH_TIMED batch (ms; -1 none)."""
        return lib().bpftime_amd_last_batch_ms(self.h)

    def exec_batch(self, kind: int, data: DeviceBuffer, count: int, stride: int, fixed_len: int = 0,
                   lens: Optional[DeviceBuffer] = None, verdicts: Optional[DeviceBuffer] = None,
                   rets: Optional[DeviceBuffer] = None, data_off_out: Optional[DeviceBuffer] = None,
                   len_out: Optional[DeviceBuffer] = None, flags: int = BATCH_SYNC, first_unit: int = 0,
                   head: int = 0, data_offset: int = 0, ifindex: int = 0, rxq: int = 0,
                   stream: int = 0, descs: Optional[DeviceBuffer] = None, umem_bytes: int = 0,
                   sys_nr: Optional[int] = None, pid_tgid_off: int = 0, ktime_off: int = 0) -> int:
        """descs: AF_XDP descriptor mode ({u64 addr; u32 len; u32 options} per
        unit, frames at data + addr inside umem_bytes; stride = chunk size).
        pid_tgid_off / ktime_off: the recorded caller / clock of a syscall
        replay unit (include/ebpf-vm.h)."""
        b = EbpfBatch(ctx_kind=kind, flags=flags, count=count, data=data.ptr + data_offset, stride=stride,
                      lens=lens.ptr if lens else None, fixed_len=fixed_len, ingress_ifindex=ifindex,
                      rx_queue_index=rxq, head=head, verdicts=verdicts.ptr if verdicts else None,
                      rets=rets.ptr if rets else None,
                      data_off_out=data_off_out.ptr if data_off_out else None,
                      len_out=len_out.ptr if len_out else None, first_unit=first_unit,
                      stream=stream or None, descs=descs.ptr if descs else None, umem_bytes=umem_bytes,
                      sys_nr=-1 if sys_nr is None else sys_nr, pid_tgid_off=pid_tgid_off,
                      ktime_off=ktime_off)
        if sys_nr is not None:
            b.flags |= BATCH_SYS_NR
        rc = lib().ebpf_exec_batch(C.c_void_p(self.h), C.byref(b))
        if rc < 0:
            e = lib().bpftime_amd_vm_error(C.c_void_p(self.h))
            raise EbpfError(f"ebpf_exec_batch failed: {e.decode() if e else '?'}")
        return rc

    def close(self) -> None:
        if self.h:
            lib().ebpf_destroy(C.c_void_p(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# prog / link records (the bpf_link attach surface)
# ---------------------------------------------------------------------------
def prog_create(code: bytes, name: str, prog_type: int, fd: int = -1) -> int:
    buf = C.create_string_buffer(code, len(code))
    r = lib().bpftime_progs_create(fd, buf, len(code) // 8, name.encode(), prog_type)
    if r < 0:
        raise EbpfError("prog create failed")
    return r


def link_create(prog_fd: int, target: int, attach_type: int, fd: int = -1) -> int:
    a = BpfLinkCreateArgs(prog_fd=prog_fd, target_fd=target, attach_type=attach_type)
    return lib().bpftime_link_create(fd, C.byref(a))


def syscall_attach(prog_fd: int, sys_nr: int, enter: bool = True) -> int:
    """A program on the sys_enter / sys_exit tracepoint of sys_nr (-1: every
    syscall; syscall_trace_attach_impl.cpp:121-166): the attach id."""
    i = lib().bpftime_amd_syscall_attach_ex(prog_fd, sys_nr, 1 if enter else 0)
    if i < 0:
        raise EbpfError(f"syscall attach failed: {_err()}")
    return i


def syscall_detach(i: int) -> int:
    return lib().bpftime_amd_syscall_detach(i)


def syscall_dispatch(records: DeviceBuffer, n: int, record_size: int = SYSCALL_RECORD_FULL,
                     out: Optional[DeviceBuffer] = None, flags: int = BATCH_SYNC, stream: int = 0) -> int:
    """dispatch_syscall over n recorded calls (64-B enter, 96-B enter + exit
    + caller, or 128-B records with the recorded clocks too); out (i64 per
    record) receives what each call returns.  flags: BATCH_* and the plan
    (DISPATCH_THREADS / DISPATCH_PROGRAMS; default: chosen from the attached
    programs' map effects, syscall_dispatch_plan)."""
    rc = lib().bpftime_amd_syscall_dispatch_records(records.ptr, n, record_size, out.ptr if out else None,
                                                     flags, stream or None)
    if rc < 0:
        raise EbpfError(f"syscall dispatch failed: {_err()}")
    return rc


def syscall_dispatch_soa(exit: Optional[DeviceBuffer], n: int, enter: Optional[DeviceBuffer] = None,
                         clock: Optional[DeviceBuffer] = None, out: Optional[DeviceBuffer] = None,
                         flags: int = BATCH_SYNC, stream: int = 0) -> int:
    """dispatch_syscall over n recorded calls in struct-of-arrays form
    (include/bpftime_amd.h struct bpftime_amd_sys_records): exit (n x 32 B
    {exit ctx, pid_tgid}), enter (n x 64 B, optional), clock (n x 16 B,
    optional)."""
    r = SysRecords(enter=enter.ptr if enter else None, exit=exit.ptr if exit else None,
                   clock=clock.ptr if clock else None, count=n)
    rc = lib().bpftime_amd_syscall_dispatch_soa(C.byref(r), out.ptr if out else None, flags, stream or None)
    if rc < 0:
        raise EbpfError(f"syscall dispatch failed: {_err()}")
    return rc


def syscall_dispatch_plan(flags: int = 0) -> int:
    """1 when a dispatch with these flags runs thread-ordered for the
    current attachments, 0 program-major."""
    rc = lib().bpftime_amd_syscall_dispatch_plan(flags)
    if rc < 0:
        raise EbpfError(f"syscall dispatch plan failed: {_err()}")
    return rc


def xdp_links() -> list:
    n = lib().bpftime_amd_xdp_links(None, None, None, 0)
    lf, pf, ifx = (C.c_int * max(n, 1))(), (C.c_int * max(n, 1))(), (C.c_uint32 * max(n, 1))()
    lib().bpftime_amd_xdp_links(lf, pf, ifx, n)
    return [(lf[i], pf[i], ifx[i]) for i in range(n)]


def hip_runtime() -> dict:
    """The HIP runtime this process's library runs on: hipRuntimeGetVersion
    and the libamdhip64 file mapped into the process (torch bundles its own
    with the same SONAME)."""
    ver = lib().bpftime_amd_hip_runtime_version()
    libs = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if "libamdhip64" in p:
                    libs.add(p)
    except OSError:
        pass
    return {"version": ver, "lib": sorted(libs)}


def prog_instantiate(prog_fd: int) -> VM:
    err = C.c_void_p()
    h = lib().bpftime_amd_prog_instantiate(prog_fd, C.byref(err))
    if not h:
        raise EbpfError(C.string_at(err.value).decode() if err.value else "instantiate failed")
    vm = VM.__new__(VM)
    vm.h = h
    return vm


class Event:
    def __init__(self):
        self.h = lib().bpftime_amd_event_create()

    def record(self, stream: int = 0) -> None:
        lib().bpftime_amd_event_record(C.c_void_p(self.h), C.c_void_p(stream) if stream else None)

    def elapsed_ms(self, later: "Event") -> float:
        return lib().bpftime_amd_event_elapsed_ms(C.c_void_p(self.h), C.c_void_p(later.h))

    def __del__(self):
        try:
            lib().bpftime_amd_event_destroy(C.c_void_p(self.h))
        except Exception:
            pass


# ---- bpf(2) commands (syscall_context.cpp:429-668) --------------------------
BPF_MAP_CREATE, BPF_MAP_LOOKUP_ELEM, BPF_MAP_UPDATE_ELEM, BPF_MAP_DELETE_ELEM = 0, 1, 2, 3
BPF_MAP_GET_NEXT_KEY, BPF_PROG_LOAD, BPF_MAP_FREEZE, BPF_LINK_CREATE = 4, 5, 22, 28


def sys_bpf(cmd: int, attr: bytearray) -> tuple:
    """bpftime_amd_handle_sysbpf over a union bpf_attr image; (ret, errno)."""
    buf = (C.c_char * len(attr)).from_buffer(attr)
    C.set_errno(0)
    r = lib().bpftime_amd_handle_sysbpf(cmd, C.addressof(buf), len(attr))
    return r, C.get_errno()


def attr_map_create(type_: int, key_size: int, value_size: int, max_entries: int, flags: int = 0,
                    name: str = "") -> bytearray:
    a = bytearray(128)
    struct.pack_into("<IIIII", a, 0, type_, key_size, value_size, max_entries, flags)
    nm = name.encode()[:15]
    a[28:28 + len(nm)] = nm
    return a


def attr_map_elem(fd: int, key_addr: int, value_addr: int = 0, flags: int = 0) -> bytearray:
    a = bytearray(128)
    struct.pack_into("<IIQQQ", a, 0, fd, 0, key_addr, value_addr, flags)
    return a


def attr_prog_load(prog_type: int, insns_addr: int, insn_cnt: int, name: str = "") -> bytearray:
    a = bytearray(128)
    struct.pack_into("<IIQ", a, 0, prog_type, insn_cnt, insns_addr)
    nm = name.encode()[:15]
    a[48:48 + len(nm)] = nm
    return a


def attr_link_create(prog_fd: int, target: int, attach_type: int, flags: int = 0) -> bytearray:
    a = bytearray(128)
    struct.pack_into("<IIII", a, 0, prog_fd, target, attach_type, flags)
    return a
