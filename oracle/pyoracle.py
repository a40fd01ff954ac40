"""ctypes wrapper of oracle/build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / timed CPU baseline (see oracle/oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_l = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _l
    if _l is None:
        if not os.path.exists(LIB):
            build()
        l = C.CDLL(LIB)
        vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
        sig = {
            "orc_vm_create": (vp, []),
            "orc_vm_destroy": (None, [vp]),
            "orc_vm_register_default_helpers": (C.c_int, [vp]),
            "orc_vm_set_unwind_index": (None, [vp, C.c_int]),
            "orc_vm_load": (C.c_int, [vp, vp, u32, C.c_char_p, C.c_size_t]),
            "orc_vm_unload": (None, [vp]),
            "orc_vm_exec": (C.c_int, [vp, vp, C.c_size_t, C.POINTER(u64)]),
            "orc_vm_insn_count": (u64, [vp]),
            "orc_vm_reset_insn_count": (None, [vp]),
            "orc_maps_reset": (None, []),
            "orc_map_create": (C.c_int, [C.c_int, u32, u32, u32, u32, u32]),
            "orc_set_ncpu": (None, [C.c_int]),
            "orc_set_cpu": (None, [C.c_int]),
            "orc_map_lookup": (vp, [C.c_int, vp]),
            "orc_map_update": (C.c_long, [C.c_int, vp, vp, u64]),
            "orc_map_delete": (C.c_long, [C.c_int, vp]),
            "orc_map_lookup_user": (vp, [C.c_int, vp]),
            "orc_map_update_user": (C.c_long, [C.c_int, vp, vp, u64]),
            "orc_map_delete_user": (C.c_long, [C.c_int, vp]),
            "orc_map_get_next_key": (C.c_int, [C.c_int, vp, vp]),
            "orc_last_errno": (C.c_int, []),
            "orc_map_value_size_user": (u32, [C.c_int]),
            "orc_map_raw": (vp, [C.c_int, C.POINTER(C.c_size_t)]),
            "orc_map_buckets": (u64, [C.c_int]),
            "orc_map_count": (u64, [C.c_int]),
            "orc_ringbuf_fetch": (C.c_int64, [C.c_int, vp, u64, C.POINTER(C.c_uint64)]),
            "orc_map_ptr_by_fd": (u64, [u32]),
            "orc_prog_create": (C.c_int, [C.c_int, vp, u32]),
            "orc_prog_close": (None, [C.c_int]),
            "orc_is_prog_fd": (C.c_int, [C.c_int]),
            "orc_map_val": (u64, [u64]),
            "orc_next_prime": (u64, [u64]),
            "orc_hash_bytes": (u64, [vp, u64]),
            "orc_run_xdp": (C.c_int, [vp, vp, u64, u64, vp, u32, vp, vp, vp, u32, u32, u32]),
            "orc_vm_register_xdp_load_bytes": (C.c_int, [vp]),
            "orc_vm_register_trace_helpers": (C.c_int, [vp]),
            "orc_trace_log": (C.c_size_t, [vp, C.c_size_t]),
            "orc_trace_log_reset": (None, []),
            "orc_set_pid_tgid": (None, [u64]),
            "orc_run_raw": (C.c_int, [vp, vp, u64, u64, u32, vp]),
            "orc_run_syscall": (C.c_int, [vp, vp, u64, vp, vp]),
            "orc_time_xdp": (C.c_double, [vp, vp, u64, u64, u32, vp, C.c_int]),
            "orc_sys_attach": (C.c_int, [vp, C.c_int64, C.c_int]),
            "orc_sys_detach": (C.c_int, [C.c_int]),
            "orc_sys_reset": (None, []),
            "orc_sys_dispatch": (C.c_int, [vp, u64, u32, vp]),
        }
        for k, (r, a) in sig.items():
            f = getattr(l, k)
            f.restype, f.argtypes = r, a
        _l = l
    return _l


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


class OracleVM:
    def __init__(self, default_helpers: bool = True):
        self.h = lib().orc_vm_create()
        if default_helpers:
            lib().orc_vm_register_default_helpers(self.h)

    def load(self, code: bytes) -> None:
        rc, msg = self.try_load(code)
        if rc < 0:
            raise RuntimeError(msg)

    def try_load(self, code: bytes):
        err = C.create_string_buffer(512)
        buf = C.create_string_buffer(code, len(code))
        rc = lib().orc_vm_load(self.h, buf, len(code), err, 512)
        return rc, err.value.decode()

    def exec(self, mem: bytearray):
        buf = (C.c_uint8 * len(mem)).from_buffer(mem) if len(mem) else None
        r = C.c_uint64(0)
        rc = lib().orc_vm_exec(self.h, buf, len(mem), C.byref(r))
        return rc, r.value

    def set_unwind(self, idx: int) -> None:
        """ubpf_set_unwind_function_index (idx = ubpf helper id)."""
        lib().orc_vm_set_unwind_index(self.h, idx)

    def register_xdp_load_bytes(self) -> None:
        """bpf_xdp_load_bytes (id 189), defined but not in a default group."""
        lib().orc_vm_register_xdp_load_bytes(self.h)

    def register_trace_helpers(self) -> None:
        """bpf_trace_printk (6) and bpf_get_current_pid_tgid (14)."""
        lib().orc_vm_register_trace_helpers(self.h)

    def run_xdp(self, slots: np.ndarray, lens: Optional[np.ndarray] = None, fixed_len: int = 0,
                want_meta: bool = False, ifindex: int = 0, rxq: int = 0, ncpu: int = 0, head: int = 0):
        """slots: (n, stride) uint8, modified in place; returns verdicts (and meta).
        With ncpu > 0 the virtual CPU of unit i is (i // 64) % ncpu, like the
        device's helper 8 / per-CPU slot assignment."""
        n, stride = slots.shape
        v = np.zeros(n, dtype=np.uint32)
        off = np.zeros(n, dtype=np.int32) if want_meta else None
        ln = np.zeros(n, dtype=np.uint32) if want_meta else None
        lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint32)
        if ncpu:
            for w0 in range(0, n, 64):
                lib().orc_set_cpu((w0 // 64) % ncpu)
                m = min(64, n - w0)
                lib().orc_run_xdp(self.h, slots[w0:].ctypes.data, m, stride,
                                  None if lens is None else lens[w0:].ctypes.data, fixed_len,
                                  v[w0:].ctypes.data, None if off is None else off[w0:].ctypes.data,
                                  None if ln is None else ln[w0:].ctypes.data, ifindex, rxq, head)
        else:
            lib().orc_run_xdp(self.h, slots.ctypes.data, n, stride, _p(lens), fixed_len, v.ctypes.data,
                              _p(off), _p(ln), ifindex, rxq, head)
        return (v, off, ln) if want_meta else v

    def run_raw(self, units: np.ndarray, length: int) -> np.ndarray:
        n, stride = units.shape
        r = np.zeros(n, dtype=np.uint64)
        lib().orc_run_raw(self.h, units.ctypes.data, n, stride, length, r.ctypes.data)
        return r

    def run_syscall(self, recs: np.ndarray):
        n = recs.shape[0]
        r = np.zeros(n, dtype=np.uint64)
        ran = np.zeros(n, dtype=np.uint8)
        lib().orc_run_syscall(self.h, recs.ctypes.data, n, r.ctypes.data, ran.ctypes.data)
        return r, ran

    def time_xdp(self, slots: np.ndarray, fixed_len: int, pin_cpu: int = 0) -> float:
        n, stride = slots.shape
        v = np.zeros(n, dtype=np.uint32)
        return lib().orc_time_xdp(self.h, slots.ctypes.data, n, stride, fixed_len, v.ctypes.data, pin_cpu)

    def insn_count(self) -> int:
        return lib().orc_vm_insn_count(self.h)

    def reset_insn_count(self) -> None:
        lib().orc_vm_reset_insn_count(self.h)

    def __del__(self):
        try:
            lib().orc_vm_destroy(self.h)
        except Exception:
            pass


class OracleMap:
    def __init__(self, type_: int, key_size: int, value_size: int, max_entries: int, flags: int = 0,
                 fd: int = -1):
        self.fd = lib().orc_map_create(fd, type_, key_size, value_size, max_entries, flags)
        if self.fd < 0:
            raise RuntimeError("oracle map create failed")
        self.type, self.key_size, self.value_size, self.max_entries = type_, key_size, value_size, max_entries

    def _k(self, key: bytes):
        return C.create_string_buffer(bytes(key), max(len(key), 1))

    def lookup(self, key: bytes, user: bool = True) -> Optional[bytes]:
        f = lib().orc_map_lookup_user if user else lib().orc_map_lookup
        p = f(self.fd, self._k(key))
        if not p:
            return None
        vs = lib().orc_map_value_size_user(self.fd) if user else self.value_size
        return C.string_at(p, vs)

    def update(self, key: bytes, value: bytes, flags: int = 0, user: bool = True) -> int:
        f = lib().orc_map_update_user if user else lib().orc_map_update
        return f(self.fd, self._k(key), C.create_string_buffer(bytes(value), len(value)), flags)

    def delete(self, key: bytes, user: bool = True) -> int:
        f = lib().orc_map_delete_user if user else lib().orc_map_delete
        return f(self.fd, self._k(key))

    def next_key(self, key: Optional[bytes]) -> Optional[bytes]:
        out = C.create_string_buffer(max(self.key_size, 1))
        rc = lib().orc_map_get_next_key(self.fd, None if key is None else self._k(key), out)
        return None if rc < 0 else out.raw[: self.key_size]

    def raw(self) -> np.ndarray:
        n = C.c_size_t(0)
        p = lib().orc_map_raw(self.fd, C.byref(n))
        return np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p)).copy() if n.value else \
            np.zeros(0, np.uint8)

    def items(self) -> dict:
        """All (key -> user value) pairs, in get_next_key order."""
        out, k = {}, self.next_key(None)
        seen = 0
        while k is not None and seen <= 10_000_000:
            out[k] = self.lookup(k)
            k = self.next_key(k)
            seen += 1
        return out

    def count(self) -> int:
        return lib().orc_map_count(self.fd)

    def ringbuf_fetch(self, cap: int = 1 << 24) -> list:
        """Consume committed ring-buffer records (ringbuf::fetch_data)."""
        buf = C.create_string_buffer(cap)
        used = C.c_uint64(0)
        n = lib().orc_ringbuf_fetch(self.fd, buf, cap, C.byref(used))
        raw, out, off = buf.raw[:used.value], [], 0
        for _ in range(max(n, 0)):
            ln = int.from_bytes(raw[off:off + 4], "little")
            out.append(raw[off + 4:off + 4 + ln])
            off += 4 + ln
        return out

    def ringbuf_drain(self, cap: int = 1 << 22) -> int:
        """Consume committed records (ringbuf::fetch_data) into a reused
        buffer without decoding them: the record count."""
        if getattr(self, "_drain", None) is None or len(self._drain) < cap:
            self._drain = C.create_string_buffer(cap)
        used = C.c_uint64(0)
        return int(lib().orc_ringbuf_fetch(self.fd, self._drain, cap, C.byref(used)))

    @staticmethod
    def errno() -> int:
        return lib().orc_last_errno()


def reset() -> None:
    lib().orc_maps_reset()
    lib().orc_sys_reset()


class OracleSyscallDispatch:
    """syscall_trace_attach_impl (attach/syscall_trace_attach_impl/src/
    syscall_trace_attach_impl.cpp:18-166) over recorded calls: programs on
    sys_enter / sys_exit tracepoints, dispatched record by record."""

    def __init__(self):
        self.vms = {}

    def attach(self, code: bytes, sys_nr: int, enter: bool = True) -> int:
        v = OracleVM()
        v.load(code)
        i = lib().orc_sys_attach(v.h, sys_nr, 1 if enter else 0)
        if i > 0:
            self.vms[i] = v  # keeps the VM alive while attached
        return i

    def detach(self, i: int) -> int:
        rc = lib().orc_sys_detach(i)
        self.vms.pop(i, None)
        return rc

    def dispatch(self, recs: np.ndarray) -> np.ndarray:
        """recs: (n, 64) or (n, 96) uint8; returns what dispatch_syscall
        returns per record (int64)."""
        n, rs = recs.shape
        recs = np.ascontiguousarray(recs)
        out = np.zeros(n, dtype=np.int64)
        rc = lib().orc_sys_dispatch(recs.ctypes.data, n, rs, out.ctypes.data)
        if rc < 0:
            raise ValueError(f"orc_sys_dispatch: {rc}")
        return out


def prog_create(fd: int, code: bytes) -> int:
    """A bpftime_progs_create record (the target of bpf_tail_call)."""
    return lib().orc_prog_create(fd, bytes(code), len(code) // 8)


def prog_close(fd: int) -> None:
    lib().orc_prog_close(fd)


def trace_log() -> bytes:
    """What bpf_trace_printk printed since the last trace_log_reset()."""
    n = lib().orc_trace_log(None, 0)
    buf = C.create_string_buffer(max(n, 1))
    lib().orc_trace_log(buf, n)
    return buf.raw[:n]


def trace_log_reset() -> None:
    lib().orc_trace_log_reset()


def set_pid_tgid(v: int) -> None:
    lib().orc_set_pid_tgid(v)


def set_ncpu(n: int) -> None:
    lib().orc_set_ncpu(n)


def set_cpu(c: int) -> None:
    lib().orc_set_cpu(c)
