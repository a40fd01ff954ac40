"""The oracle's syscall dispatch with both halves (attach/syscall_trace_attach_impl/
src/syscall_trace_attach_impl.cpp:18-166; ctx layouts include/
syscall_trace_attach_impl.hpp:17-36), pinned on CPU before the device is
compared with it:

* syscount's sys_exit program (example/tracing/syscount/syscount.bpf.c:49-87)
  over 96-B replay records against an independent numpy count of the same
  records (the id == -1 skip, filter_failed / filter_errno on ret,
  count_by_process on the recorded caller's pid, exit / exit_group skipped by
  the dispatch);
* dispatch_syscall's order and return: per-syscall then global programs,
  enter before exit, an enter override (bpf_override_return) returns at once
  and skips the exit programs, an exit bpf_set_retval replaces ret, exit /
  exit_group return ret with no program run, ids outside [0, 512) reach only
  the global programs;
* the override helpers outside a dispatch fail the exec (the reference
  throws when no return callback is set, base_attach_impl.hpp:94-105).
"""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs
from bpftime_amd.isa import Asm

DATA_T = 32
MAX_ENTRIES = 8192  # syscount.h


def _maps(po, count_by_process=False, filter_failed=False, filter_errno=0, filter_pid=0):
    data = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, DATA_T, MAX_ENTRIES)
    ro = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1)
    ro.update(b"\0" * 4, programs.syscount_rodata(count_by_process, filter_failed, filter_errno, filter_pid))
    return data, ro


def _counts(m):
    return {struct.unpack("<I", k)[0]: struct.unpack("<Q", v[:8])[0] for k, v in m.items().items()}


def _expected(recs, count_by_process=False, filter_failed=False, filter_errno=0, filter_pid=0):
    w = recs.view(np.int64).reshape(len(recs), 12)
    ids, ret, pt = w[:, 9], w[:, 10], w[:, 11].view(np.uint64)
    pid = (pt >> np.uint64(32)).astype(np.int64)
    keep = ~np.isin(ids, [60, 231]) & (ids != -1)
    if filter_pid:
        keep &= pid == filter_pid
    if filter_failed:
        keep &= ret < 0
    if filter_errno:
        keep &= ret == -filter_errno
    key = pid if count_by_process else ids
    k, c = np.unique(key[keep], return_counts=True)
    return {int(a) & 0xFFFFFFFF: int(b) for a, b in zip(k, c)}


@pytest.mark.parametrize("opts", [{}, {"filter_failed": True}, {"filter_errno": 13},
                                  {"count_by_process": True}, {"filter_pid": 1005, "filter_failed": True}])
def test_syscount_exit_counts(fresh_oracle, opts):
    po = fresh_oracle
    data, ro = _maps(po, **opts)
    n = 60000
    recs = gen.syscall_records_full(n)
    d = po.OracleSyscallDispatch()
    assert d.attach(programs.syscount_exit(data.fd, ro.fd), -1, enter=False) > 0
    out = d.dispatch(recs)
    assert _counts(data) == _expected(recs, **opts)
    # no program overrides: every record returns its recorded ret
    assert (out == recs.view(np.int64).reshape(n, 12)[:, 10]).all()


def test_generator_fields():
    n = 20000
    recs = gen.syscall_records_full(n)
    w = recs.view(np.int64).reshape(n, 12)
    enter = gen.syscall_records(n).view(np.int64).reshape(n, 8)
    assert (w[:, 0] == 0).all() and (w[:, 8] == 0).all()        # ent zeroed in both ctxs
    assert (w[:, 1] == w[:, 9]).all()                             # one id per record
    same = w[:, 1] != -1
    assert (w[same, :8] == enter[same]).all()                     # the config 5 enter record
    assert 0.003 < (~same).mean() < 0.008                         # id -1: 0.5 %
    assert 0.17 < (w[:, 10] < 0).mean() < 0.23 and w[:, 10].min() >= -133
    tgid = w[:, 11].view(np.uint64) >> np.uint64(32)
    assert tgid.min() >= 1000 and tgid.max() < 1064


def _counter(map_fd, slot):
    """counters[slot] += 1; returns 0 (a program of either ctx kind)."""
    return (Asm().ld_map_value(2, map_fd, 8 * slot).ldx(8, 3, 2, 0).add64(3, 1).stx(8, 2, 0, "r3")
            .mov64(0, 0).exit().assemble())


def _order_prog(map_fd, slot, tag):
    """log[slot] = log[slot] * 16 + tag: the order programs run in is the
    digits of the value."""
    return (Asm().ld_map_value(2, map_fd, 8 * slot).ldx(8, 3, 2, 0).alu64("lsh", 3, 4).add64(3, tag)
            .stx(8, 2, 0, "r3").mov64(0, 0).exit().assemble())


def test_dispatch_order_overrides_and_returns(fresh_oracle):
    po = fresh_oracle
    cnt = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 64, 1)
    d = po.OracleSyscallDispatch()
    # attach out of order: global exit, per-nr exit, global enter, per-nr enter
    d.attach(_order_prog(cnt.fd, 0, 4), -1, enter=False)
    d.attach(_order_prog(cnt.fd, 0, 3), 1, enter=False)
    d.attach(_order_prog(cnt.fd, 0, 2), -1, enter=True)
    d.attach(_order_prog(cnt.fd, 0, 1), 1, enter=True)
    rec = np.zeros((1, 96), np.uint8)
    w = rec.view(np.int64)
    w[0, 1] = w[0, 9] = 1
    w[0, 10] = 77
    assert d.dispatch(rec)[0] == 77
    assert struct.unpack("<Q", cnt.lookup(b"\0" * 4)[:8])[0] == 0x1234


def test_dispatch_override_semantics(fresh_oracle):
    po = fresh_oracle
    cnt = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 64, 1)
    d = po.OracleSyscallDispatch()
    d.attach(programs.inject_enter(3, -1), 1, enter=True)      # write: override when args[2] % 3 == 0
    d.attach(_counter(cnt.fd, 0), -1, enter=True)              # every entered record
    d.attach(_counter(cnt.fd, 1), -1, enter=False)             # every exited record
    d.attach(programs.exit_clamp(0), -1, enter=False)          # ret < 0 and odd id -> 0
    n = 40000
    recs = gen.syscall_records_full(n)
    w = recs.view(np.int64).reshape(n, 12)
    w[::7, 1] = w[::7, 9] = 1                                   # plenty of writes
    w[3::97, 1] = w[3::97, 9] = 700                             # ids past the callback arrays
    out = d.dispatch(recs)
    ids, args2, ret = w[:, 1], w[:, 4], w[:, 10]
    skip = np.isin(ids, [60, 231])
    ovr = ~skip & (ids == 1) & (args2 % 3 == 0)
    clamp = ~skip & ~ovr & (ret < 0) & ((ids & 1) == 1)
    want = np.where(ovr, -1, np.where(clamp, 0, ret))
    assert (out == want).all()
    c = struct.unpack("<8Q", cnt.lookup(b"\0" * 4))
    assert c[0] == (~skip).sum()          # enter programs all ran (the override comes after them)
    assert c[1] == (~skip & ~ovr).sum()   # exit programs skip the overridden records


def test_override_outside_dispatch_fails(fresh_oracle):
    po = fresh_oracle
    v = po.OracleVM()
    v.load(programs.inject_enter(1))
    ctx = bytearray(64)
    rc, _ = v.exec(ctx)
    assert rc == -1
    v2 = po.OracleVM()
    v2.load(programs.exit_clamp())
    ctx = bytearray(struct.pack("<qqq", 0, 1, -5))
    assert v2.exec(ctx)[0] == -1
    ctx = bytearray(struct.pack("<qqq", 0, 1, 5))               # no call: runs
    assert v2.exec(ctx) == (0, 0)


def test_attach_range(fresh_oracle):
    po = fresh_oracle
    d = po.OracleSyscallDispatch()
    code = programs.inject_enter(3)
    assert d.attach(code, 512) < 0 and d.attach(code, -2) < 0
    assert d.attach(code, 511) > 0 and d.attach(code, -1) > 0
    i = d.attach(code, 0, enter=False)
    assert d.detach(i) == 0 and d.detach(i) < 0
    with pytest.raises(ValueError):
        d.dispatch(np.zeros((4, 80), np.uint8))
