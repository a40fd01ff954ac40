"""The sys_exit half of the syscall dispatch on the device
(attach/syscall_trace_attach_impl/src/syscall_trace_attach_impl.cpp:18-166;
trace_event_raw_sys_exit at include/syscall_trace_attach_impl.hpp:31-36),
through the C ABI against the oracle's record-by-record dispatch
(tests/test_oracle_syscall_exit.py pins that oracle against numpy):

* syscount's sys_exit program (example/tracing/syscount/syscount.bpf.c:49-87)
  at 2^22 96-B records with negative rets and id == -1 records, each option
  of its .rodata, bit-exact (every data_t of the HASH map) -- the per-record
  return values too;
* enter + exit programs with bpf_override_return at sys_enter (the record
  returns the override and its exit programs do not run) and bpf_set_retval
  at sys_exit, per-syscall and global, bit-exact in returns and counters;
* a program that stores into its ctx runs on a copy, as each reference
  callback gets its own (:43-45): the next program sees the record unchanged;
* the named error of a launch whose block does not fit the CU's LDS.
"""
import os
import struct

import numpy as np
import pytest

from bpftime_amd import _lib, gen, isa, programs
from bpftime_amd.isa import Asm

from _helpers import make_maps

pytestmark = pytest.mark.gpu

TRACEPOINT = 5  # BPF_PROG_TYPE_TRACEPOINT


def _syscount_maps(po, dev, **opts):
    (od, oro), (dd, dro) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192),
                                      (isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1)], po, dev)
    ro = programs.syscount_rodata(**opts)
    assert oro.update(b"\0" * 4, ro) == 0 and dro.update(b"\0" * 4, ro) == 0
    return od, dd, dro.fd


@pytest.mark.parametrize("opts", [{}, {"filter_failed": True}, {"filter_errno": 2},
                                  {"count_by_process": True}])
def test_syscount_exit_bit_exact(fresh_oracle, fresh_runtime, opts):
    po, dev = fresh_oracle, fresh_runtime
    od, dd, ro_fd = _syscount_maps(po, dev, **opts)
    code = programs.syscount_exit(dd.fd, ro_fd)
    n = 1 << 22
    recs = gen.syscall_records_full(n)
    w = recs.view(np.int64).reshape(n, 12)
    assert (w[:, 9] == -1).sum() > 1000 and (w[:, 10] < 0).sum() > n // 8
    pfd = dev.prog_create(code, "sys_exit", TRACEPOINT)
    aid = dev.syscall_attach(pfd, -1, enter=False)
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    assert dev.syscall_dispatch(d, n, out=out) == 0
    o = po.OracleSyscallDispatch()
    o.attach(code, -1, enter=False)
    want = o.dispatch(recs)
    assert dd.hash_items() == od.items()
    assert len(od.items()) > 50 if not opts.get("count_by_process") else len(od.items()) == 64
    assert (out.download(np.int64) == want).all()
    assert (want == w[:, 10]).all()
    # the device generator writes the same records
    d2 = dev.DeviceBuffer(96 * n)
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(335, 1.2))
    assert _lib.lib().bpftime_amd_gen_syscall_full(d2.ptr, n, gen.SEED_CFG5, 0, cdf.ptr, 335, None) == 0
    assert (d2.download().reshape(n, 96) == recs).all()
    assert dev.syscall_detach(aid) == 0


def _counter(map_fd, slot):
    return (Asm().ld_map_value(2, map_fd, 8 * slot).ldx(8, 3, 2, 0).add64(3, 1).stx(8, 2, 0, "r3")
            .mov64(0, 0).exit().assemble())


@pytest.mark.parametrize("ordered", [False, True])
def test_enter_override_and_exit_retval(fresh_oracle, fresh_runtime, ordered):
    po, dev = fresh_oracle, fresh_runtime
    (ocnt,), (dcnt,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 64, 1)], po, dev)
    progs = [(programs.inject_enter(3, -1), 1, True),        # sys_enter_write: override
             (_counter(dcnt.fd, 0), -1, True),
             (_counter(dcnt.fd, 1), -1, False),
             (programs.exit_clamp(0), -1, False),            # sys_exit: set_retval
             (_counter(dcnt.fd, 2), 0, False),               # sys_exit_read
             (programs.inject_enter(5, 99), 3, True)]        # sys_enter_close
    o = po.OracleSyscallDispatch()
    for code, nr, enter in progs:
        dev.syscall_attach(dev.prog_create(code, "p", TRACEPOINT), nr, enter)
        o.attach(code, nr, enter)
    n = 1 << 16 if ordered else 1 << 21
    recs = gen.syscall_records_full(n)
    w = recs.view(np.int64).reshape(n, 12)
    w[::7, 1] = w[::7, 9] = 1
    w[3::97, 1] = w[3::97, 9] = 700                         # past the callback arrays: globals only
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    flags = dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0)
    assert dev.syscall_dispatch(d, n, out=out, flags=flags) == 0
    want = o.dispatch(recs)
    got = out.download(np.int64)
    assert (got == want).all(), np.flatnonzero(got != want)[:10]
    assert dcnt.lookup(b"\0" * 4) == ocnt.lookup(b"\0" * 4)
    c = struct.unpack("<8Q", ocnt.lookup(b"\0" * 4))
    assert c[1] < c[0] and c[2] > 0 and (want == -1).sum() > n // 40 and (want == 99).sum() > 0
    # the records were not written
    assert (d.download().reshape(n, 96) == recs).all()
    # without out_rets the exit programs still skip overridden records
    assert dev.syscall_dispatch(d, n, flags=flags) == 0
    o.dispatch(recs)
    assert dcnt.lookup(b"\0" * 4) == ocnt.lookup(b"\0" * 4)


def test_ctx_store_runs_on_a_copy(fresh_oracle, fresh_runtime):
    """An enter program that overwrites args[0] and counts it, then a global
    enter program and an exit program that sum what they read: the reference
    gives each callback a fresh ctx copy, so the later ones see the record."""
    po, dev = fresh_oracle, fresh_runtime
    (osum,), (dsum,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 32, 1)], po, dev)
    writer = (Asm().st(8, 1, 16, 12345).ldx(8, 3, 1, 16).ld_map_value(2, dsum.fd, 0).atomic(8, isa.ATOMIC_ADD, 2, 0, 3)
              .mov64(0, 0).exit().assemble())
    reader = (Asm().ldx(8, 3, 1, 16).ld_map_value(2, dsum.fd, 8).atomic(8, isa.ATOMIC_ADD, 2, 0, 3)
              .mov64(0, 0).exit().assemble())
    xreader = (Asm().st(8, 1, 16, 3).ldx(8, 3, 1, 16).ld_map_value(2, dsum.fd, 16).atomic(8, isa.ATOMIC_ADD, 2, 0, 3)
               .mov64(0, 0).exit().assemble())
    xsum = (Asm().ldx(8, 3, 1, 16).ld_map_value(2, dsum.fd, 24).atomic(8, isa.ATOMIC_ADD, 2, 0, 3)
            .mov64(0, 0).exit().assemble())
    o = po.OracleSyscallDispatch()
    for code, nr, enter in ((writer, 0, True), (reader, -1, True), (xreader, -1, False), (xsum, -1, False)):
        dev.syscall_attach(dev.prog_create(code, "p", TRACEPOINT), nr, enter)
        o.attach(code, nr, enter)
    n = 1 << 18
    recs = gen.syscall_records_full(n)
    d = dev.DeviceBuffer.from_array(recs)
    assert dev.syscall_dispatch(d, n) == 0
    o.dispatch(recs)
    assert dsum.lookup(b"\0" * 4) == osum.lookup(b"\0" * 4)
    s = struct.unpack("<4Q", osum.lookup(b"\0" * 4))
    w = recs.view(np.int64).reshape(n, 12)
    live = ~np.isin(w[:, 1], [60, 231])
    assert s[1] == int(w[live, 2].view(np.uint64).sum(dtype=np.uint64))   # args[0] as recorded
    assert s[3] == int(w[live, 10].view(np.uint64).sum(dtype=np.uint64))  # ret as recorded
    assert (d.download().reshape(n, 96) == recs).all()


def test_dispatch_errors(fresh_runtime):
    dev = fresh_runtime
    code = programs.exit_clamp()
    pfd = dev.prog_create(code, "p", TRACEPOINT)
    l = _lib.lib()
    assert l.bpftime_amd_syscall_attach_ex(pfd, 512, 0) < 0
    assert l.bpftime_amd_syscall_attach_ex(pfd, -2, 1) < 0
    i = dev.syscall_attach(pfd, -1, enter=False)
    d = dev.DeviceBuffer(96 * 16)
    with pytest.raises(dev.EbpfError, match="96-B form"):
        dev.syscall_dispatch(d, 16, record_size=64)
    with pytest.raises(dev.EbpfError, match="record size"):
        dev.syscall_dispatch(d, 16, record_size=80)
    assert dev.syscall_detach(i) == 0 and dev.syscall_detach(i) < 0
    # bpf_set_retval with no dispatch: the unit fails (the reference throws)
    vm = dev.VM()
    vm.load(code)
    recs = np.zeros((4, 96), np.uint8)
    w = recs.view(np.int64)
    w[:, 9], w[:, 10] = 1, -5
    d = dev.DeviceBuffer.from_array(recs)
    assert vm.exec_batch(dev.CTX_SYSCALL_EXIT, d, 4, 96, data_offset=64) == 4
    w[:, 10] = 5
    d = dev.DeviceBuffer.from_array(recs)
    assert vm.exec_batch(dev.CTX_SYSCALL_EXIT, d, 4, 96, data_offset=64) == 0


def test_lds_overflow_is_named(fresh_runtime, monkeypatch):
    """A combining table the CU cannot hold beside the block's other LDS
    (BPFTIME_AMD_COMB_ENTRIES) fails the batch with a named error, before
    any launch; the next batch without it runs."""
    dev = fresh_runtime
    flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, 1 << 16)
    vm = dev.VM()
    vm.load(programs.flow_hash(flows.fd))
    n = 1 << 16
    pk, lens = gen.flow_packets(n, nflows=4096, stride=2048)
    d = dev.DeviceBuffer.from_array(pk)
    ld = dev.DeviceBuffer.from_array(lens)
    v = dev.DeviceBuffer(4 * n)
    monkeypatch.setenv("BPFTIME_AMD_COMB_ENTRIES", "8000")
    with pytest.raises(dev.EbpfError, match="does not fit the CU's LDS"):
        vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=ld, verdicts=v)
    monkeypatch.delenv("BPFTIME_AMD_COMB_ENTRIES")
    assert vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=ld, verdicts=v) == 0
