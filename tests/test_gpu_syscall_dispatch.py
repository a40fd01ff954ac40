"""Syscall tracepoint dispatch (attach/syscall_trace_attach_impl/src/
syscall_trace_attach_impl.cpp:18-95; the "multiple" case of its
test/test_syscall_dispatch.cpp:61-170): a global sys_enter program and
programs attached to read (0) and write (1) over recorded sys_enter records;
exit / exit_group skipped; detaching stops a program.  Counters in an ARRAY
map against the oracle run per program over the records it would see."""
import struct

import numpy as np
import pytest

from bpftime_amd import _lib, gen, isa
from bpftime_amd.isa import Asm

from _helpers import make_maps

pytestmark = pytest.mark.gpu


def counter_prog(map_fd, slot, add_arg=False):
    """counters[slot] += 1 (or += args[0]); returns 0."""
    a = Asm().mov64(6, "r1").ld_map_value(2, map_fd, 8 * slot)
    if add_arg:
        a.ldx(8, 3, 6, 16)
    else:
        a.mov64(3, 1)
    a.ldx(8, 4, 2, 0).alu64("add", 4, "r3").stx(8, 2, 0, "r4").mov64(0, 0).exit()
    return a.assemble()


def test_dispatch_per_syscall_then_global(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    L = _lib.lib()
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 32, 1)], po, dev)
    progs = {"global": (counter_prog(dm.fd, 0), -1), "read": (counter_prog(dm.fd, 1), 0),
             "write": (counter_prog(dm.fd, 2), 1), "global_args": (counter_prog(dm.fd, 3, True), -1)}
    ids = {}
    for name, (code, nr) in progs.items():
        pfd = dev.prog_create(code, name, 5)  # BPF_PROG_TYPE_TRACEPOINT
        ids[name] = L.bpftime_amd_syscall_attach(pfd, nr)
        assert ids[name] > 0
    n = 20000
    recs = gen.syscall_records(n)
    ids_col = recs.view(np.uint64).reshape(n, 8)[:, 1]
    ids_col[:] = np.array([0, 1, 57, 0, 1, 60, 231, 3], np.uint64)[np.arange(n) % 8]
    d = dev.DeviceBuffer.from_array(recs)
    assert L.bpftime_amd_syscall_dispatch(d.ptr, n, dev.BATCH_SYNC, None) == 0

    def oracle_pass(active):
        for name, (code, nr) in progs.items():
            if name not in active:
                continue
            sel = recs if nr < 0 else recs[ids_col == nr]
            v = po.OracleVM()
            v.load(code)
            v.run_syscall(sel.copy())
    oracle_pass(set(progs))
    assert dm.lookup(b"\0\0\0\0") == om.lookup(b"\0\0\0\0")
    c = struct.unpack("<QQQQ", om.lookup(b"\0\0\0\0"))
    live = ~np.isin(ids_col, [60, 231])
    assert c[0] == live.sum() and c[1] == (ids_col == 0).sum() and c[2] == (ids_col == 1).sum()
    # detach the global counter and the read program: the others keep counting
    assert L.bpftime_amd_syscall_detach(ids["global"]) == 0
    assert L.bpftime_amd_syscall_detach(ids["read"]) == 0
    assert L.bpftime_amd_syscall_detach(ids["read"]) < 0
    assert L.bpftime_amd_syscall_dispatch(d.ptr, n, dev.BATCH_SYNC, None) == 0
    oracle_pass({"write", "global_args"})
    assert dm.lookup(b"\0\0\0\0") == om.lookup(b"\0\0\0\0")
    for name in ("write", "global_args"):
        assert L.bpftime_amd_syscall_detach(ids[name]) == 0
