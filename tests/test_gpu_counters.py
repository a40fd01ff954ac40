"""Counter visibility: a unit sees its own counter increments.

The reference runs `cnt++` as ldx/add/stx one unit at a time
(runtime/src/bpftime_prog.cpp:231-260), so a later load of `cnt` in the same
unit sees the increment, and in index order unit i sees init + i + 1.  The
device fuses the three instructions into one atomic add and may sum adds
per wave / block before they reach memory -- only where nothing the unit
executes afterwards can observe the counter (loader.cpp counter_nodefer);
ORDERED batches never defer.  Checked against the oracle: bit-exact in
ORDERED mode and through ebpf_exec, and in parallel mode through the
properties any serial order has (own increment seen, exact totals, distinct
fetch results)."""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs
from bpftime_amd.isa import Asm

from _helpers import make_maps, u64s

pytestmark = pytest.mark.gpu

INIT = 1000


def _bss(po, dev, init=INIT):
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 64, 1)], po, dev)
    v = struct.pack("<Q", init) + bytes(56)
    for m in (om, dm):
        if m is not None:
            m.update(b"\0\0\0\0", v)
    return om, dm


def _run_raw(po, dev, code, n, flags):
    units = gen.sm64(7, np.arange(n, dtype=np.uint64)).view(np.uint8).reshape(n, 8)
    ovm = po.OracleVM()
    ovm.load(code)
    orets = ovm.run_raw(units.copy(), 8)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    failed = vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr, flags=flags)
    return orets, dr.download(np.uint64), failed, vm


def prog_inc_then_read(fd):
    """cnt++ (fused ldx/add/stx, r2 dead); r0 = cnt."""
    a = Asm().ld_map_value(1, fd, 0)
    a.ldx(8, 2, 1, 0).add64(2, 1).stx(8, 1, 0, "r2")
    a.ldx(8, 0, 1, 0).exit()
    return a.assemble()


def prog_inc_fetch(fd):
    """r0 = ++cnt (the loaded register stays live: the fetch form)."""
    a = Asm().ld_map_value(1, fd, 0)
    a.ldx(8, 2, 1, 0).add64(2, 1).stx(8, 1, 0, "r2")
    a.mov64(0, "r2").exit()
    return a.assemble()


def prog_atomic_then_read(fd):
    """__sync_fetch_and_add(&cnt, 1) without fetch, then r0 = cnt."""
    a = Asm().ld_map_value(1, fd, 8).mov64(3, 1)
    a.atomic(8, isa.ATOMIC_ADD, 1, 0, 3)
    a.ldx(8, 0, 1, 0).exit()
    return a.assemble()


def prog_loop_read_inc(fd):
    """Three rounds of r0 += cnt; cnt++ (the load is reached again through
    the back edge after the add)."""
    a = Asm().ld_map_value(1, fd, 0).mov64(0, 0).mov64(3, 0)
    a.label("top").jmp("jge", 3, 3, "done")
    a.ldx(8, 4, 1, 0).add64(0, "r4")
    a.ldx(8, 2, 1, 0).add64(2, 1).stx(8, 1, 0, "r2")
    a.add64(3, 1).ja("top")
    a.label("done").exit()
    return a.assemble()


def prog_inc_then_reset(fd):
    """cnt++; cnt32 = unit's low byte: the later store overwrites the add."""
    a = Asm().ldx(1, 5, 1, 0).ld_map_value(1, fd, 16)
    a.ldx(4, 2, 1, 0).add64(2, 3).stx(4, 1, 0, "r2")
    a.stx(4, 1, 0, "r5").mov64(0, 0).exit()
    return a.assemble()


@pytest.mark.parametrize("make,direct", [(prog_inc_then_read, 1), (prog_inc_fetch, 1),
                                         (prog_atomic_then_read, 1), (prog_loop_read_inc, 1),
                                         (prog_inc_then_reset, 1)])
@pytest.mark.parametrize("n", [1, 65, 3000])
def test_ordered_counter_reads_match_oracle(fresh_oracle, fresh_runtime, make, direct, n):
    po, dev = fresh_oracle, fresh_runtime
    om, dm = _bss(po, dev)
    code = make(dm.fd)
    o, d, failed, vm = _run_raw(po, dev, code, n, dev.BATCH_SYNC | dev.BATCH_ORDERED)
    assert failed == 0
    assert vm.counter_info(dev.CTX_RAW)[1] == direct
    np.testing.assert_array_equal(d, o)
    assert dm.lookup(b"\0\0\0\0") == om.lookup(b"\0\0\0\0")


def test_ebpf_exec_sees_own_increment(fresh_oracle, fresh_runtime):
    """ebpf_exec (one unit, ORDERED) repeated: r0 = init + k at call k."""
    po, dev = fresh_oracle, fresh_runtime
    om, dm = _bss(po, dev)
    code = prog_inc_then_read(dm.fd)
    ovm, vm = po.OracleVM(), dev.VM()
    ovm.load(code)
    vm.load(code)
    for k in range(1, 6):
        orc, oret = ovm.exec(bytearray(8))
        rc, ret = vm.exec(bytearray(8))
        assert rc == 0 and orc == 0 and ret == oret == INIT + k
    assert dm.lookup(b"\0\0\0\0") == om.lookup(b"\0\0\0\0")


@pytest.mark.parametrize("n", [64, 4096, 200003])
def test_parallel_unit_sees_its_increment(fresh_runtime, n):
    """Parallel mode: every unit's read includes its own add and no more
    than all of them; the final total is exact."""
    dev = fresh_runtime
    _, dm = _bss(None, dev)
    for make in (prog_inc_then_read, prog_atomic_then_read):
        code = make(dm.fd)
        vm = dev.VM()
        vm.load(code)
        assert vm.counter_info(dev.CTX_RAW) == (0, 1)
        d = dev.DeviceBuffer(8 * n)
        dr = dev.DeviceBuffer(8 * n)
        before = u64s(dm.lookup(b"\0\0\0\0"))
        slot = 0 if make is prog_inc_then_read else 1
        base = int(before[slot]) if slot == 0 else int(before[1])
        assert vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr) == 0
        r = dr.download(np.uint64).astype(np.int64)
        after = u64s(dm.lookup(b"\0\0\0\0"))
        if slot == 0:
            assert int(after[0]) == base + n
            assert (r >= base + 1).all() and (r <= base + n).all()
        else:
            # the atomic adds to cnt + 8, the read is of cnt (offset 8 too)
            assert int(after[1]) == base + n
            assert (r >= base + 1).all() and (r <= base + n).all()


@pytest.mark.parametrize("n", [64, 5000, 100000])
def test_parallel_fetch_values_distinct(fresh_runtime, n):
    """r0 = ++cnt in parallel: the adds are linearised, every unit gets a
    different value and together they are init+1 .. init+n."""
    dev = fresh_runtime
    _, dm = _bss(None, dev)
    vm = dev.VM()
    vm.load(prog_inc_fetch(dm.fd))
    d = dev.DeviceBuffer(8 * n)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr) == 0
    r = np.sort(dr.download(np.uint64))
    np.testing.assert_array_equal(r, np.arange(INIT + 1, INIT + n + 1, dtype=np.uint64))
    assert int(u64s(dm.lookup(b"\0\0\0\0"))[0]) == INIT + n


def prog_sampler(cnt_fd, rb_fd, every=64):
    """if (++cnt % every == 0) ringbuf_output(&count, 8): the count stays
    live after the increment (fetch form)."""
    a = Asm().ld_map_value(6, cnt_fd, 0)
    a.ldx(8, 2, 6, 0).add64(2, 1).stx(8, 6, 0, "r2")
    a.mov64(7, "r2").alu64("mod", 2, every).jmp("jne", 2, 0, "out")
    a.stx(8, 10, -8, "r7")
    a.ld_map_fd(1, rb_fd).mov64(2, "r10").add64(2, -8).mov64(3, 8).mov64(4, 0)
    a.call(isa.BPF_FUNC_ringbuf_output)
    a.label("out").mov64(0, isa.XDP_PASS).exit()
    return a.assemble()


@pytest.mark.parametrize("n", [63, 64, 6401])
def test_sampler_every_64(fresh_oracle, fresh_runtime, n):
    po, dev = fresh_oracle, fresh_runtime
    (oc, orb), (dc, drb) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 1),
                                      (isa.BPF_MAP_TYPE_RINGBUF, 0, 0, 1 << 16)], po, dev)
    code = prog_sampler(dc.fd, drb.fd)
    slots = gen.xdp_packets(n)
    ovm = po.OracleVM()
    ovm.load(code)
    ov = ovm.run_xdp(slots.copy(), fixed_len=64)
    orecs = orb.ringbuf_fetch()
    assert [struct.unpack("<Q", r)[0] for r in orecs] == [64 * (k + 1) for k in range(n // 64)]
    for flags in (dev.BATCH_SYNC | dev.BATCH_ORDERED, dev.BATCH_SYNC):
        dc.update(b"\0\0\0\0", bytes(8))
        vm = dev.VM()
        vm.load(code)
        d = dev.DeviceBuffer.from_array(slots)
        dv = dev.DeviceBuffer(4 * n)
        assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv, flags=flags) == 0
        np.testing.assert_array_equal(dv.download(np.uint32), ov)
        recs = drb.ringbuf_fetch()
        if flags & dev.BATCH_ORDERED:
            assert recs == orecs
        else:
            assert sorted(recs) == sorted(orecs)
        assert dc.lookup(b"\0\0\0\0") == oc.lookup(b"\0\0\0\0")


def test_unobserved_counters_still_deferred(fresh_runtime):
    """The headline programs keep their per-wave / per-block counter sums:
    nothing they run after an add reads the counter."""
    dev = fresh_runtime
    ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2)
    bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)
    flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, 1024)
    counts = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 1024)
    for code, kind, want in ((programs.xdp_counter(ctl.fd, bss.fd), dev.CTX_XDP, (1, 0)),
                             (programs.flow_hash(flows.fd), dev.CTX_XDP, (2, 0)),
                             (programs.syscall_agg(counts.fd), dev.CTX_SYSCALL, (2, 0))):
        vm = dev.VM()
        vm.load(code)
        assert vm.counter_info(kind) == want


def test_hash_value_add_then_read(fresh_oracle, fresh_runtime):
    """v = lookup(h, key); v->n += 1 (atomic); r0 = v->n -- a map-value
    counter read after its add, ORDERED vs the oracle and parallel
    properties."""
    po, dev = fresh_oracle, fresh_runtime
    (oh,), (dh,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 8, 64)], po, dev)
    for k in range(8):
        oh.update(struct.pack("<I", k), struct.pack("<Q", 100 * k))
        dh.update(struct.pack("<I", k), struct.pack("<Q", 100 * k))
    a = Asm().ldx(1, 6, 1, 0).alu64("and", 6, 7).stx(4, 10, -4, "r6")
    a.ld_map_fd(1, dh.fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.mov64(1, 0).jmp("jeq", 0, 0, "out")
    a.mov64(3, 1).atomic(8, isa.ATOMIC_ADD, 0, 0, 3).ldx(8, 1, 0, 0)
    a.label("out").mov64(0, "r1").exit()
    code = a.assemble()
    n = 4000
    o, d, failed, vm = _run_raw(po, dev, code, n, dev.BATCH_SYNC | dev.BATCH_ORDERED)
    assert failed == 0 and vm.counter_info(dev.CTX_RAW) == (0, 1)
    np.testing.assert_array_equal(d, o)
    for k in range(8):
        key = struct.pack("<I", k)
        assert dh.lookup(key) == oh.lookup(key)
