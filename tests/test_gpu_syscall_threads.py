"""Thread-ordered syscall dispatch on the device (include/bpftime_amd.h
"Order"; csrc/syscall_dispatch.cpp, interp.hip k_sys_seq, group.hip) against
the oracle's record-by-record dispatch_syscall
(attach/syscall_trace_attach_impl/src/syscall_trace_attach_impl.cpp:18-95;
oracle/drivers.c orc_sys_dispatch):

* syscount's sys_enter + sys_exit pair with measure_latency
  (example/tracing/syscount/syscount.bpf.c:33-87): sys_enter stores
  start[tid] = bpf_ktime_get_ns(), sys_exit reads it back -- the recorded
  clocks of 128-B records (bpf_helper.cpp:357-362 replayed) -- at 2^22
  records over 64 threads, with and without filter_pid: every data_t, every
  start entry and every return bit-exact;
* an enter ``start[tid] = args[0]`` / exit ``sum += start[tid]`` pair:
  bit-exact thread-ordered, and shown to diverge under the program-major plan
  (each program once over the batch: the exit reads the thread's LAST enter);
* EBPF_BATCH_ORDERED: programs that share state ACROSS threads, one lane over
  every record in record order = the serial reference run, bit-exact;
* overrides (bpf_override_return at sys_enter, bpf_set_retval at sys_exit)
  and per-syscall attachments in the thread-ordered plan;
* the plan each attachment set gets (commuting sets keep program-major);
* bpf_ktime_get_ns replayed in the program-major plan too (ktime_off), and the
  named errors of bad pid_tgid_off / ktime_off batches;
* two host threads dispatching on the null stream at once (the per-stream
  dispatch lock): both results exact.
"""
import struct
import threading

import numpy as np
import pytest

from bpftime_amd import isa, gen, programs
from bpftime_amd.isa import Asm

from _helpers import make_maps

pytestmark = pytest.mark.gpu

TRACEPOINT = 5  # BPF_PROG_TYPE_TRACEPOINT
HASH, ARRAY = isa.BPF_MAP_TYPE_HASH, isa.BPF_MAP_TYPE_ARRAY


def _attach(dev, o, code, nr, enter):
    dev.syscall_attach(dev.prog_create(code, "p", TRACEPOINT), nr, enter)
    o.attach(code, nr, enter)


def _syscount(po, dev, **opts):
    (ostart, odata, oro), (dstart, ddata, dro) = make_maps(
        [(HASH, 4, 8, 10240), (HASH, 4, 32, 10240), (ARRAY, 4, programs.SYSCOUNT_RODATA, 1)], po, dev)
    ro = programs.syscount_rodata(measure_latency=True, **opts)
    assert oro.update(b"\0" * 4, ro) == 0 and dro.update(b"\0" * 4, ro) == 0
    o = po.OracleSyscallDispatch()
    _attach(dev, o, programs.syscount_enter(dstart.fd, dro.fd), -1, True)
    _attach(dev, o, programs.syscount_exit(ddata.fd, dro.fd, dstart.fd), -1, False)
    return o, (ostart, odata), (dstart, ddata)


@pytest.mark.parametrize("filter_pid", [0, 1003])
def test_syscount_latency_pair_bit_exact(fresh_oracle, fresh_runtime, filter_pid):
    po, dev = fresh_oracle, fresh_runtime
    o, (ostart, odata), (dstart, ddata) = _syscount(po, dev, filter_pid=filter_pid)
    assert dev.syscall_dispatch_plan() == 1  # start[] is written at enter and read at exit
    n = 1 << 22
    recs = gen.syscall_records_timed(n, threads=64)
    w = recs.view(np.int64).reshape(n, 16)
    assert len(np.unique(w[:, 11])) == 64
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, out=out) == 0
    want = o.dispatch(recs)
    assert (out.download(np.int64) == want).all()
    assert ddata.hash_items() == odata.items()
    assert dstart.hash_items() == ostart.items()
    items = odata.items()
    assert len(items) > 50
    total = sum(struct.unpack("<QQ", v[:16])[1] for v in items.values())
    assert total > 0  # the latency path ran
    if filter_pid:
        assert len(ostart.items()) == 4  # tgid 1003: threads 12..15


@pytest.mark.parametrize("tier", ["asm", "cpp"])
def test_syscount_pair_both_tiers(fresh_oracle, fresh_runtime, monkeypatch, tier):
    """The callbacks run in the asm tier when every stack fits the LDS stacks
    (vm_api.cpp seq_dispatch), else -- or with BPFTIME_AMD_SEQ_ASM=0 -- in
    the C++ tier: both bit-exact, over 256 threads."""
    po, dev = fresh_oracle, fresh_runtime
    monkeypatch.setenv("BPFTIME_AMD_SEQ_ASM", "1" if tier == "asm" else "0")
    o, (ostart, odata), (dstart, ddata) = _syscount(po, dev)
    n = 1 << 18
    recs = gen.syscall_records_timed(n, threads=256)
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, out=out) == 0
    assert (out.download(np.int64) == o.dispatch(recs)).all()
    assert ddata.hash_items() == odata.items()
    assert dstart.hash_items() == ostart.items()


def test_big_stack_callbacks_run_in_cpp(fresh_oracle, fresh_runtime):
    """A callback whose stack exceeds the LDS stacks (kLdsStackMax) keeps the
    C++ tier and its private stack: a start[tid] pair keyed through fp-200."""
    po, dev = fresh_oracle, fresh_runtime
    (ostart, osum), (dstart, dsum) = make_maps([(HASH, 4, 8, 1024), (ARRAY, 4, 16, 1)], po, dev)
    enter = (Asm().call(isa.BPF_FUNC_get_current_pid_tgid).stx(4, 10, -200, "r0").ldx(8, 3, 1, 16)
             .stx(8, 10, -192, "r3").ld_map_fd(1, dstart.fd).mov64(2, "r10").add64(2, -200)
             .mov64(3, "r10").add64(3, -192).mov64(4, 0).call(isa.BPF_FUNC_map_update_elem)
             .mov64(0, 0).exit().assemble())
    exit_ = (Asm().call(isa.BPF_FUNC_get_current_pid_tgid).stx(4, 10, -200, "r0").ld_map_fd(1, dstart.fd)
             .mov64(2, "r10").add64(2, -200).call(isa.BPF_FUNC_map_lookup_elem).jmp("jeq", 0, 0, "out")
             .ldx(8, 3, 0, 0).ld_map_value(2, dsum.fd, 0).atomic(8, isa.ATOMIC_ADD, 2, 0, 3)
             .label("out").mov64(0, 0).exit().assemble())
    o = po.OracleSyscallDispatch()
    _attach(dev, o, enter, -1, True)
    _attach(dev, o, exit_, -1, False)
    assert dev.syscall_dispatch_plan() == 1
    n = 1 << 16
    recs = gen.syscall_records_timed(n, threads=128)
    d = dev.DeviceBuffer.from_array(recs)
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED) == 0
    o.dispatch(recs)
    assert dsum.lookup(b"\0" * 4) == osum.lookup(b"\0" * 4)
    assert dstart.hash_items() == ostart.items()


def test_tid_state_pair_threads_vs_programs(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    (ostart, osum), (dstart, dsum) = make_maps([(HASH, 4, 8, 1024), (ARRAY, 4, 16, 1)], po, dev)
    o = po.OracleSyscallDispatch()
    _attach(dev, o, programs.tid_state_enter(dstart.fd), -1, True)
    _attach(dev, o, programs.tid_state_exit(dstart.fd, dsum.fd), -1, False)
    n = 1 << 20
    recs = gen.syscall_records_timed(n, threads=64)
    d = dev.DeviceBuffer.from_array(recs)
    assert dev.syscall_dispatch_plan() == 1
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED) == 0
    o.dispatch(recs)
    want = osum.lookup(b"\0" * 4)
    assert dsum.lookup(b"\0" * 4) == want
    assert dstart.hash_items() == ostart.items()
    # the program-major plan runs every enter before every exit: each exit
    # reads its thread's last enter, not its own call's
    zero = b"\0" * 16
    assert dsum.update(b"\0" * 4, zero) == 0
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED,
                                flags=dev.BATCH_SYNC | dev.DISPATCH_PROGRAMS) == 0
    assert dsum.lookup(b"\0" * 4) != want


def _shared_last(po, dev):
    """Cross-thread state: enter stores last = args[1] in an ARRAY slot, exit
    adds last * (ret | 1) -- order-dependent across threads."""
    (olast,), (dlast,) = make_maps([(ARRAY, 4, 16, 1)], po, dev)
    enter = (Asm().ldx(8, 3, 1, 24).ld_map_value(2, dlast.fd, 0).stx(8, 2, 0, "r3").mov64(0, 0).exit().assemble())
    exit_ = (Asm().ldx(8, 4, 1, 16).alu64("or", 4, 1).ld_map_value(2, dlast.fd, 0).ldx(8, 3, 2, 0)
             .alu64("mul", 3, "r4").atomic(8, isa.ATOMIC_ADD, 2, 8, 3).mov64(0, 0).exit().assemble())
    return (olast, dlast), enter, exit_


def test_ordered_is_the_serial_run(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    (olast, dlast), enter, exit_ = _shared_last(po, dev)
    o = po.OracleSyscallDispatch()
    _attach(dev, o, enter, -1, True)
    _attach(dev, o, exit_, -1, False)
    assert dev.syscall_dispatch_plan(dev.BATCH_ORDERED) == 1
    n = 1 << 14
    recs = gen.syscall_records_timed(n, threads=16)
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, out=out,
                                flags=dev.BATCH_SYNC | dev.BATCH_ORDERED) == 0
    want = o.dispatch(recs)
    assert (out.download(np.int64) == want).all()
    assert dlast.lookup(b"\0" * 4) == olast.lookup(b"\0" * 4)


def test_64b_records_are_one_thread(fresh_oracle, fresh_runtime):
    """64-B records carry no caller: every call is the dispatching thread's,
    so the thread-ordered plan is the serial run (one lane)."""
    po, dev = fresh_oracle, fresh_runtime
    (olast, dlast), enter, _ = _shared_last(po, dev)
    (ocnt,), (dcnt,) = make_maps([(ARRAY, 4, 8, 1)], po, dev)
    reader = (Asm().ld_map_value(2, dlast.fd, 0).ldx(8, 3, 2, 0).ld_map_value(2, dcnt.fd, 0)
              .atomic(8, isa.ATOMIC_ADD, 2, 0, 3).mov64(0, 0).exit().assemble())
    o = po.OracleSyscallDispatch()
    _attach(dev, o, enter, -1, True)
    _attach(dev, o, reader, 1, True)
    assert dev.syscall_dispatch_plan() == 1
    n = 1 << 12
    recs = gen.syscall_records(n)
    recs.view(np.int64).reshape(n, 8)[::3, 1] = 1
    d = dev.DeviceBuffer.from_array(recs)
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD) == 0
    o.dispatch(recs)
    assert dcnt.lookup(b"\0" * 4) == ocnt.lookup(b"\0" * 4)
    assert dlast.lookup(b"\0" * 4) == olast.lookup(b"\0" * 4)


def test_overrides_and_per_syscall_thread_ordered(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    (ostart, osum, ocnt), (dstart, dsum, dcnt) = make_maps(
        [(HASH, 4, 8, 1024), (ARRAY, 4, 16, 1), (ARRAY, 4, 64, 1)], po, dev)
    counter = lambda slot: (Asm().ld_map_value(2, dcnt.fd, 8 * slot).ldx(8, 3, 2, 0).add64(3, 1)
                            .stx(8, 2, 0, "r3").mov64(0, 0).exit().assemble())
    progs = [(programs.inject_enter(3, -1), 1, True),        # sys_enter_write: override
             (programs.tid_state_enter(dstart.fd), -1, True),
             (counter(0), 0, True),
             (programs.tid_state_exit(dstart.fd, dsum.fd), -1, False),
             (programs.exit_clamp(0), -1, False),            # sys_exit: set_retval
             (counter(1), 0, False),                         # sys_exit_read
             (counter(2), -1, False)]
    o = po.OracleSyscallDispatch()
    for code, nr, enter in progs:
        _attach(dev, o, code, nr, enter)
    n = 1 << 20
    recs = gen.syscall_records_timed(n, threads=256)
    w = recs.view(np.int64).reshape(n, 16)
    w[::7, 1] = w[::7, 9] = 1
    w[3::97, 1] = w[3::97, 9] = 700                         # past the callback arrays: globals only
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    assert dev.syscall_dispatch_plan() == 1
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, out=out) == 0
    want = o.dispatch(recs)
    got = out.download(np.int64)
    assert (got == want).all(), np.flatnonzero(got != want)[:10]
    assert dsum.lookup(b"\0" * 4) == osum.lookup(b"\0" * 4)
    assert dcnt.lookup(b"\0" * 4) == ocnt.lookup(b"\0" * 4)
    c = struct.unpack("<8Q", ocnt.lookup(b"\0" * 4))
    assert c[2] < n and c[0] > 0 and c[1] > 0 and (want == -1).sum() > n // 40
    assert (d.download().reshape(n, 128) == recs).all()      # the records were not written


def test_plan_selection(fresh_runtime):
    dev = fresh_runtime
    start, data, ro, cnt = (dev.Map(HASH, 4, 8, 1024), dev.Map(HASH, 4, 32, 1024),
                            dev.Map(ARRAY, 4, programs.SYSCOUNT_RODATA, 1), dev.Map(ARRAY, 4, 64, 1))
    ids = []
    att = lambda code, nr, enter: ids.append(dev.syscall_attach(dev.prog_create(code, "p", TRACEPOINT), nr, enter))
    att(programs.syscount_exit(data.fd, ro.fd), -1, False)
    assert dev.syscall_dispatch_plan() == 0            # one program
    att((Asm().ld_map_value(2, cnt.fd, 0).ldx(8, 3, 2, 0).add64(3, 1).stx(8, 2, 0, "r3")
         .mov64(0, 0).exit().assemble()), -1, True)
    assert dev.syscall_dispatch_plan() == 0            # counter adds beside a disjoint map
    att(programs.syscall_agg(data.fd), 1, True)
    assert dev.syscall_dispatch_plan() == 1            # syscall_agg writes data, syscount_exit writes data
    dev.syscall_detach(ids.pop())
    assert dev.syscall_dispatch_plan() == 0
    att(programs.syscount_enter(start.fd, ro.fd), -1, True)
    assert dev.syscall_dispatch_plan() == 0            # syscount_exit without the latency path never reads start
    att(programs.syscount_exit(data.fd, ro.fd, start.fd), -1, False)
    assert dev.syscall_dispatch_plan() == 1            # ... with it, it does
    assert dev.syscall_dispatch_plan(dev.DISPATCH_PROGRAMS) == 0
    assert dev.syscall_dispatch_plan(dev.BATCH_ORDERED | dev.DISPATCH_PROGRAMS) == 1
    for i in ids:
        dev.syscall_detach(i)
    att(programs.syscount_exit(data.fd, ro.fd), -1, False)
    assert dev.syscall_dispatch_plan(dev.DISPATCH_THREADS) == 1


def _ktime_sum(fd, slot):
    return (Asm().call(isa.BPF_FUNC_ktime_get_ns).ld_map_value(2, fd, 8 * slot)
            .atomic(8, isa.ATOMIC_ADD, 2, 0, 0).mov64(0, 0).exit().assemble())


@pytest.mark.parametrize("plan", ["programs", "threads"])
def test_ktime_replay(fresh_oracle, fresh_runtime, plan):
    """bpf_ktime_get_ns inside a 128-B record's callbacks returns the recorded
    clock: its enter value at sys_enter, its exit value at sys_exit."""
    po, dev = fresh_oracle, fresh_runtime
    (osum,), (dsum,) = make_maps([(ARRAY, 4, 16, 1)], po, dev)
    o = po.OracleSyscallDispatch()
    _attach(dev, o, _ktime_sum(dsum.fd, 0), -1, True)
    _attach(dev, o, _ktime_sum(dsum.fd, 1), 0, False)
    n = 1 << 18
    recs = gen.syscall_records_timed(n)
    d = dev.DeviceBuffer.from_array(recs)
    flags = dev.BATCH_SYNC | (dev.DISPATCH_PROGRAMS if plan == "programs" else dev.DISPATCH_THREADS)
    assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, flags=flags) == 0
    o.dispatch(recs)
    got = dsum.lookup(b"\0" * 4)
    assert got == osum.lookup(b"\0" * 4)
    w = recs.view(np.uint64).reshape(n, 16)
    live = ~np.isin(w[:, 1], [60, 231])
    s0, s1 = struct.unpack("<QQ", got)
    assert s0 == int(w[live, 12].sum(dtype=np.uint64))
    assert s1 == int(w[live & (w[:, 1] == 0), 13].sum(dtype=np.uint64))


def test_replay_offsets_are_checked(fresh_runtime):
    """pid_tgid_off / ktime_off: syscall kinds only, 8-aligned, the u64 inside
    the unit -- else the batch fails, named, before a launch."""
    dev = fresh_runtime
    vm = dev.VM()
    vm.load(_ktime_sum(dev.Map(ARRAY, 4, 16, 1).fd, 0))
    d = dev.DeviceBuffer(128 * 64)
    for kind, stride, kw in [(dev.CTX_RAW, 128, {"pid_tgid_off": 88}),
                             (dev.CTX_SYSCALL, 128, {"ktime_off": 124}),
                             (dev.CTX_SYSCALL, 96, {"ktime_off": 96}),
                             (dev.CTX_SYSCALL, 128, {"ktime_off": -8}),
                             (dev.CTX_SYSCALL, 128, {"pid_tgid_off": 84}),
                             (dev.CTX_SYSCALL_EXIT, 96, {"ktime_off": 40}),
                             (dev.CTX_SYSCALL_EXIT, 128, {"ktime_off": 64})]:
        with pytest.raises(dev.EbpfError, match="_off"):
            vm.exec_batch(kind, d, 8, stride, fixed_len=64, **kw)
    assert vm.exec_batch(dev.CTX_SYSCALL, d, 8, 128, ktime_off=96, pid_tgid_off=88) == 0
    assert vm.exec_batch(dev.CTX_SYSCALL_EXIT, d, 8, 128, data_offset=64, ktime_off=40, pid_tgid_off=24) == 0


def test_concurrent_dispatches_one_stream(fresh_oracle, fresh_runtime):
    """Two host threads dispatching on the null stream at once: the dispatch
    holds the stream's scratch until it has queued its last launch, so each
    record set gets its own override state."""
    po, dev = fresh_oracle, fresh_runtime
    o = po.OracleSyscallDispatch()
    _attach(dev, o, programs.inject_enter(3, -1), 1, True)
    _attach(dev, o, programs.exit_clamp(0), -1, False)
    sets = []
    for k, n in enumerate((1 << 18, 1 << 19)):
        recs = gen.syscall_records_full(n, seed=gen.SEED_CFG5 + k)
        w = recs.view(np.int64).reshape(n, 12)
        w[k::5, 1] = w[k::5, 9] = 1                        # (the exit half names the same call)
        sets.append((recs, dev.DeviceBuffer.from_array(recs), dev.DeviceBuffer(8 * n)))
    errs = []

    def run(i):
        try:
            recs, d, out = sets[i]
            for _ in range(4):
                dev.syscall_dispatch(d, len(recs), out=out)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    for recs, d, out in sets:
        assert (out.download(np.int64) == o.dispatch(recs)).all()


# ---- struct-of-arrays records (include/bpftime_amd.h struct bpftime_amd_sys_records) ----

def _soa_bufs(dev, recs, with_enter=True):
    enter, exit_, clock = gen.syscall_records_soa(recs)
    return (dev.DeviceBuffer.from_array(exit_), dev.DeviceBuffer.from_array(enter) if with_enter else None,
            dev.DeviceBuffer.from_array(clock) if clock is not None else None)


def test_soa_syscount_exit_only(fresh_oracle, fresh_runtime):
    """syscount's sys_exit program over 32-B exit records (no enter array):
    every data_t and every return as the oracle's run over the 96-B records;
    the device generator writes the same arrays."""
    po, dev = fresh_oracle, fresh_runtime
    (odata, oro), (ddata, dro) = make_maps([(HASH, 4, 32, 8192), (ARRAY, 4, programs.SYSCOUNT_RODATA, 1)], po, dev)
    ro = programs.syscount_rodata(filter_failed=True)
    assert oro.update(b"\0" * 4, ro) == 0 and dro.update(b"\0" * 4, ro) == 0
    o = po.OracleSyscallDispatch()
    _attach(dev, o, programs.syscount_exit(ddata.fd, dro.fd), -1, False)
    n = 1 << 21
    recs = gen.syscall_records_full(n)
    x, _, _ = _soa_bufs(dev, recs, with_enter=False)
    out = dev.DeviceBuffer(8 * n)
    assert dev.syscall_dispatch_soa(x, n, out=out) == 0
    want = o.dispatch(recs)
    assert (out.download(np.int64) == want).all()
    assert ddata.hash_items() == odata.items()
    # the device generator: the same calls, both layouts
    from bpftime_amd import _lib
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(335, 1.2))
    e2, x2 = dev.DeviceBuffer(64 * n), dev.DeviceBuffer(32 * n)
    assert _lib.lib().bpftime_amd_gen_syscall_soa(e2.ptr, x2.ptr, n, gen.SEED_CFG5, 0, cdf.ptr, 335, None) == 0
    enter, exit_, _ = gen.syscall_records_soa(recs)
    assert (x2.download().reshape(n, 32) == exit_).all() and (e2.download().reshape(n, 64) == enter).all()
    # an enter program needs the enter array
    _attach(dev, o, programs.inject_enter(3), 1, True)
    with pytest.raises(dev.EbpfError, match="enter ctxs"):
        dev.syscall_dispatch_soa(x, n)


@pytest.mark.parametrize("plan", ["programs", "threads"])
def test_soa_matches_aos(fresh_oracle, fresh_runtime, plan):
    """Enter and exit programs reading the recorded caller and clock, with
    overrides, over SoA records: the oracle's results over the 128-B
    records, in both plans (pid / clock through the arrays in the enter
    batches, at an offset of the 32-B exit record in the exit batches)."""
    po, dev = fresh_oracle, fresh_runtime
    (ocnt,), (dcnt,) = make_maps([(ARRAY, 4, 64, 1)], po, dev)
    pid_sum = lambda slot: (Asm().call(isa.BPF_FUNC_get_current_pid_tgid).ld_map_value(2, dcnt.fd, 8 * slot)
                            .atomic(8, isa.ATOMIC_ADD, 2, 0, 0).mov64(0, 0).exit().assemble())
    o = po.OracleSyscallDispatch()
    for code, nr, enter in [(programs.inject_enter(3, -1), 1, True), (pid_sum(0), -1, True),
                            (_ktime_sum(dcnt.fd, 1), 0, True), (pid_sum(2), -1, False),
                            (_ktime_sum(dcnt.fd, 3), -1, False), (programs.exit_clamp(0), -1, False)]:
        _attach(dev, o, code, nr, enter)
    n = 1 << 19
    recs = gen.syscall_records_timed(n, threads=512)
    w = recs.view(np.int64).reshape(n, 16)
    w[::7, 1] = w[::7, 9] = 1
    x, e, c = _soa_bufs(dev, recs)
    out = dev.DeviceBuffer(8 * n)
    flags = dev.BATCH_SYNC | (dev.DISPATCH_PROGRAMS if plan == "programs" else dev.DISPATCH_THREADS)
    assert dev.syscall_dispatch_soa(x, n, enter=e, clock=c, out=out, flags=flags) == 0
    want = o.dispatch(recs)
    assert (out.download(np.int64) == want).all()
    assert dcnt.lookup(b"\0" * 4) == ocnt.lookup(b"\0" * 4)
    assert all(struct.unpack("<8Q", ocnt.lookup(b"\0" * 4))[:4])
