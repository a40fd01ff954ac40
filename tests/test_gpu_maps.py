"""Device maps: the reference map unit-test assertions against the device
registry (syscall-side API), and the hash / per-CPU configs of BASELINE.json
(flow-hash = configs[2], syscall-agg = configs[4]) against the oracle."""
import errno
import random
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs
from bpftime_amd.isa import (Asm, ATOMIC_ADD, BPF_FUNC_map_lookup_elem, BPF_FUNC_map_update_elem,
                             BPF_NOEXIST)

from _helpers import make_maps

pytestmark = pytest.mark.gpu

I32 = lambda v: struct.pack("<i", v)  # noqa: E731
I64 = lambda v: struct.pack("<q", v)  # noqa: E731


def test_device_hash_map_kat(fresh_runtime):
    dev = fresh_runtime
    m = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 8, 10)
    assert m.geometry()[0] == 11  # next_prime(10) buckets
    assert m.update(I32(1234), I64(5678)) == 0 and m.update(I32(4321), I64(8765)) == 0
    assert m.lookup(I32(1234)) == I64(5678) and m.lookup(I32(4321)) == I64(8765)
    assert m.lookup(I32(9999)) is None
    assert m.update(I32(1234), I64(1)) == 0 and m.lookup(I32(1234)) == I64(1)
    assert m.count() == 2
    assert m.delete(I32(1234)) == 0 and m.lookup(I32(1234)) is None and m.count() == 1
    for i in range(10):
        m.update(I32(100 + i), I64(i))
    assert m.count() == 10
    assert m.update(I32(999), I64(1)) == 0 and m.lookup(I32(999)) is None  # full, returns 0


def test_device_array_map_kat(fresh_runtime):
    dev = fresh_runtime
    m = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 2)
    assert m.update(I32(1), I64(1234), isa.BPF_ANY) == 0
    assert m.update(I32(1), I64(0), isa.BPF_NOEXIST) < 0
    assert m.lookup(I32(1)) == I64(1234) and m.lookup(I32(0)) == I64(0)
    assert m.update(I32(2), I64(0), isa.BPF_EXIST) < 0 and m.lookup(I32(2)) is None
    assert m.next_key(None) == I32(0) and m.next_key(I32(0)) == I32(1) and m.next_key(I32(1)) is None
    assert m.delete(I32(1)) < 0


def test_hash_next_key_matches_oracle_layout(fresh_oracle, fresh_runtime):
    """Same hash (h*31+b) and linear probing as bpftime_hash_map: inserting
    the same keys in the same order gives the same bucket order."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 4, 97)], po, dev)
    keys = random.Random(5).sample(range(1 << 31), 60)
    for k in keys:
        om.update(I32(k), I32(k + 1))
        dm.update(I32(k), I32(k + 1))
    walk_o, k = [], om.next_key(None)
    while k is not None:
        walk_o.append(k)
        k = om.next_key(k)
    walk_d, k = [], dm.next_key(None)
    while k is not None:
        walk_d.append(k)
        k = dm.next_key(k)
    assert walk_d == walk_o


def _duplicate_keys(m):
    nb, ss, ko, vo, nc = m.geometry()
    raw = m.snapshot().reshape(nb, ss)
    filled = raw[raw[:, :4].view(np.uint32)[:, 0] == 1]
    keys = [bytes(r[ko:ko + m.key_size]) for r in filled]
    return len(keys) - len(set(keys))


def _flow_setup(po, dev, nflows_max=65536):
    return make_maps([(isa.BPF_MAP_TYPE_HASH, 16, 16, nflows_max)], po, dev)


# (1 << 21, 65536): config 3's own shape -- Zipf(1.1) keys over 65,536 flows
# into the 65,537-bucket table, most flows present, at 2^21 frames
@pytest.mark.parametrize("n,nflows", [(4096, 300), (50000, 4000), (1 << 21, 65536)])
def test_flow_hash_parity(fresh_oracle, fresh_runtime, n, nflows):
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = _flow_setup(po, dev)
    code = programs.flow_hash(dm.fd)
    slots, lens = gen.flow_packets(n, nflows=nflows, stride=2048)
    ovm = po.OracleVM()
    ovm.load(code)
    ov = ovm.run_xdp(slots.copy(), lens=lens)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=dl, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    # map contents as key -> value sets (bucket order may differ under races)
    o_items = om.items()
    d_items = dm.hash_items()
    assert d_items == o_items
    # size-independent property: totals = exact histogram of the input
    if nflows == 65536:
        assert len(d_items) > 50000
    tot_pkts = sum(struct.unpack("<QQ", v)[0] for v in d_items.values())
    tot_bytes = sum(struct.unpack("<QQ", v)[1] for v in d_items.values())
    ip = (slots[:, 12] == 0x08) & (slots[:, 13] == 0)
    assert tot_pkts == int(ip.sum()) and tot_bytes == int(lens[ip].sum())


def test_syscall_agg_parity(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192)], po, dev)
    code = programs.syscall_agg(dm.fd)
    n = 60000
    recs = gen.syscall_records(n)
    ovm = po.OracleVM()
    ovm.load(code)
    orets, ran = ovm.run_syscall(recs)
    vm = dev.VM()
    vm.load(code)
    assert vm.info()["fused_rmw"] == 2
    d = dev.DeviceBuffer.from_array(recs)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_SYSCALL, d, n, 64, rets=dr) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), orets)
    assert _duplicate_keys(dm) == 0
    assert dm.hash_items() == om.items()
    ids = recs.view(np.uint64).reshape(n, 8)[:, 1]
    live = (ids != 60) & (ids != 231)
    counts = {struct.unpack("<I", k)[0]: struct.unpack("<QQ", v[:16]) for k, v in dm.hash_items().items()}
    assert sum(c for c, _ in counts.values()) == int(live.sum())
    assert 60 not in counts and 231 not in counts


def test_percpu_array_counter(fresh_oracle, fresh_runtime):
    """bpf_get_smp_processor_id + PERCPU_ARRAY: virtual CPU of unit i is
    (i // 64) % ncpu on both sides."""
    po, dev = fresh_oracle, fresh_runtime
    ncpu = 8
    po.set_ncpu(ncpu)
    dev.set_ncpu(ncpu)
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 4)], po, dev)
    a = Asm()
    a.ldx(8, 6, 1, 0)                      # r6 = unit word
    a.alu64("and", 6, 3).stx(4, 10, -4, "r6")
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).call(1)
    a.jmp("jeq", 0, 0, "out")
    a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, "r1")
    a.call(isa.BPF_FUNC_get_smp_processor_id)
    a.label("out").exit()
    code = a.assemble()
    n = 5000
    units = gen.sm64(8, np.arange(n, dtype=np.uint64)).view(np.uint8).reshape(n, 8)
    ovm = po.OracleVM()
    ovm.load(code)
    o = np.zeros(n, dtype=np.uint64)
    for w0 in range(0, n, 64):
        po.set_cpu((w0 // 64) % ncpu)
        o[w0:w0 + 64] = ovm.run_raw(units[w0:w0 + 64].copy(), 8)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), o)
    for k in range(4):
        assert dm.lookup(I32(k)) == om.lookup(I32(k)), k


def test_percpu_hash_update_lookup(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    ncpu = 4
    po.set_ncpu(ncpu)
    dev.set_ncpu(ncpu)
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_PERCPU_HASH, 4, 8, 1024)], po, dev)
    # each unit writes value = unit word into key (word & 15) on its cpu slot
    # (last writer wins: run ORDERED for the reference's sequential result)
    a = Asm()
    a.ldx(8, 6, 1, 0).mov64(7, "r6").alu64("and", 7, 15).stx(4, 10, -4, "r7")
    a.stx(8, 10, -16, "r6")
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -16).mov64(4, 0).call(2)
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).call(1)
    a.jmp("jeq", 0, 0, "out").ldx(8, 0, 0, 0).label("out").exit()
    code = a.assemble()
    n = 64 * ncpu
    units = np.zeros((n, 8), dtype=np.uint8)
    units.view(np.uint64)[:, 0] = np.arange(n, dtype=np.uint64) * 7 + 3
    ovm = po.OracleVM()
    ovm.load(code)
    o = np.zeros(n, dtype=np.uint64)
    for w0 in range(0, n, 64):
        po.set_cpu((w0 // 64) % ncpu)
        o[w0:w0 + 64] = ovm.run_raw(units[w0:w0 + 64].copy(), 8)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), o)
    assert {k: v for k, v in dm.hash_items().items()} == om.items()


# ---- hash lookup index (common.hpp ix_pos): same results as the reference
# probe, including keys orphaned by deletions (bpftime_hash_map.hpp:182-199)

def _ref_hash(key: bytes) -> int:
    h = 0
    for b in key:
        h = (h * 31 + b) & ((1 << 64) - 1)
    return h


def _lookup_prog(fd):
    """r0 = *(u64 *)lookup(map, *(u32 *)unit) or 0xdead on a miss (raw ctx)."""
    a = Asm().ldx(4, 2, 1, 0).stx(4, 10, -4, "r2").mov64(2, "r10").add64(2, -4).ld_map_fd(1, fd).call(1)
    a.jmp("jeq", 0, 0, "miss").ldx(8, 0, 0, 0).exit()
    return a.label("miss").mov64(0, 0xDEAD).exit().assemble()


def _delete_prog(fd):
    a = Asm().ldx(4, 2, 1, 0).stx(4, 10, -4, "r2").mov64(2, "r10").add64(2, -4).ld_map_fd(1, fd).call(3)
    return a.mov64(0, 0).exit().assemble()


def _run_raw_both(po, dev, code, keys):
    units = np.zeros((len(keys), 16), np.uint8)
    units[:, :4] = np.array(keys, np.uint32).view(np.uint8).reshape(-1, 4)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_raw(units.copy(), 16)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * len(keys))
    assert vm.exec_batch(dev.CTX_RAW, d, len(keys), 16, fixed_len=16, rets=dr) == 0
    return dr.download(np.uint64), want


def test_hash_index_orphaned_keys(fresh_oracle, fresh_runtime):
    """Host deletes orphan a colliding key: the device (index rebuilt at the
    next launch) must miss it exactly like the reference probe."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 8, 10)], po, dev)
    nb = dm.geometry()[0]
    by_home = {}
    for k in range(1, 5000):
        by_home.setdefault(_ref_hash(I32(k)) % nb, []).append(k)
    a, b, c = next(v for v in by_home.values() if len(v) >= 3)[:3]
    other = [k for v in by_home.values() for k in v if k not in (a, b, c)][:4]
    for m in (om, dm):
        for k in (a, b, c, *other):
            m.update(I32(k), I64(k * 10))
    probe = [a, b, c, *other, 777777] * 40
    got, want = _run_raw_both(po, dev, _lookup_prog(dm.fd), probe)
    np.testing.assert_array_equal(got, want)
    for m in (om, dm):
        m.delete(I32(a))          # b and c are now unreachable
    got, want = _run_raw_both(po, dev, _lookup_prog(dm.fd), probe)
    np.testing.assert_array_equal(got, want)
    assert (got[1::len(probe) // 40] == 0xDEAD).all()
    for m in (om, dm):
        m.update(I32(c), I64(5))  # re-inserted at a's bucket, shadows the orphan
    got, want = _run_raw_both(po, dev, _lookup_prog(dm.fd), probe)
    np.testing.assert_array_equal(got, want)
    # the table now holds c twice (the orphan and the shadowing copy), so
    # compare what lookups see, as the oracle's items() does
    o_items = om.items()
    assert {k: dm.lookup(k) for k in o_items} == o_items


def test_hash_index_device_deletes(fresh_oracle, fresh_runtime):
    """A program that deletes invalidates the index; lookups afterwards
    (index rebuilt from the table) agree with the oracle."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 8, 64)], po, dev)
    keys = list(range(1000, 1060))
    for m in (om, dm):
        for k in keys:
            m.update(I32(k), I64(k))
    got, want = _run_raw_both(po, dev, _delete_prog(dm.fd), keys[::3])
    np.testing.assert_array_equal(got, want)
    got, want = _run_raw_both(po, dev, _lookup_prog(dm.fd), keys * 8)
    np.testing.assert_array_equal(got, want)
    o_items = om.items()  # keys orphaned by the deletes map to None
    assert {k: dm.lookup(k) for k in o_items} == o_items


@pytest.mark.parametrize("index", [True, False])
def test_flow_hash_full_table(fresh_oracle, fresh_runtime, monkeypatch, index):
    """A nearly full table (config 3's shape at small size): two
    passes, the second all hits through the lookup index, equal to the
    oracle with and without the index."""
    if not index:
        monkeypatch.setenv("BPFTIME_AMD_NO_HASH_INDEX", "1")
    po, dev = fresh_oracle, fresh_runtime
    nflows = 1024
    (om,), (dm,) = _flow_setup(po, dev, nflows_max=nflows)
    code = programs.flow_hash(dm.fd)
    n = 40000
    slots, lens = gen.flow_packets(n, nflows=nflows, stride=2048)
    ovm = po.OracleVM()
    ovm.load(code)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    for _ in range(2):
        ov = ovm.run_xdp(slots.copy(), lens=lens)
        assert vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=dl, verdicts=dv) == 0
        np.testing.assert_array_equal(dv.download(np.uint32), ov)
    assert _duplicate_keys(dm) == 0
    assert dm.hash_items() == om.items()
    assert dm.count() == len(om.items())


def test_lookup_cache_against_concurrent_deleter(fresh_runtime):
    """A launch whose hash lookups use the block's LDS lookup cache trusts a
    found slot for the rest of the launch.  A deleting program launched on
    another stream, or a host delete, therefore waits for it (and a cached
    launch waits for a deleter): the results are those of the serial order
    of the calls.  Reader: r0 = the value or 0xdead; deleter:
    deletes the unit's key; 4-byte keys (the cache holds them as tags)."""
    dev = fresh_runtime
    L = dev.lib()
    m = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 8, 4096)
    for k in range(2000):
        m.update(struct.pack("<I", k), struct.pack("<Q", 1000 + k))
    rd = Asm().ldx(4, 2, 1, 0).stx(4, 10, -4, "r2")
    rd.ld_map_fd(1, m.fd).mov64(2, "r10").add64(2, -4).call(1)
    rd.jmp("jeq", 0, 0, "miss").ldx(8, 0, 0, 0).exit().label("miss").mov64(0, 0xdead).exit()
    de = Asm().ldx(4, 2, 1, 0).stx(4, 10, -4, "r2")
    de.ld_map_fd(1, m.fd).mov64(2, "r10").add64(2, -4).call(3).mov64(0, 0).exit()
    reader, deleter = dev.VM(), dev.VM()
    reader.load(rd.assemble())
    deleter.load(de.assemble())
    n = 1 << 18
    keys = (np.arange(n, dtype=np.uint64) % 2000).astype(np.uint32)
    units = np.zeros((n, 8), np.uint8)
    units.view(np.uint32)[:, 0] = keys
    evens = units[keys % 2 == 0]
    d = dev.DeviceBuffer.from_array(units)
    de_d = dev.DeviceBuffer.from_array(evens)
    r1, r2 = dev.DeviceBuffer(8 * n), dev.DeviceBuffer(8 * n)
    s1, s2 = L.bpftime_amd_stream_create(), L.bpftime_amd_stream_create()
    try:
        reader.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=r1, flags=0, stream=s1)
        deleter.exec_batch(dev.CTX_RAW, de_d, len(evens), 8, fixed_len=8, flags=0, stream=s2)
        reader.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=r2, flags=0, stream=s1)
        m.delete(struct.pack("<I", 1))                 # a host delete behind the cached launch
        L.bpftime_amd_sync()
    finally:
        L.bpftime_amd_stream_destroy(s1)
        L.bpftime_amd_stream_destroy(s2)
    vals = 1000 + keys.astype(np.uint64)
    np.testing.assert_array_equal(r1.download(np.uint64), vals)
    np.testing.assert_array_equal(r2.download(np.uint64), np.where(keys % 2 == 0, 0xdead, vals))
    assert m.lookup(struct.pack("<I", 1)) is None and m.lookup(struct.pack("<I", 3)) is not None


def _u32_counter_prog(fd):
    """Per-key u32 counters through a hash value {u32 hits, u32 bytes}:
    key = the frame's first byte, lookup_or_try_init, two 4-byte atomic adds
    (deferred: nothing reads them back in the unit)."""
    a = Asm()
    a.ldx(8, 2, 1, 0).ldx(8, 3, 1, 8)
    a.mov64(6, "r3").alu64("sub", 6, "r2")
    a.ldx(1, 4, 2, 0).stx(4, 10, -4, "r4")
    a.st(8, 10, -16, 0)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(BPF_FUNC_map_lookup_elem)
    a.jmp("jne", 0, 0, "have")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -16).mov64(4, BPF_NOEXIST)
    a.call(BPF_FUNC_map_update_elem)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(BPF_FUNC_map_lookup_elem)
    a.mov64(1, "r0").mov64(0, 0).jmp("jeq", 1, 0, "out").mov64(0, "r1")
    a.label("have")
    a.mov64(1, 1)
    a.atomic(4, ATOMIC_ADD, 0, 0, "r1")
    a.atomic(4, ATOMIC_ADD, 0, 4, "r6")
    a.mov64(0, 2)
    a.label("out").exit()
    return a.assemble()


# The combining tables' miss log (common.hpp kMissParts, interp.hip
# k_miss_merge; opt-in, BPFTIME_AMD_MISS_LOG=1): the smallest table makes
# most adds miss, a tiny per-partition capacity makes the log overflow into
# direct adds.  cap "0": the log off, misses add directly
@pytest.mark.parametrize("cap", [None, "2", "0"])
def test_miss_log_parity(fresh_oracle, fresh_runtime, monkeypatch, cap):
    po, dev = fresh_oracle, fresh_runtime
    monkeypatch.setenv("BPFTIME_AMD_MISS_LOG", "0" if cap == "0" else "1")
    monkeypatch.setenv("BPFTIME_AMD_COMB_ENTRIES", "256")
    if cap and cap != "0":
        monkeypatch.setenv("BPFTIME_AMD_MISS_CAP", cap)
    # 8-byte pairs: flow-hash at config 3's key shape
    (om,), (dm,) = _flow_setup(po, dev)
    code = programs.flow_hash(dm.fd)
    n = 1 << 20
    slots, lens = gen.flow_packets(n, nflows=65536, stride=2048)
    ovm = po.OracleVM()
    ovm.load(code)
    ov = ovm.run_xdp(slots.copy(), lens=lens)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=dl, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    assert dm.hash_items() == om.items()
    # 4-byte counters, 256 keys
    (om4,), (dm4,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 8, 512)], po, dev)
    code4 = _u32_counter_prog(dm4.fd)
    n4 = 1 << 19
    pk = gen.xdp_packets(n4, seed=77)
    lens4 = (64 + (np.arange(n4) % 7)).astype(np.uint32)
    ov4 = po.OracleVM()
    ov4.load(code4)
    want = ov4.run_xdp(pk.copy(), lens=lens4)
    vm4 = dev.VM()
    vm4.load(code4)
    d4 = dev.DeviceBuffer.from_array(pk)
    dl4 = dev.DeviceBuffer.from_array(lens4)
    dv4 = dev.DeviceBuffer(4 * n4)
    assert vm4.exec_batch(dev.CTX_XDP, d4, n4, 64, lens=dl4, verdicts=dv4) == 0
    np.testing.assert_array_equal(dv4.download(np.uint32), want)
    assert dm4.hash_items() == om4.items()


def _ctx_flow_program(flows_fd):
    """flow_hash with a generic ctx read (ctx->ingress_ifindex: the lanes'
    48-B ctx must sit in LDS), a 64-B stack and the same hash lookup, whose
    pkts counter adds the ifindex: a 1024-lane block of it would not fit
    the CU with a doubled lookup cache."""
    from bpftime_amd.isa import Asm
    body = programs.flow_hash(flows_fd)
    a = Asm()
    a.ldx(4, 9, 1, 20)                    # r9 = ctx->ingress_ifindex
    a.stx(8, 10, -64, "r9")               # the stack reaches fp-64
    pre = a.assemble()
    insns = [body[i:i + 8] for i in range(0, len(body), 8)]
    # the body's `pkts += 1` (mov64 r1, 1 before the first atomic add) adds
    # the ifindex spilled at fp-64 instead
    out = []
    for i, ins in enumerate(insns):
        if ins[0] == 0xb7 and ins[1] & 0xf == 1 and struct.unpack("<i", ins[4:])[0] == 1 and \
                i + 1 < len(insns) and insns[i + 1][0] == 0xdb:
            out.append(bytes([0x79, 0x01 | (10 << 4)]) + struct.pack("<hi", -64, 0))  # r1 = *(u64 *)(fp-64)
        else:
            out.append(ins)
    return pre + b"".join(out)


@pytest.mark.parametrize("nflows", [300, 4000])
def test_ctx_stack_lookup_fits_cu(fresh_oracle, fresh_runtime, nflows):
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = _flow_setup(po, dev)
    code = _ctx_flow_program(dm.fd)
    n = 1 << 17
    slots, lens = gen.flow_packets(n, nflows=nflows, stride=2048)
    ovm = po.OracleVM()
    ovm.load(code)
    ov = ovm.run_xdp(slots.copy(), lens=lens, ifindex=7)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=dl, verdicts=dv, ifindex=7) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    assert dm.hash_items() == om.items()
    tot = sum(struct.unpack("<QQ", v)[0] for v in om.items().values())
    ip = (slots[:, 12] == 0x08) & (slots[:, 13] == 0)
    assert tot == 7 * int(ip.sum())


def _keyed_counter_prog(map_fd, ksz):
    """The flow-hash idiom over a key of ksz bytes copied from the packet's
    first bytes: lookup, else insert zero (BPF_NOEXIST) and look up again,
    then add 1 to the value."""
    a = Asm()
    a.mov64(6, "r1")
    a.ldx(8, 2, 6, 0).ldx(8, 3, 6, 8)
    a.mov64(4, "r2").add64(4, 32).mov64(0, isa.XDP_DROP).jmp("jgt", 4, "r3", "out")
    for i in range(ksz // 4):
        a.ldx(4, 5, 2, 4 * i).stx(4, 10, -32 + 4 * i, "r5")
    a.st(8, 10, -48, 0)
    a.ld_map_fd(1, map_fd).mov64(2, "r10").add64(2, -32).call(BPF_FUNC_map_lookup_elem)
    a.jmp("jne", 0, 0, "have")
    a.ld_map_fd(1, map_fd).mov64(2, "r10").add64(2, -32).mov64(3, "r10").add64(3, -48)
    a.mov64(4, BPF_NOEXIST).call(BPF_FUNC_map_update_elem)
    a.ld_map_fd(1, map_fd).mov64(2, "r10").add64(2, -32).call(BPF_FUNC_map_lookup_elem)
    a.mov64(1, "r0").mov64(0, isa.XDP_ABORTED).jmp("jeq", 1, 0, "out")
    a.mov64(0, "r1")
    a.label("have")
    a.mov64(1, 1).atomic(8, ATOMIC_ADD, 0, 0, "r1")
    a.mov64(0, isa.XDP_PASS)
    a.label("out")
    a.exit()
    return a.assemble()


@pytest.mark.parametrize("ksz", [4, 8, 12, 16, 20])
def test_keyed_index_inserts_and_lookups(fresh_oracle, fresh_runtime, ksz):
    """Hash lookups through the keyed lookup index (common.hpp ix_key_stride:
    keys of at most 16 B compare in the index, longer ones in the bucket)
    while the same launch inserts: 300 keys that share all but their last
    dword, the all-zero key among them (a key line an XCD's L2 holds from
    before the insert reads zero: gen_fast.py index_probe confirms zero-key
    hits in the bucket), a Zipf-like mix over 2^18 frames, one cold launch
    then a warm one, against the oracle's counts."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, ksz, 8, 512)], po, dev)
    code = _keyed_counter_prog(dm.fd, ksz)
    rng = np.random.default_rng(ksz)
    keys = np.zeros((300, 32), np.uint8)
    keys[1:, :ksz] = rng.integers(0, 256, ksz, dtype=np.uint8)   # a shared prefix
    keys[1:, ksz - 4:ksz] = rng.integers(0, 256, (299, 4), dtype=np.uint8)
    n = 1 << 18
    pick = np.minimum((rng.pareto(1.2, n) * 10).astype(np.int64), 299)
    pk = np.zeros((n, 64), np.uint8)
    pk[:, :32] = keys[pick]
    ovm = po.OracleVM()
    ovm.load(code)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    for _ in range(2):
        want = ovm.run_xdp(pk.copy(), fixed_len=64)
        assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
        np.testing.assert_array_equal(dv.download(np.uint32), want)
        assert dm.hash_items() == om.items()
    assert len(om.items()) == len(set(pick.tolist())) and (pick == 0).sum() > 1000


@pytest.mark.parametrize("present", [1.0, 0.5])
def test_hash_update_existing_keys_in_asm(fresh_oracle, fresh_runtime, present):
    """bpf_map_update_elem of a HASH map with key and value on the stack
    (gen_fast.py call_update_stk): a wave whose lanes all find their key
    overwrites the values in asm; new keys, and a lane whose lookup of the
    key just missed (the lookup-or-init race rule), take the C++ helper.
    Each unit updates its own key (unit index % keys) with 16 bytes of its
    data, then looks the key up, reads the value back and returns it: every
    map value and every return bit-exact against the oracle.  present: the
    fraction of keys inserted by the host first."""
    po, dev = fresh_oracle, fresh_runtime
    n = 4096
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 16, 2 * n)], po, dev)
    for k in range(int(n * present)):
        key, val = struct.pack("<I", k), struct.pack("<QQ", 7 * k, k)
        assert om.update(key, val) == 0 and dm.update(key, val) == 0
    a = Asm()
    a.ldx(4, 2, 1, 0).stx(4, 10, -4, "r2")                 # key = unit word 0
    a.ldx(8, 3, 1, 8).stx(8, 10, -24, "r3")                # value = unit bytes 8..23
    a.ldx(8, 3, 1, 16).stx(8, 10, -16, "r3")
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -24).mov64(4, 0)
    a.call(isa.BPF_FUNC_map_update_elem)
    a.mov64(6, "r0")
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "miss")
    a.ldx(8, 0, 0, 8).alu64("add", 0, "r6").exit()
    a.label("miss").mov64(0, 99).exit()
    code = a.assemble()
    units = np.zeros((n, 32), dtype=np.uint8)
    w = units.view(np.uint32)
    w[:, 0] = np.arange(n, dtype=np.uint32)
    units.view(np.uint64)[:, 1] = gen.sm64(11, np.arange(n, dtype=np.uint64))
    units.view(np.uint64)[:, 2] = gen.sm64(12, np.arange(n, dtype=np.uint64))
    ovm = po.OracleVM()
    ovm.load(code)
    orets = ovm.run_raw(units.copy(), 32)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 32, fixed_len=32, rets=dr, flags=dev.BATCH_SYNC) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), orets)
    assert dm.hash_items() == om.items()
