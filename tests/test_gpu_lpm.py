"""LPM trie on the device: the reference's LPM unit-test assertions against
the device registry (host-side writes, device replica), and an XDP routing
program (longest-prefix match of the IPv4 destination) bit-exact against
the oracle over random routes and packets."""
import socket
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa
from bpftime_amd.isa import Asm

from _helpers import make_maps
from test_oracle_lpm import k4, lpm_kats, LPM

pytestmark = pytest.mark.gpu


def test_device_lpm_kats(fresh_runtime):
    dev = fresh_runtime
    lpm_kats(lambda t, k, v, mx: dev.Map(t, k, v, mx))


@pytest.mark.parametrize("ksize,vsize,mx", [(4, 4, 10), (261, 4, 10), (8, 0, 10), (8, 4, 0)])
def test_device_lpm_constructor_validation(fresh_runtime, ksize, vsize, mx):
    with pytest.raises(Exception):
        fresh_runtime.Map(LPM, ksize, vsize, mx)


def route_prog(fd):
    """XDP: verdict = u32 value of the longest prefix containing the IPv4
    destination (key {32, daddr} on the stack), PASS when no route or not IPv4."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, 2)
    a.mov64(4, "r2").add64(4, 34).jmp("jgt", 4, "r3", "out")
    a.ldx(2, 4, 2, 12).jmp("jne", 4, 0x0008, "out")
    a.st(4, 10, -8, 32).ldx(4, 4, 2, 30).stx(4, 10, -4, "r4")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).call(1)
    a.mov64(1, "r0").mov64(0, 2).jmp("jeq", 1, 0, "out").ldx(4, 0, 1, 0)
    a.label("out").exit()
    return a.assemble()


def test_lpm_routing_program(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(5)
    (om,), (dm,) = make_maps([(LPM, 8, 4, 4096)], po, dev)
    routes = []
    for i in range(3000):
        plen = int(rng.choice([8, 12, 16, 20, 24, 28, 32]))
        net = int(rng.integers(0, 1 << 32)) & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF)
        routes.append((plen, net, int(rng.integers(1, 4))))   # DROP / PASS / TX
    for plen, net, v in routes:
        key = struct.pack("<I", plen) + struct.pack(">I", net)
        for m in (om, dm):
            m.update(key, struct.pack("<I", v))
    assert dm.count() == om.count()
    # delete some routes (logical deletion keeps the trie shape)
    for plen, net, v in routes[::7]:
        key = struct.pack("<I", plen) + struct.pack(">I", net)
        assert dm.delete(key) == om.delete(key)
    n = 1 << 16
    pk = gen.xdp_packets(n, seed=9)
    pk[:, 12:14] = [0x08, 0x00]
    picks = rng.integers(0, len(routes), n)
    dst = np.array([routes[i][1] for i in picks], np.uint64)
    noise = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    host = (np.array([32 - routes[i][0] for i in picks]))
    mask = ((np.uint64(1) << host.astype(np.uint64)) - np.uint64(1))
    addr = np.where(rng.random(n) < 0.8, dst | (noise & mask), noise).astype(np.uint32)
    pk[:, 30:34] = addr.astype(">u4").view(np.uint8).reshape(n, 4)
    pk[::97, 12] = 0x86                                             # some non-IPv4 frames
    code = route_prog(dm.fd)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), fixed_len=64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    got = dv.download(np.uint32)
    np.testing.assert_array_equal(got, want)
    assert len(set(got.tolist())) >= 3
    # host-side change after a batch: the replica follows at the next launch
    for m in (om, dm):
        m.update(k4(0, "0.0.0.0"), struct.pack("<I", 1))               # default route: DROP
    want2 = ovm.run_xdp(pk.copy(), fixed_len=64)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), want2)
    assert not np.array_equal(want, want2)


def route_prog_null_check(fd, taken_on_hit):
    """route_prog with the lookup's result tested directly (`if r0 == 0` /
    `if r0 != 0` right after the call, the LPM lookup running in the fused
    CALL_LOOKUP_STK3 dispatch and the check in the jump handler that
    follows)."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(6, 2)
    a.mov64(4, "r2").add64(4, 34).jmp("jgt", 4, "r3", "out")
    a.ldx(2, 4, 2, 12).jmp("jne", 4, 0x0008, "out")
    a.st(4, 10, -8, 32).ldx(4, 4, 2, 30).stx(4, 10, -4, "r4")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).call(1)
    if taken_on_hit:
        a.jmp("jne", 0, 0, "hit").mov64(6, 4).ja("out")
        a.label("hit").ldx(4, 6, 0, 0)
    else:
        a.jmp("jeq", 0, 0, "out").ldx(4, 6, 0, 0)
    a.label("out").mov64(0, "r6").exit()
    return a.assemble()


@pytest.mark.parametrize("taken_on_hit", [False, True])
@pytest.mark.parametrize("hit_rate", [0.0, 0.8, 1.0])
def test_lpm_lookup_direct_null_check(fresh_oracle, fresh_runtime, taken_on_hit, hit_rate):
    """Waves whose lanes all miss, all hit, or split between the two at the
    null check right after an asm-tier LPM lookup, bit-exact against the
    oracle."""
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(11)
    (om,), (dm,) = make_maps([(LPM, 8, 4, 1024)], po, dev)
    nets = []
    for i in range(500):
        plen = int(rng.choice([16, 20, 24, 32]))
        net = int(rng.integers(1 << 31, 1 << 32)) & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF)
        nets.append((plen, net))
        for m in (om, dm):
            m.update(struct.pack("<I", plen) + struct.pack(">I", net), struct.pack("<I", 1 + i % 3))
    n = 1 << 15
    pk = gen.xdp_packets(n, seed=12)
    pk[:, 12:14] = [0x08, 0x00]
    picks = rng.integers(0, len(nets), n)
    hit = np.array([nets[i][1] for i in picks], np.uint64)
    miss = rng.integers(0, 1 << 31, n, dtype=np.uint64)          # below every route
    addr = np.where(rng.random(n) < hit_rate, hit, miss).astype(np.uint32)
    pk[:, 30:34] = addr.astype(">u4").view(np.uint8).reshape(n, 4)
    code = route_prog_null_check(dm.fd, taken_on_hit)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), fixed_len=64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    got = dv.download(np.uint32)
    np.testing.assert_array_equal(got, want)
    if hit_rate == 0.0:
        assert set(got.tolist()) == {4 if taken_on_hit else 2}
    else:
        assert len(set(got.tolist())) >= 3


def learn_prog(fd):
    """Route learning over 16-B raw units {u32 op, u32 prefixlen, 4 address
    bytes (network order), u32 value}: op & 0xff = 0 lookup (r0 = the value,
    0xffff on a miss), 1 map_update_elem with flags op >> 8 (r0 = 1000 +
    result), 2 map_delete_elem (r0 = 2000 + result)."""
    a = Asm().mov64(6, "r1").ldx(4, 7, 6, 0)
    a.ldx(4, 2, 6, 4).stx(4, 10, -8, "r2").ldx(4, 2, 6, 8).stx(4, 10, -4, "r2")
    a.ldx(4, 2, 6, 12).stx(4, 10, -16, "r2")
    a.mov64(8, "r7").alu64("and", 8, 0xff)
    a.jmp("jeq", 8, 1, "upd").jmp("jeq", 8, 2, "del")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).call(1)
    a.jmp("jeq", 0, 0, "miss").ldx(4, 0, 0, 0).exit()
    a.label("miss").mov64(0, 0xffff).exit()
    a.label("upd").ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).mov64(3, "r10").add64(3, -16)
    a.mov64(4, "r7").alu64("rsh", 4, 8).call(2).add64(0, 1000).exit()
    a.label("del").ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).call(3).add64(0, 2000).exit()
    return a.assemble()


def learn_units(rng, n, nets=400):
    """A stream of lookups, updates (flags ANY / NOEXIST / EXIST, some
    invalid) and deletes over a small pool of prefixes, so keys repeat, get
    deleted and come back, and the trie splits, grows parents and fills."""
    pool = []
    for _ in range(nets):
        plen = int(rng.choice([0, 1, 7, 8, 12, 16, 20, 23, 24, 28, 31, 32]))
        net = int(rng.integers(0, 1 << 32)) & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF)
        pool.append((plen, net))
    u = np.zeros((n, 16), np.uint8)
    w = u.view(np.uint32)
    pick = rng.integers(0, nets, n)
    op = rng.choice([0, 0, 0, 1, 1, 2], n)
    flags = rng.choice([0, 1, 2, 0, 4], n)                        # 4: EINVAL
    w[:, 0] = op | np.where(op == 1, flags, 0) << 8
    w[:, 1] = [pool[i][0] for i in pick]
    addr = np.array([pool[i][1] for i in pick], np.uint64)
    noise = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    look = op == 0
    addr = np.where(look & (rng.random(n) < 0.7), addr | (noise & np.uint64(0xFF)), addr)
    w[:, 1] = np.where(look, 32, w[:, 1])
    w[:, 1] = np.where(rng.random(n) < 0.01, 33, w[:, 1])          # prefixlen > 32: EINVAL
    u[:, 8:12] = addr.astype(np.uint32).astype(">u4").view(np.uint8).reshape(n, 4)
    w[:, 3] = rng.integers(1, 1 << 31, n)
    return u


@pytest.mark.parametrize("mx", [64, 4096])
def test_lpm_program_writes_ordered(fresh_oracle, fresh_runtime, mx):
    """Program-side map_update_elem / map_delete_elem on an LPM trie
    (lpm_trie_map.cpp:266-541) in ORDERED batches, bit-exact against the
    oracle: every unit's r0 (lookups see the writes of the units before
    them; EEXIST / ENOENT / ENOSPC (mx 64 fills) / EINVAL), then the host's
    view of the trie (lookups of every prefix, count, first key), a host
    write after the batch and a parallel routing launch over the result."""
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(11)
    (om,), (dm,) = make_maps([(LPM, 8, 4, mx)], po, dev)
    for plen, net in ((8, 0x0A000000), (16, 0x0A010000)):
        key = struct.pack("<I", plen) + struct.pack(">I", net)
        for m in (om, dm):
            m.update(key, struct.pack("<I", 7))
    code = learn_prog(dm.fd)
    ovm = po.OracleVM()
    ovm.load(code)
    vm = dev.VM()
    vm.load(code)
    seen = set()
    for rnd in range(3):
        n = 3000
        units = learn_units(rng, n)
        want = ovm.run_raw(units.copy(), 16)
        d = dev.DeviceBuffer.from_array(units)
        dr = dev.DeviceBuffer(8 * n)
        assert vm.exec_batch(dev.CTX_RAW, d, n, 16, fixed_len=16, rets=dr,
                             flags=dev.BATCH_SYNC | dev.BATCH_ORDERED) == 0
        got = dr.download(np.uint64)
        np.testing.assert_array_equal(got, want)
        seen |= set(got.tolist())
        assert dm.count() == om.count()
        for row in units[::7]:
            for plen in (32, int(row[4])):
                key = struct.pack("<I", min(plen, 32)) + bytes(row[8:12])
                assert dm.lookup(key) == om.lookup(key), (rnd, key)
        assert dm.next_key(None) == om.next_key(None)
    assert {999, 1000, 1999, 0xffff} <= seen and len(seen) > 50
    # a host write on the trie the batch left, then a parallel launch of a
    # reading program (flat table rebuilt from the pulled trie at 2^16 units)
    for m in (om, dm):
        m.update(k4(0, "0.0.0.0"), struct.pack("<I", 1))
    n = 1 << 16
    pk = gen.xdp_packets(n, seed=12)
    pk[:, 12:14] = [0x08, 0x00]
    pk[: n // 2, 30:34] = units[rng.integers(0, len(units), n // 2), 8:12]
    rcode = route_prog(dm.fd)
    ovm2 = po.OracleVM()
    ovm2.load(rcode)
    want = ovm2.run_xdp(pk.copy(), fixed_len=64)
    vm2 = dev.VM()
    vm2.load(rcode)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm2.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), want)


def test_lpm_program_writes_refused_in_parallel(fresh_runtime):
    """A parallel batch of a program that may write an LPM trie is refused
    with an error naming the helper and the map; ORDERED batches run it,
    and programs that only read the trie run in parallel."""
    dev = fresh_runtime
    dm = dev.Map(LPM, 8, 4, 64)
    vm = dev.VM()
    vm.load(learn_prog(dm.fd))
    units = np.zeros((64, 16), np.uint8)
    d = dev.DeviceBuffer.from_array(units)
    with pytest.raises(dev.EbpfError, match=r"bpf_map_(update|delete)_elem on LPM_TRIE map fd %d" % dm.fd):
        vm.exec_batch(dev.CTX_RAW, d, 64, 16, fixed_len=16)
    assert vm.exec_batch(dev.CTX_RAW, d, 64, 16, fixed_len=16, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED) == 0
    # a program that updates another map and only looks the trie up
    (hm,) = [dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 4, 16)]
    a = Asm().st(4, 10, -8, 32).st(4, 10, -4, 0)
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -8).call(1)
    a.st(4, 10, -12, 1).ld_map_fd(1, hm.fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -12)
    a.mov64(4, 0).call(2).exit()
    vm2 = dev.VM()
    vm2.load(a.assemble())
    assert vm2.exec_batch(dev.CTX_RAW, d, 64, 16, fixed_len=16) == 0


def churn_prog(fd, per_unit=4):
    """RAW units {u32 id}: per_unit times insert the /32 (id * 16 + i), then
    delete it -- the trie's entries stay small while its nodes (logically
    deleted, lpm_trie_map.cpp:490-541) keep growing."""
    a = Asm().ldx(4, 6, 1, 0).alu64("lsh", 6, 4).mov64(7, 0)
    a.label("loop")
    a.st(4, 10, -8, 32).mov64(2, "r6").alu64("add", 2, "r7").stx(4, 10, -4, "r2").st(4, 10, -12, 1)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).mov64(3, "r10").add64(3, -12).mov64(4, 0).call(2)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -8).call(3)
    a.add64(7, 1).jmp("jlt", 7, per_unit, "loop")
    a.mov64(0, 0).exit()
    return a.assemble()


def test_lpm_device_pool_exhausted_fails_the_batch(fresh_oracle, fresh_runtime):
    """An ORDERED batch whose program-side updates outgrow the replica's node
    pool (sized before the launch for two nodes per update site and unit)
    fails with an error naming the trie, where the reference's heap would
    have grown; the host keeps the trie as it was before the batch (ADVICE
    r03).  A batch within the pool gives the oracle's trie."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(LPM, 8, 4, 16)], po, dev)
    for m in (om, dm):
        m.update(k4(8, "10.0.0.0"), struct.pack("<I", 7))
    code = churn_prog(dm.fd, per_unit=1)   # two new nodes per unit at most: the pool holds them
    vm = dev.VM()
    vm.load(code)
    small = np.arange(16, dtype=np.uint32).reshape(16, 1).view(np.uint8)
    d = dev.DeviceBuffer.from_array(np.ascontiguousarray(small))
    assert vm.exec_batch(dev.CTX_RAW, d, 16, 4, fixed_len=4, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED) == 0
    ovm = po.OracleVM()
    ovm.load(code)
    ovm.run_raw(np.ascontiguousarray(small).copy(), 4)
    assert dm.count() == om.count() == 1 and dm.lookup(k4(8, "10.0.0.0")) == struct.pack("<I", 7)
    n = 4096
    big = np.arange(n, dtype=np.uint32).reshape(n, 1).view(np.uint8) + 0   # ids 0..4095: fresh /32s
    d2 = dev.DeviceBuffer.from_array(np.ascontiguousarray(big))
    vm4 = dev.VM()
    vm4.load(churn_prog(dm.fd, per_unit=4))  # four inserts per unit behind one update site
    with pytest.raises(dev.EbpfError, match=r"LPM_TRIE map fd %d: .*node pool" % dm.fd):
        vm4.exec_batch(dev.CTX_RAW, d2, n, 4, fixed_len=4, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED)
    # the report sticks: host ops fail with ENOMEM, and so does
    # any launch of a program naming a trie, until it is acknowledged
    import ctypes as C
    L = dev.lib()
    assert dm.lookup(k4(8, "10.0.0.0")) is None and C.get_errno() == 12
    with pytest.raises(dev.EbpfError, match=r"LPM_TRIE map fd %d: .*node pool" % dm.fd):
        vm.exec_batch(dev.CTX_RAW, d, 16, 4, fixed_len=4, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED)
    assert L.bpftime_amd_map_ack_error(dm.fd) == 1 and L.bpftime_amd_map_ack_error(dm.fd) == 0
    assert dm.count() == 1 and dm.lookup(k4(8, "10.0.0.0")) == struct.pack("<I", 7)
    assert dm.lookup(k4(32, "0.0.1.0")) is None


def test_lpm_writer_and_reader_on_two_streams(fresh_oracle, fresh_runtime):
    """An ORDERED batch writing routes on one stream and a parallel routing
    batch on another, launched back to back without waiting: the reader sees
    every route the writer added (the second launch waits for the device),
    as the serial order writer-then-reader gives."""
    po, dev = fresh_oracle, fresh_runtime
    L = dev.lib()
    (om,), (dm,) = make_maps([(LPM, 8, 4, 4096)], po, dev)
    rng = np.random.default_rng(21)
    n = 2000
    units = np.zeros((n, 16), np.uint8)
    w = units.view(np.uint32)
    plens = rng.choice([8, 16, 24, 32], n)
    nets = rng.integers(0, 1 << 32, n, dtype=np.uint64) & ((np.uint64(0xFFFFFFFF) << (np.uint64(32) - plens.astype(np.uint64))) & np.uint64(0xFFFFFFFF))
    w[:, 0] = 1                                                  # update, flags ANY
    w[:, 1] = plens
    units[:, 8:12] = nets.astype(np.uint32).astype(">u4").view(np.uint8).reshape(n, 4)
    w[:, 3] = rng.integers(1, 4, n)                              # DROP / PASS / TX
    wcode = learn_prog(dm.fd)
    rcode = route_prog(dm.fd)
    npk = 1 << 16
    pk = gen.xdp_packets(npk, seed=22)
    pk[:, 12:14] = [0x08, 0x00]
    pk[: npk // 2, 30:34] = units[rng.integers(0, n, npk // 2), 8:12]
    ow = po.OracleVM()
    ow.load(wcode)
    ow.run_raw(units.copy(), 16)
    orr = po.OracleVM()
    orr.load(rcode)
    want = orr.run_xdp(pk.copy(), fixed_len=64)
    vw, vr = dev.VM(), dev.VM()
    vw.load(wcode)
    vr.load(rcode)
    s1, s2 = L.bpftime_amd_stream_create(), L.bpftime_amd_stream_create()
    try:
        du = dev.DeviceBuffer.from_array(units)
        dp = dev.DeviceBuffer.from_array(pk)
        dv = dev.DeviceBuffer(4 * npk)
        vw.exec_batch(dev.CTX_RAW, du, n, 16, fixed_len=16, flags=dev.BATCH_ORDERED, stream=s1)
        vr.exec_batch(dev.CTX_XDP, dp, npk, 64, fixed_len=64, verdicts=dv, flags=0, stream=s2)
        L.bpftime_amd_stream_sync(s2)
        np.testing.assert_array_equal(dv.download(np.uint32), want)
        assert dm.count() == om.count()
    finally:
        L.bpftime_amd_sync()
        L.bpftime_amd_stream_destroy(s1)
        L.bpftime_amd_stream_destroy(s2)
