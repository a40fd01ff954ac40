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
