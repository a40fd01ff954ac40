"""Ring buffer (BPF_MAP_TYPE_RINGBUF, helpers 130-133; ringbuf_map.cpp,
bpf_helper.cpp:451-504): the oracle's reserve / submit / discard / output
and consumer rules, and an XDP sampler on the device whose records match
the oracle's as a multiset (the device interleaves producers, the reference
runs them in packet order)."""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa
from bpftime_amd.isa import Asm

RB = isa.BPF_MAP_TYPE_RINGBUF


def sampler(rb_fd):
    """byte0 % 16 == 0: ringbuf_output(first 12 bytes); == 1: reserve 16 B,
    fill {u64 bytes 0-7, u32 len, u32 byte1}, submit if byte1 is odd else
    discard.  Verdict PASS, DROP when the ring had no room."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, 2)
    a.mov64(4, "r2").add64(4, 14).jmp("jgt", 4, "r3", "out")
    a.mov64(6, "r2").mov64(7, "r3").alu64("sub", 7, "r2")              # r6 = data, r7 = len
    a.ldx(1, 8, 6, 0).alu64("and", 8, 15)
    a.jmp("jeq", 8, 0, "out0").jmp("jeq", 8, 1, "res").ja("out")
    a.label("out0")
    a.ld_map_fd(1, rb_fd).mov64(2, "r6").mov64(3, 12).mov64(4, 0).call(130)
    a.mov64(1, "r0").mov64(0, 2).jmp("jeq", 1, 0, "out").mov64(0, 1).ja("out")
    a.label("res")
    a.ld_map_fd(1, rb_fd).mov64(2, 16).mov64(3, 0).call(131)
    a.mov64(1, "r0").mov64(0, 1).jmp("jeq", 1, 0, "out")
    a.ldx(8, 2, 6, 0).stx(8, 1, 0, "r2").stx(4, 1, 8, "r7").ldx(1, 2, 6, 1).stx(4, 1, 12, "r2")
    a.alu64("and", 2, 1).jmp("jeq", 2, 0, "disc")
    a.mov64(2, 0).call(132).mov64(0, 2).ja("out")
    a.label("disc").mov64(2, 0).call(133).mov64(0, 2)
    a.label("out").exit()
    return a.assemble()


def test_oracle_ringbuf_rules(fresh_oracle):
    po = fresh_oracle
    with pytest.raises(RuntimeError):
        po.OracleMap(RB, 0, 0, 3000)                        # not a power of two
    m = po.OracleMap(RB, 0, 0, 1 << 20)
    v = po.OracleVM()
    v.load(sampler(m.fd))
    pk = gen.xdp_packets(4096, seed=4)
    pk[:, 0] = np.where(np.arange(4096) % 16 == 0, 0, 2)   # every 16th: output 12 B (24-B record)
    out = v.run_xdp(pk.copy(), fixed_len=64)
    recs = m.ringbuf_fetch()
    assert recs == [bytes(p[:12]) for p in pk[::16]]      # in packet order
    assert (out == 2).all() and m.ringbuf_fetch() == []
    # reserve + submit / discard: only submitted records are delivered
    pk[:, 0] = 1
    pk[:, 1] = np.arange(4096) % 4
    out = v.run_xdp(pk.copy(), fixed_len=64)
    recs = m.ringbuf_fetch()
    assert (out == 2).all() and len(recs) == 2048
    assert recs[0] == bytes(pk[1, :8]) + struct.pack("<II", 64, 1)
    # a full ring: 170 records of 24 B fit in 4096 B, the rest fail (DROP)
    small = po.OracleMap(RB, 0, 0, 4096)
    v2 = po.OracleVM()
    v2.load(sampler(small.fd))
    pk[:, 0] = 0
    out = v2.run_xdp(pk.copy(), fixed_len=64)
    assert (out == 2).sum() == 4096 // 24 and (out == 1).sum() == 4096 - 4096 // 24
    assert len(small.ringbuf_fetch()) == 4096 // 24


@pytest.mark.gpu
@pytest.mark.parametrize("size,frac", [(1 << 20, None), (4096, 0), (1 << 26, None)])
def test_device_ringbuf_sampler(fresh_oracle, fresh_runtime, size, frac):
    """(1 << 26: a ring large enough for block staging, dev_helpers.hpp
    RbStage: records reach the ring through per-block chunks whose unused
    tails are DISCARD records the consumer skips)"""
    po, dev = fresh_oracle, fresh_runtime
    dm = dev.Map(RB, 0, 0, size)
    om = po.OracleMap(RB, 0, 0, size, fd=dm.fd)
    code = sampler(dm.fd)
    n = 1 << 16
    pk = gen.xdp_packets(n, seed=8)
    if frac is not None:
        pk[:, 0] = frac                                      # everyone outputs: the ring overflows
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), fixed_len=64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    got = dv.download(np.uint32)
    drecs, orecs = dm.ringbuf_fetch(), om.ringbuf_fetch()
    if frac is None:
        np.testing.assert_array_equal(got, want)
        assert sorted(drecs) == sorted(orecs) and len(drecs) > 1000
    else:
        # which packets win the room depends on order; how many does not
        assert (got == 2).sum() == (want == 2).sum() == size // 24
        assert len(drecs) == len(orecs) == size // 24
        assert set(drecs) <= {bytes(p[:12]) for p in pk}
    assert dm.ringbuf_fetch() == []                          # consumed
