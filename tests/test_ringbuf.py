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


def sampler(rb_fd, out_size=12):
    """byte0 % 16 == 0: ringbuf_output(first out_size bytes); == 1: reserve 16 B,
    fill {u64 bytes 0-7, u32 len, u32 byte1}, submit if byte1 is odd else
    discard.  Verdict PASS, DROP when the ring had no room."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, 2)
    a.mov64(4, "r2").add64(4, 14).jmp("jgt", 4, "r3", "out")
    a.mov64(6, "r2").mov64(7, "r3").alu64("sub", 7, "r2")              # r6 = data, r7 = len
    a.ldx(1, 8, 6, 0).alu64("and", 8, 15)
    a.jmp("jeq", 8, 0, "out0").jmp("jeq", 8, 1, "res").ja("out")
    a.label("out0")
    a.ld_map_fd(1, rb_fd).mov64(2, "r6").mov64(3, out_size).mov64(4, 0).call(130)
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
    RbStage: records reach the ring when their block ends, in the bytes it
    reserves for exactly them)"""
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


def _output_program(rb_fd, size, off):
    """byte0 % 8 == 0: bpf_ringbuf_output(data + off, size); verdict TX when
    it succeeded, DROP when not, PASS for the others."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, 2)
    a.mov64(4, "r2").add64(4, 32).jmp("jgt", 4, "r3", "out")
    a.ldx(1, 8, 2, 0).alu64("and", 8, 7).jmp("jne", 8, 0, "out")
    a.ld_map_fd(1, rb_fd).add64(2, off).mov64(3, size).mov64(4, 0).call(130)
    a.mov64(1, "r0").mov64(0, 3).jmp("jeq", 1, 0, "out").mov64(0, 1)
    a.label("out").exit()
    return a.assemble()


@pytest.mark.gpu
@pytest.mark.parametrize("size,off", [(4, 0), (8, 4), (12, 0), (16, 16), (12, 2), (0, 8), (20, 0)])
def test_device_ringbuf_output_sizes(fresh_oracle, fresh_runtime, size, off):
    """bpf_ringbuf_output of packet bytes [off, off + size) through a staged
    ring: dword-aligned sources of up to 16 B are written by the asm tier
    from the staged window (gen_fast.py call_rbout), the others (an odd
    offset, 20 B) by the C++ tier; verdicts equal and the record multiset
    equals the oracle's."""
    po, dev = fresh_oracle, fresh_runtime
    dm = dev.Map(RB, 0, 0, 1 << 26)
    om = po.OracleMap(RB, 0, 0, 1 << 26, fd=dm.fd)
    code = _output_program(dm.fd, size, off)
    n = 1 << 17
    pk = gen.xdp_packets(n, seed=40 + size + off)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), fixed_len=64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), want)
    drecs, orecs = dm.ringbuf_fetch(cap=1 << 24), om.ringbuf_fetch()
    assert len(drecs) == int((pk[:, 0] % 8 == 0).sum()) > 1000
    assert sorted(drecs) == sorted(orecs)


def _wrap_stream(rounds, n, seed):
    """Per-round frames of a wrap test: every 16th frame outputs 12 B (a 24-B
    record), frames with byte0 % 16 == 1 reserve 16 B and submit or discard."""
    for r in range(rounds):
        pk = gen.xdp_packets(n, seed=seed + r)
        sel = np.arange(n) % 16
        pk[:, 0] = np.where(sel == 0, 0, np.where(sel == 5, 1, 2))
        yield pk


def test_oracle_ringbuf_wraps(fresh_oracle):
    """A 4096-B ring wrapped 40 times by bpf_ringbuf_output records (24 B;
    4096 is not a multiple, so records straddle the end and one in 512 has
    its data at the ring's first byte), consumed after every round.
    bpf_ringbuf_output submits by the fd it reserved from
    (bpf_helper.cpp:460-465) -- the oracle once read the fd in front of the
    data there and left that record BUSY, stalling the consumer.
    The reference ring is not double-mapped (ringbuf_map.cpp:157-176: a plain
    2 x max_ent buffer): a record whose data wrapped is written at data[0]
    but fetch_data hands out data + (cons & mask) + 8 = data[max_ent..], the
    bytes the last straddling record left past the end (4 of them; the rest
    zero).  Restated exactly."""
    po = fresh_oracle
    size = 4096
    m = po.OracleMap(RB, 0, 0, size)
    v = po.OracleVM()
    v.load(sampler(m.fd))
    pos, tail, wrapped = 0, bytes(12), 0
    for pk in _wrap_stream(40, 1024, 100):
        pk[:, 0] = np.where(pk[:, 0] == 1, 2, pk[:, 0])      # output records only
        out = v.run_xdp(pk.copy(), fixed_len=64)
        assert (out == 2).all()
        want = []
        for p in pk[pk[:, 0] == 0]:
            rec = bytes(p[:12])
            o = (pos + 8) % size
            if o == 0:                                       # data wrapped to data[0]
                want.append(tail)
                wrapped += 1
            else:
                want.append(rec)
                if o + 12 > size:                            # straddles: bytes past the end
                    tail = rec[size - o:] + bytes(12 - (o + 12 - size))
            pos += 24
        assert m.ringbuf_fetch() == want
    assert wrapped >= 2


def test_oracle_ringbuf_submit_at_wrap(fresh_oracle):
    """bpf_ringbuf_submit reads the fd from ptr[-1] (bpf_helper.cpp:478-479).
    A reserved record whose data wrapped to the ring's first byte has the
    zeroed word in front of the ring's data there (the reference's producer
    page), fd 0: unless fd 0 is a ring the submit fails and the record stays
    BUSY, and the consumer stops at it."""
    po = fresh_oracle
    m = po.OracleMap(RB, 0, 0, 4096, fd=7)
    v = po.OracleVM()
    v.load(sampler(m.fd))
    pk = gen.xdp_packets(512, seed=3)
    pk[:, 0] = 1
    pk[:, 1] = 1                                             # reserve 16 B + submit: 24-B records
    got = 0
    for r in range(15):
        out = v.run_xdp(pk[:50].copy(), fixed_len=64)
        got += len(m.ringbuf_fetch())
    # the record at position 2 * 4096 - 8 (data at offset 0) stays BUSY
    assert got == (2 * 4096 - 8) // 24
    assert (out == 1).any()                                  # the ring then fills: DROP


@pytest.mark.gpu
@pytest.mark.parametrize("ordered", [False, True])
def test_device_ringbuf_wraps(fresh_oracle, fresh_runtime, ordered):
    """40 rounds over a 4096-B ring (no staging: rings under 64 MiB reserve
    directly), consumed between rounds.  ORDERED batches run the mixed
    sampler (12-B outputs, reserve + submit / discard): records straddle the
    end, some have their data at the ring's first byte (fetched from past
    the end, and a reserved one stays BUSY: its submit reads fd 0, not a map
    here), the consumer stalls and the ring fills -- records and verdicts
    identical to the oracle's in order.  Parallel batches run 8-B outputs
    (16-B records that never straddle), record multisets equal per round."""
    po, dev = fresh_oracle, fresh_runtime
    dm = dev.Map(RB, 0, 0, 4096, fd=7)
    om = po.OracleMap(RB, 0, 0, 4096, fd=7)
    code = sampler(dm.fd, 12 if ordered else 8)
    ovm = po.OracleVM()
    ovm.load(code)
    vm = dev.VM()
    vm.load(code)
    n = 1024
    drops = 0
    for pk in _wrap_stream(40, n, 200):
        if not ordered:
            pk[:, 0] = np.where(pk[:, 0] == 1, 2, pk[:, 0])
        want = ovm.run_xdp(pk.copy(), fixed_len=64)
        d = dev.DeviceBuffer.from_array(pk)
        dv = dev.DeviceBuffer(4 * n)
        flags = dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0)
        assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv, flags=flags) == 0
        np.testing.assert_array_equal(dv.download(np.uint32), want)
        drops += int((want == 1).sum())
        drecs, orecs = dm.ringbuf_fetch(), om.ringbuf_fetch()
        if ordered:
            assert drecs == orecs
        else:
            assert sorted(drecs) == sorted(orecs) and len(drecs) == (pk[:, 0] == 0).sum()
    assert (drops > 0) == ordered


@pytest.mark.gpu
@pytest.mark.parametrize("ordered", [True, False])
def test_device_ringbuf_fills_within_launch(fresh_oracle, fresh_runtime, ordered):
    """A 1 MiB ring that starts the launch empty and fills part way through
    it (2^17 frames, each writing a 24-B record, 43690 fit): ORDERED batches
    reproduce the oracle's records, order and verdicts exactly; parallel
    batches accept exactly as many records as fit (lane-exact CAS
    reservations once the ring is too full for a wave's fetch-and-add), with
    DROP verdicts for the rest."""
    po, dev = fresh_oracle, fresh_runtime
    size = 1 << 20
    dm = dev.Map(RB, 0, 0, size, fd=7)
    om = po.OracleMap(RB, 0, 0, size, fd=7)
    code = sampler(dm.fd)
    n = 1 << 17
    pk = gen.xdp_packets(n, seed=31)
    pk[:, 0] = 0                                             # every frame outputs 12 B
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), fixed_len=64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    flags = dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv, flags=flags) == 0
    got = dv.download(np.uint32)
    drecs, orecs = dm.ringbuf_fetch(), om.ringbuf_fetch()
    assert (want == 2).sum() == size // 24 and len(orecs) == size // 24
    if ordered:
        np.testing.assert_array_equal(got, want)
        assert drecs == orecs
    else:
        assert (got == 2).sum() == size // 24 and (got == 1).sum() == n - size // 24
        assert len(drecs) == size // 24
        assert set(drecs) <= {bytes(p[:12]) for p in pk}


@pytest.mark.gpu
def test_device_ringbuf_staged_ring_fills_within_launch(fresh_oracle, fresh_runtime):
    """A 64 MiB ring (large enough for block staging, dev_helpers.hpp RbStage)
    filled part way through one parallel launch: staged blocks reserve
    exactly the bytes they used when they end and no ring byte is wasted, so
    the ring accepts exactly what the reference's serial reservations
    accept, room / record size (ringbuf_map.cpp:262-295); every accepted
    record is delivered and the verdicts agree with the records."""
    po, dev = fresh_oracle, fresh_runtime
    size = 1 << 26
    dm = dev.Map(RB, 0, 0, size, fd=7)
    n = 3 << 20                                              # 72 MiB of 24-B records
    pk = gen.xdp_packets(n, seed=32)
    pk[:, 0] = 0
    vm = dev.VM()
    vm.load(sampler(dm.fd))
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    got = dv.download(np.uint32)
    drecs = dm.ringbuf_fetch(cap=1 << 27)
    fit = size // 24
    ok = int((got == 2).sum())
    assert ok == len(drecs) and ok + int((got == 1).sum()) == n
    assert ok == fit


def two_ring_sampler(fd_a, fd_b):
    """bpf_ringbuf_output of the first 16 bytes to ring A when byte1 is odd,
    else ring B; verdict PASS on success, DROP when the ring had no room."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, 2)
    a.mov64(4, "r2").add64(4, 16).jmp("jgt", 4, "r3", "out")
    a.mov64(6, "r2").ldx(1, 8, 6, 1).alu64("and", 8, 1)
    a.jmp("jeq", 8, 0, "b")
    a.ld_map_fd(1, fd_a).ja("go")
    a.label("b").ld_map_fd(1, fd_b)
    a.label("go").mov64(2, "r6").mov64(3, 16).mov64(4, 0).call(130)
    a.mov64(1, "r0").mov64(0, 2).jmp("jeq", 1, 0, "out").mov64(0, 1)
    a.label("out").exit()
    return a.assemble()


@pytest.mark.gpu
def test_device_two_staged_rings_fill_within_launch(fresh_oracle, fresh_runtime):
    """a block holding its staging promise on one ring and
    waiting for room on another could wait for a block doing the reverse.
    One program fills two 64 MiB staged rings in one parallel launch: the
    launch ends, and each ring accepts exactly room / record size, every
    accepted record delivered (ringbuf_map.cpp:262-295)."""
    po, dev = fresh_oracle, fresh_runtime
    size = 1 << 26
    ra = dev.Map(RB, 0, 0, size, fd=7)
    rb = dev.Map(RB, 0, 0, size, fd=8)
    n = 3 << 21                                              # ~75 MB of 24-B records per ring
    pk = gen.xdp_packets(n, seed=33)
    vm = dev.VM()
    vm.load(two_ring_sampler(ra.fd, rb.fd))
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    got = dv.download(np.uint32)
    fit = size // 24
    odd = (pk[:, 1] & 1) == 1
    assert odd.sum() > fit and (~odd).sum() > fit
    ra_recs = ra.ringbuf_fetch(cap=1 << 27)
    rb_recs = rb.ringbuf_fetch(cap=1 << 27)
    assert len(ra_recs) == fit and len(rb_recs) == fit
    assert int((got[odd] == 2).sum()) == fit and int((got[~odd] == 2).sum()) == fit
    assert int((got == 1).sum()) == n - 2 * fit
    # every delivered record is the first 16 bytes of an accepted frame of its ring
    acc_a = {bytes(pk[i, :16]) for i in np.flatnonzero(odd & (got == 2))}
    assert all(r in acc_a for r in ra_recs[:1000])
