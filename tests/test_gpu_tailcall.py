"""bpf_tail_call + BPF_MAP_TYPE_PROG_ARRAY on the device against the oracle:
the reference's user-to-user tail-call test
(runtime/unit-test/tailcall/test_user_to_user_tailcall.cpp), then an XDP
batch whose lanes take different targets (a packet writer, a map counter, an
empty slot, a 32-deep self recursion), and relinking after the prog array
or a target changes."""
import errno
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa
from bpftime_amd.isa import Asm

import _tailcall as tc

pytestmark = pytest.mark.gpu

I32 = lambda v: struct.pack("<i", v)  # noqa: E731
PA_FD, TARGET_FD, PA2_FD = 1001, 1002, 1003


def test_device_prog_array_map_kat(fresh_runtime):
    dev = fresh_runtime
    with pytest.raises(Exception):
        dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 8, 4)
    m = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    assert m.fd == PA_FD
    assert m.update(I32(0), I32(TARGET_FD)) < 0
    assert dev.prog_create(tc.ref_kat_target(), "tail_call_target", 1, fd=TARGET_FD) == TARGET_FD
    assert m.update(I32(0), I32(TARGET_FD)) == 0
    assert m.lookup(I32(0)) == I32(TARGET_FD)
    assert m.lookup(I32(1)) is None and m.lookup(I32(4)) is None
    assert m.next_key(None) == I32(0) and m.next_key(I32(2)) == I32(3) and m.next_key(I32(3)) is None
    assert m.delete(I32(0)) == 0 and m.lookup(I32(0)) is None
    assert m.update(I32(0), I32(TARGET_FD)) == 0
    dev.close_fd(TARGET_FD)
    assert m.lookup(I32(0)) is None


@pytest.mark.parametrize("tail_then_exit", [True, False])
def test_reference_tailcall_kat_device(fresh_oracle, fresh_runtime, tail_then_exit):
    po, dev = fresh_oracle, fresh_runtime
    m = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    dev.prog_create(tc.ref_kat_target(), "tail_call_target", 1, fd=TARGET_FD)
    assert m.update(I32(0), I32(TARGET_FD)) == 0
    vm = dev.VM()
    vm.load(tc.ref_kat_caller(PA_FD, tail_then_exit))
    rc, ret = vm.exec(bytearray(64))
    assert rc == 0 and ret == (0x1234 if tail_then_exit else 0xdead)
    # a batch of raw units takes the same path
    n = 300
    d = dev.DeviceBuffer(64 * n)
    d.zero()
    rets = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 64, fixed_len=64, rets=rets) == 0
    assert (rets.download(np.uint64) == (0x1234 if tail_then_exit else 0xdead)).all()
    # closing the target: the slot reads empty and the call returns -1
    dev.close_fd(TARGET_FD)
    rc, ret = vm.exec(bytearray(64))
    assert rc == 0 and ret == ((1 << 64) - 1 if tail_then_exit else 0xdead)


def _xdp_pair(po, dev):
    pa_o = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    pa_d = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    cnt_d = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)
    cnt_o = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4, fd=cnt_d.fd)
    progs = {900: tc.target_write(0xA1), 901: tc.target_count(cnt_d.fd),
             903: tc.target_recurse(PA_FD, cnt_d.fd, 3), 904: tc.target_write(0xB2)}
    for fd, code in progs.items():
        po.prog_create(fd, code)
        assert dev.prog_create(code, f"t{fd}", 6, fd=fd) == fd
    for k, fd in ((0, 900), (1, 901), (3, 903)):
        assert pa_o.update(I32(k), I32(fd)) == 0 and pa_d.update(I32(k), I32(fd)) == 0
    return (pa_o, cnt_o), (pa_d, cnt_d)


def _run_both(po, dev, ovm, dvm, n, seed, cnt_o, cnt_d):
    pk = gen.xdp_packets(n, seed=seed)
    pk[:, 0] = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
    opk = pk.copy()
    ov = ovm.run_xdp(opk, fixed_len=64, ifindex=5)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert dvm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv, ifindex=5) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    for i in range(4):
        assert cnt_d.lookup(I32(i)) == cnt_o.lookup(I32(i)), i
    return ov, opk


@pytest.mark.parametrize("n", [1, 64, 1000, 70000])
def test_xdp_tailcall_parity(fresh_oracle, fresh_runtime, n):
    po, dev = fresh_oracle, fresh_runtime
    (pa_o, cnt_o), (pa_d, cnt_d) = _xdp_pair(po, dev)
    code = tc.xdp_caller(PA_FD, cnt_d.fd)
    ovm = po.OracleVM()
    ovm.load(code)
    dvm = dev.VM()
    dvm.load(code)
    ov, opk = _run_both(po, dev, ovm, dvm, n, 11 + n, cnt_o, cnt_d)
    idx = opk[:, 0] & 3
    assert (ov[idx == 3] == 31 + 1005).all() and (ov[idx == 2] == (0xFFFFFFFF + 1005) & 0xFFFFFFFF).all()


# frame tiers: the asm tier's frames of the first depths in LDS (default:
# as many depths as keep the residency), none (TAIL_LDS 0), one depth; C++
# pops of asm-pushed frames (DBG 16) and C++ frames only (DBG 8)
@pytest.mark.parametrize("env", [{"BPFTIME_AMD_TAIL_LDS": "0"}, {"BPFTIME_AMD_TAIL_LDS": "1"},
                                 {"BPFTIME_AMD_DBG": "16"}, {"BPFTIME_AMD_DBG": "8"}])
def test_xdp_tailcall_frame_tiers(fresh_oracle, fresh_runtime, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    test_xdp_tailcall_parity(fresh_oracle, fresh_runtime, 70000)


def _mixed_array_caller():
    """Like xdp_caller, but lanes with data[1] odd tail-call through a second
    prog array (same slots): the map fd is not wave-uniform, so the C++ tier
    pushes those waves' depth-0 frames (full frames, in global memory) and
    the asm tier pops them at the targets' exits only through C++, while the
    recursion target pushes its own frames in the asm tier."""
    a = Asm()
    a.mov64(6, "r1")
    a.ldx(8, 2, 6, 0).ldx(8, 3, 6, 8)
    a.mov64(4, "r2").add64(4, 2).jmp("jgt", 4, "r3", "short")
    a.ldx(1, 7, 2, 0).alu64("and", 7, 3)
    a.ldx(1, 8, 2, 1).alu64("and", 8, 1)
    a.lddw(9, 0x1111222233334444).stx(8, 10, -8, 9)
    a.ld_map_fd(2, PA_FD)
    a.jmp("jeq", 8, 0, "one")
    a.ld_map_fd(2, PA2_FD)
    a.label("one")
    a.mov64(1, "r6").mov64(3, "r7").call(tc.TAIL)
    a.ldx(8, 1, 10, -8).lddw(2, 0x1111222233334444).jmp("jne", 1, "r2", "bad")
    a.add64(0, 1000)
    a.label("bad")
    a.ldx(4, 1, 6, 20).alu64("add", 0, "r1")
    a.exit()
    a.label("short").mov64(0, 1).exit()
    return a.assemble()


@pytest.mark.parametrize("lds", ["0", "4"])
def test_xdp_tailcall_full_and_masked_frames(fresh_oracle, fresh_runtime, monkeypatch, lds):
    monkeypatch.setenv("BPFTIME_AMD_TAIL_LDS", lds)
    po, dev = fresh_oracle, fresh_runtime
    (pa_o, cnt_o), (pa_d, cnt_d) = _xdp_pair(po, dev)
    pa2_o = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA2_FD)
    pa2_d = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA2_FD)
    for k, fd in ((0, 900), (1, 901), (3, 903)):
        assert pa2_o.update(I32(k), I32(fd)) == 0 and pa2_d.update(I32(k), I32(fd)) == 0
    code = _mixed_array_caller()
    ovm = po.OracleVM()
    ovm.load(code)
    dvm = dev.VM()
    dvm.load(code)
    ov, opk = _run_both(po, dev, ovm, dvm, 70000, 5, cnt_o, cnt_d)
    idx = opk[:, 0] & 3
    assert (ov[idx == 3] == 31 + 1005).all() and (ov[idx == 1] == 2 + 1005).all()


def test_xdp_tailcall_relink(fresh_oracle, fresh_runtime):
    """Prog array writes between launches relink the image: slot 1 now names
    another writer, slot 0 is deleted, then the recursion target is closed."""
    po, dev = fresh_oracle, fresh_runtime
    (pa_o, cnt_o), (pa_d, cnt_d) = _xdp_pair(po, dev)
    code = tc.xdp_caller(PA_FD, cnt_d.fd)
    ovm = po.OracleVM()
    ovm.load(code)
    dvm = dev.VM()
    dvm.load(code)
    _run_both(po, dev, ovm, dvm, 4096, 1, cnt_o, cnt_d)
    for m in (pa_o, pa_d):
        assert m.update(I32(1), I32(904)) == 0 and m.delete(I32(0)) == 0
    ov, opk = _run_both(po, dev, ovm, dvm, 4096, 2, cnt_o, cnt_d)
    assert (opk[(opk[:, 0] & 3) == 1, 1] == 0xB2).all()
    po.prog_close(903)
    dev.close_fd(903)
    ov, opk = _run_both(po, dev, ovm, dvm, 4096, 3, cnt_o, cnt_d)
    assert (ov[(opk[:, 0] & 3) == 3] == (0xFFFFFFFF + 1005) & 0xFFFFFFFF).all()


def test_image_atomic_adds_summed_per_address(fresh_oracle, fresh_runtime):
    """In a linked image, adds without fetch run in the C++ tier summed per
    address across the wave: 4-byte adds to eight lane-dependent slots and
    8-byte adds to one slot equal the oracle's sequential sums."""
    po, dev = fresh_oracle, fresh_runtime
    pa_d = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 1, fd=PA_FD)
    pa_o = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 1, fd=PA_FD)
    c32_d = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 48, 1)
    c32_o = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 48, 1, fd=c32_d.fd)
    seven = Asm().mov64(0, 7).exit().assemble()
    po.prog_create(TARGET_FD, seven)
    dev.prog_create(seven, "seven", 6, fd=TARGET_FD)
    for m in (pa_o, pa_d):
        assert m.update(I32(0), I32(TARGET_FD)) == 0
    a = Asm().mov64(6, "r1")
    a.ldx(8, 7, 6, 0).ldx(8, 3, 6, 8).mov64(4, "r7").add64(4, 1).jmp("jgt", 4, "r3", "out")
    a.ldx(1, 8, 7, 0).alu64("and", 8, 7).alu64("lsh", 8, 2)       # r8 = 4 * (data[0] & 7)
    a.mov64(1, "r6").ld_map_fd(2, PA_FD).mov64(3, 0).call(tc.TAIL)
    a.mov64(9, "r0")
    a.ld_map_value(1, c32_d.fd, 0).alu64("add", 1, "r8").atomic(4, 0x00, 1, 0, 9)
    a.ld_map_value(1, c32_d.fd, 0).mov64(2, 1).atomic(8, 0x00, 1, 32, 2)
    a.label("out").mov64(0, 2).exit()
    code = a.assemble()
    ovm = po.OracleVM()
    ovm.load(code)
    dvm = dev.VM()
    dvm.load(code)
    n = 20000
    pk = gen.xdp_packets(n, seed=3)
    ov = ovm.run_xdp(pk.copy(), fixed_len=64)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert dvm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    assert c32_d.lookup(I32(0)) == c32_o.lookup(I32(0))
    got = np.frombuffer(c32_d.lookup(I32(0)), dtype=np.uint32)
    assert int(got[:8].sum()) == 7 * n and struct.unpack_from("<Q", c32_d.lookup(I32(0)), 32)[0] == n


def test_tailcall_batches_on_two_streams(fresh_oracle, fresh_runtime):
    """Two tail-call batches in flight at once on two streams (the same VM
    and a second VM): each launch has its own frames (per-stream buffers),
    so neither resumes the other's callers."""
    po, dev = fresh_oracle, fresh_runtime
    (pa_o, cnt_o), (pa_d, cnt_d) = _xdp_pair(po, dev)
    code = tc.xdp_caller(PA_FD, cnt_d.fd)
    ovm = po.OracleVM()
    ovm.load(code)
    vms = [dev.VM(), dev.VM()]
    for v in vms:
        v.load(code)
    streams = [dev.lib().bpftime_amd_stream_create() for _ in range(3)]
    n = 50000
    jobs = []
    for i, (vm, s) in enumerate(((vms[0], streams[0]), (vms[0], streams[1]), (vms[1], streams[2]))):
        pk = gen.xdp_packets(n, seed=100 + i)
        pk[:, 0] = np.random.default_rng(100 + i).integers(0, 256, n, dtype=np.uint8)
        opk = pk.copy()
        ov = ovm.run_xdp(opk, fixed_len=64, ifindex=5)
        d = dev.DeviceBuffer.from_array(pk)
        dv = dev.DeviceBuffer(4 * n)
        assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv, ifindex=5, flags=0, stream=s) == 0
        jobs.append((d, dv, ov, opk))
    for s in streams:
        assert dev.lib().bpftime_amd_stream_sync(s) == 0
        dev.lib().bpftime_amd_stream_destroy(s)
    for d, dv, ov, opk in jobs:
        np.testing.assert_array_equal(dv.download(np.uint32), ov)
        np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    for i in range(4):
        assert cnt_d.lookup(I32(i)) == cnt_o.lookup(I32(i)), i


def test_prog_array_lookup_returns_a_copy(fresh_oracle, fresh_runtime):
    """map_lookup_elem on a PROG_ARRAY hands out a copy of the fd
    (prog_array.cpp:113-143, a thread-local): writing through it leaves the
    array and the following tail call unchanged; r0 = the fd read back +
    the target's result."""
    po, dev = fresh_oracle, fresh_runtime
    (pa_o, cnt_o), (pa_d, cnt_d) = _xdp_pair(po, dev)
    a = isa.Asm().mov64(6, "r1").st(4, 10, -4, 0)
    a.ld_map_fd(1, PA_FD).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.mov64(7, 0).jmp("jeq", 0, 0, "call").ldx(4, 7, 0, 0).st(4, 0, 0, 901)   # overwrite the copy
    a.label("call").mov64(1, "r6").ld_map_fd(2, PA_FD).mov64(3, 0).call(12)
    a.alu64("lsh", 7, 16).alu64("add", 0, "r7").exit()
    code = a.assemble()
    ovm = po.OracleVM()
    ovm.load(code)
    dvm = dev.VM()
    dvm.load(code)
    ov, opk = _run_both(po, dev, ovm, dvm, 3000, 5, cnt_o, cnt_d)
    assert ((ov >> 16) == 900).all() and ((ov & 0xFFFF) == 64 + 0xA1).all()
    assert pa_d.lookup(I32(0)) == I32(900)
