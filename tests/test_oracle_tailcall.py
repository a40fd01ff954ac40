"""Oracle (CPU checker) for bpf_tail_call and BPF_MAP_TYPE_PROG_ARRAY,
pinned by runtime/unit-test/tailcall/test_user_to_user_tailcall.cpp and the
prog_array.cpp semantics it exercises.  The reference test runs the llvm VM
(the caller ends with the target's 0x1234); under the interpreter backend
this path restates (ubpf + bpftime_tail_call, bpf_helper.cpp:568-650) the
helper returns the target's r0 and the caller continues, so the caller that
exits right after the call gives 0x1234 under both."""
import errno
import struct

import numpy as np

from bpftime_amd import gen, isa

import _tailcall as tc

I32 = lambda v: struct.pack("<i", v)  # noqa: E731
PA_FD, TARGET_FD = 1001, 1002         # the reference test's fds


def test_prog_array_map_kat(fresh_oracle):
    po = fresh_oracle
    try:
        po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 8, 4)
        raise AssertionError("value size 8 accepted")
    except RuntimeError:
        pass
    m = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    assert m.update(I32(0), I32(TARGET_FD)) == -1 and m.errno() == errno.EBADF   # not a prog fd
    assert po.prog_create(TARGET_FD, tc.ref_kat_target()) == TARGET_FD
    assert m.update(I32(0), I32(TARGET_FD)) == 0
    assert m.lookup(I32(0)) == I32(TARGET_FD)
    assert m.lookup(I32(1)) is None and m.errno() == errno.ENOENT                # INVALID_ENTRY
    assert m.lookup(I32(4)) is None and m.errno() == errno.EINVAL
    assert m.update(I32(-1), I32(TARGET_FD)) == -1 and m.errno() == errno.EINVAL
    assert m.next_key(None) == I32(0) and m.next_key(I32(2)) == I32(3)
    assert m.next_key(I32(3)) is None and m.errno() == errno.ENOENT
    assert m.delete(I32(0)) == 0 and m.lookup(I32(0)) is None
    assert m.update(I32(0), I32(TARGET_FD)) == 0
    po.prog_close(TARGET_FD)                                                     # the reference test's last check
    assert m.lookup(I32(0)) is None


def _ref_kat(po, tail_then_exit):
    m = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    po.prog_create(TARGET_FD, tc.ref_kat_target())
    assert m.update(I32(0), I32(TARGET_FD)) == 0
    vm = po.OracleVM()
    vm.load(tc.ref_kat_caller(PA_FD, tail_then_exit))
    return vm


def test_reference_tailcall_kat(fresh_oracle):
    vm = _ref_kat(fresh_oracle, True)
    rc, ret = vm.exec(bytearray(64))
    assert rc == 0 and ret == 0x1234


def test_tailcall_returns_to_caller_in_interpreter(fresh_oracle):
    vm = _ref_kat(fresh_oracle, False)
    rc, ret = vm.exec(bytearray(64))
    assert rc == 0 and ret == 0xdead


def test_tailcall_failures_return_minus_one(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA_FD)
    arr = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 4, fd=PA_FD + 1)
    po.prog_create(TARGET_FD, tc.ref_kat_target())
    m.update(I32(0), I32(TARGET_FD))
    for fd, idx in ((PA_FD, 1), (PA_FD, 4), (PA_FD, -1), (arr.fd, 0), (999, 0)):
        vm = po.OracleVM()
        from bpftime_amd.isa import Asm
        vm.load(Asm().lddw(2, fd).mov64(3, idx).call(tc.TAIL).exit().assemble())
        rc, ret = vm.exec(bytearray(64))
        assert rc == 0 and ret == (1 << 64) - 1, (fd, idx)




def test_xdp_tailcall_chain_oracle(fresh_oracle):
    po = fresh_oracle
    pa = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4)
    cnt = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)
    po.prog_create(900, tc.target_write(0xA1))
    po.prog_create(901, tc.target_count(cnt.fd))
    po.prog_create(903, tc.target_recurse(pa.fd, cnt.fd, 3))
    for k, fd in ((0, 900), (1, 901), (3, 903)):
        assert pa.update(I32(k), I32(fd)) == 0
    vm = po.OracleVM()
    vm.load(tc.xdp_caller(pa.fd, cnt.fd))
    n = 64
    pk = gen.xdp_packets(n, seed=7)
    pk[:, 0] = np.arange(n) & 3
    v = vm.run_xdp(pk, fixed_len=64, ifindex=5)
    idx = np.arange(n) & 3
    exp = np.where(idx == 0, 64 + 0xA1, np.where(idx == 1, 2, np.where(idx == 2, 0xFFFFFFFF, 31)))
    exp = (exp.astype(np.uint64) + 1000 + 5) & 0xFFFFFFFF
    np.testing.assert_array_equal(v, exp.astype(np.uint32))
    assert (pk[idx == 0, 1] == 0xA1).all()                       # packet write through the copy's data
    c = [struct.unpack("<Q", cnt.lookup(I32(i)))[0] for i in range(4)]
    assert c[1] == 2 * (n // 4) and c[2] == n // 4 + 32 * (n // 4)  # 32 nested levels per idx-3 packet
    assert c[0] == n // 4 and c[3] == n // 4
