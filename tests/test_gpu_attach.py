"""Attach-plugin boundary (attach/base_attach_impl/base_attach_impl.hpp:24-71,
attach/simple_attach_impl/simple_attach_impl.cpp:7-55) through the C ABI:
bpftime_amd_attach_run has the ebpf_run_callback shape, the simple attach
impl triggers device batches.  Results against the oracle."""
import ctypes as C
import struct

import numpy as np
import pytest

from bpftime_amd import gen, programs
from bpftime_amd._lib import EbpfBatch

from _helpers import xdp_counter_maps

pytestmark = pytest.mark.gpu

CB = C.CFUNCTYPE(C.c_int, C.c_char_p, C.c_void_p, C.c_void_p)


def test_attach_run_is_an_ebpf_run_callback(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    L = dev.lib()
    code = programs.kat_add_mem()
    pfd = dev.prog_create(code, "add", 1)
    a = L.bpftime_amd_attach_create(pfd, dev.CTX_RAW)
    assert a
    ovm = po.OracleVM()
    ovm.load(code)
    for x, y in ((1, 2), (0xFFFFFFFF, 7), (123456, 654321)):
        mem = bytearray(struct.pack("<II", x, y))
        buf = (C.c_uint8 * 8).from_buffer(mem)
        ret = C.c_uint64(7)
        assert L.bpftime_amd_attach_run(a, buf, 8, C.byref(ret)) == 0
        assert ret.value == ovm.exec(mem)[1] == x + y
    L.bpftime_amd_attach_destroy(a)
    assert not L.bpftime_amd_attach_create(999, -1)


def test_simple_attach_impl_triggers_device_batches(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    L = dev.lib()
    (octl, obss), (dctl, dbss) = xdp_counter_maps(po, dev)
    code = programs.xdp_counter(dctl.fd, dbss.fd)
    pfd = dev.prog_create(code, "xdp_pass", 6)
    seen = []
    n = 7000
    pk = gen.xdp_packets(n, seed=21)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)

    @CB
    def on_trigger(argument, trig, attach):
        # the user callback: the attach-time argument, the trigger argument
        # (here the batch size) and the attach entry to run
        seen.append((argument.decode(), trig))
        b = EbpfBatch(ctx_kind=dev.CTX_XDP, flags=dev.BATCH_SYNC, count=trig, data=d.ptr, stride=64,
                      fixed_len=64, verdicts=dv.ptr, sys_nr=-1)
        return L.bpftime_amd_attach_run_batch(attach, C.byref(b))

    ATTACH_TYPE = 1008
    impl = L.bpftime_amd_simple_attach_impl_create(ATTACH_TYPE, C.cast(on_trigger, C.c_void_p))
    assert impl > 0
    assert L.bpftime_amd_simple_trigger(impl, C.c_void_p(n)) == 1          # nothing attached yet
    assert L.bpftime_amd_simple_attach(impl, pfd, -1, b"ifname=eth0", ATTACH_TYPE + 1) == -1  # wrong type
    aid = L.bpftime_amd_simple_attach(impl, pfd, -1, b"ifname=eth0", ATTACH_TYPE)
    assert aid > 0
    assert L.bpftime_amd_simple_attach(impl, pfd, -1, b"again", ATTACH_TYPE) == -1   # one instance
    assert L.bpftime_amd_simple_trigger(impl, C.c_void_p(n)) == 0
    assert seen == [("ifname=eth0", n)]
    ovm = po.OracleVM()
    ovm.load(programs.xdp_counter(octl.fd, obss.fd))
    opk = pk.copy()
    ov = ovm.run_xdp(opk, fixed_len=64)
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    assert dbss.lookup(b"\0\0\0\0") == obss.lookup(b"\0\0\0\0")
    assert L.bpftime_amd_simple_detach(impl, aid + 1) == -1
    assert L.bpftime_amd_simple_detach(impl, aid) == 0
    assert L.bpftime_amd_simple_trigger(impl, C.c_void_p(n)) == 1
    assert L.bpftime_amd_simple_attach_impl_destroy(impl) == 0
