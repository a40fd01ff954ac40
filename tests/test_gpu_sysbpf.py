"""A libbpf loader's bpf(2) sequence through bpftime_amd_handle_sysbpf
(runtime/syscall-server/syscall_context.cpp:429-668): BPF_MAP_CREATE for
xdp-counter's two maps, BPF_MAP_UPDATE_ELEM of ctl_array, BPF_PROG_LOAD,
BPF_LINK_CREATE(BPF_XDP); the runner finds the link, runs a batch on the
device, and the loader reads the counter back with BPF_MAP_LOOKUP_ELEM --
verdicts, packets and the counter against the oracle."""
import ctypes as C
import errno
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs

from _helpers import xdp_counter_maps

pytestmark = pytest.mark.gpu


def _buf(b):
    a = bytearray(b)
    return a, C.addressof((C.c_char * max(len(a), 1)).from_buffer(a))


def test_libbpf_sequence_through_sysbpf(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    ctl, e = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array"))
    assert ctl >= 0, e
    bss, e = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1,
                                                                 name="xdp_coun.bss"))
    assert bss >= 0 and bss != ctl
    k, kp = _buf(struct.pack("<I", 0))
    v, vp = _buf(struct.pack("<I", 0))
    assert dev.sys_bpf(dev.BPF_MAP_UPDATE_ELEM, dev.attr_map_elem(ctl, kp, vp, isa.BPF_ANY))[0] == 0
    code = programs.xdp_counter(ctl, bss)
    ins, ip = _buf(code)
    pfd, e = dev.sys_bpf(dev.BPF_PROG_LOAD, dev.attr_prog_load(6, ip, len(code) // 8, name="xdp_pass"))
    assert pfd >= 0, e
    lfd, e = dev.sys_bpf(dev.BPF_LINK_CREATE, dev.attr_link_create(pfd, 3, 37))
    assert lfd >= 0, e
    assert dev.sys_bpf(dev.BPF_LINK_CREATE, dev.attr_link_create(999, 3, 37))[0] == -1
    links = dev.xdp_links()
    assert (lfd, pfd, 3) in links
    vm = dev.prog_instantiate(pfd)
    n = 5000
    pk = gen.xdp_packets(n, seed=44)
    (octl, obss), _ = xdp_counter_maps(po, None)
    ovm = po.OracleVM()
    ovm.load(programs.xdp_counter(octl.fd, obss.fd))
    opk = pk.copy()
    ov = ovm.run_xdp(opk, fixed_len=64)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    out, op = _buf(bytes(4096))
    assert dev.sys_bpf(dev.BPF_MAP_LOOKUP_ELEM, dev.attr_map_elem(bss, kp, op))[0] == 0
    assert bytes(out) == obss.lookup(struct.pack("<I", 0))
    assert struct.unpack_from("<Q", out)[0] == n
    # syscall-side errors: array key out of range, delete on an array, last key
    k2, k2p = _buf(struct.pack("<I", 2))
    assert dev.sys_bpf(dev.BPF_MAP_LOOKUP_ELEM, dev.attr_map_elem(ctl, k2p, vp)) == (-1, errno.ENOENT)
    assert dev.sys_bpf(dev.BPF_MAP_DELETE_ELEM, dev.attr_map_elem(ctl, kp))[0] == -1
    nk, nkp = _buf(bytes(4))
    assert dev.sys_bpf(dev.BPF_MAP_GET_NEXT_KEY, dev.attr_map_elem(ctl, 0, nkp))[0] == 0 and bytes(nk) == bytes(4)
    k1, k1p = _buf(struct.pack("<I", 1))
    assert dev.sys_bpf(dev.BPF_MAP_GET_NEXT_KEY, dev.attr_map_elem(ctl, k1p, nkp))[0] == -1
