"""A libbpf-style xdp-counter object (tests/_elf.py) loaded through the
object loader, attached with bpf_link (BPF_XDP) and run on the device:
verdicts, packet bytes and both maps bit-exact against the oracle running
the hand-assembled Appendix A program on the same maps."""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs
from bpftime_amd.object import BpfObject

import _elf

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("legacy", [False, True])
def test_object_load_attach_run(fresh_oracle, fresh_runtime, legacy):
    po, dev = fresh_oracle, fresh_runtime
    o = BpfObject.from_bytes(_elf.xdp_counter_object(legacy_maps=legacy), "xdp-counter")
    o.load()
    ctl, bss = o.map_fd("ctl_array"), o.map_fd("xdp_coun.bss")
    pfd = o.program_fd("xdp_pass")
    assert ctl >= 0 and bss >= 0 and pfd >= 0 and o.program_fd_by_secname("xdp") == pfd
    link = dev.link_create(pfd, 7, 37)  # BPF_XDP (bpftime_epoll.h:1158), target = ifindex
    assert link >= 0
    assert any(p == pfd and ifx == 7 for _, p, ifx in dev.xdp_links())
    octl = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, fd=ctl)
    obss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, fd=bss)
    vm = dev.prog_instantiate(pfd)
    n = 1 << 16
    pk = gen.xdp_packets(n)
    pk[:64, 12:] = 0  # some frames shorter than an Ethernet header below
    lens = np.full(n, 64, np.uint32)
    lens[:64] = np.arange(64) % 14
    d = dev.DeviceBuffer.from_array(pk)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, lens=dl, verdicts=dv) == 0
    ovm = po.OracleVM()
    ovm.load(programs.xdp_counter(ctl, bss))
    opk = pk.copy()
    ov = ovm.run_xdp(opk, lens=lens)
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    want = obss.lookup(b"\0\0\0\0")
    assert dev.Map.from_fd(bss).lookup(b"\0\0\0\0") == want
    assert struct.unpack_from("<Q", want)[0] == n
