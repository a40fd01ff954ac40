"""Edge cases of the batch path: empty batches, batch sizes that are not
multiples of a wave or a block, zero-length and runt frames, and the
largest program the reference accepts (vm/vm-core/include/ebpf-vm.h:33-35:
65536 instructions) executed end to end."""
import numpy as np
import pytest

from bpftime_amd import gen, programs
from bpftime_amd.isa import Asm

from _helpers import xdp_counter_maps

pytestmark = pytest.mark.gpu


def test_empty_batch_launches_nothing(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    _, (ctl, bss) = xdp_counter_maps(None, dev)
    vm = dev.VM()
    vm.load(programs.xdp_counter(ctl.fd, bss.fd))
    d = dev.DeviceBuffer(64)
    assert vm.exec_batch(dev.CTX_XDP, d, 0, 64, fixed_len=64) == 0
    assert bss.lookup(b"\0\0\0\0") == bytes(4096)


@pytest.mark.parametrize("n", [1, 63, 65, 255, 257, 1000, 4097])
def test_ragged_batch_sizes(fresh_oracle, fresh_runtime, n):
    po, dev = fresh_oracle, fresh_runtime
    (octl, obss), (ctl, bss) = xdp_counter_maps(po, dev)
    code = programs.xdp_counter(ctl.fd, bss.fd)
    pk = gen.xdp_packets(n, seed=n)
    lens = (np.arange(n) * 7 % 80).astype(np.uint32)          # 0 .. 79 bytes, runts included
    lens = np.minimum(lens, 64).astype(np.uint32)
    ovm = po.OracleVM()
    ovm.load(code)
    opk = pk.copy()
    ov = ovm.run_xdp(opk, lens=lens)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, lens=dl, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    assert bss.lookup(b"\0\0\0\0") == obss.lookup(b"\0\0\0\0")
    assert (ov[lens < 14] == 1).all()                            # DROP for runts and empty frames


def test_largest_program(fresh_oracle, fresh_runtime):
    """65536 instructions load and run (a straight line of adds); 65537 are
    refused at load with the oracle's error."""
    po, dev = fresh_oracle, fresh_runtime
    k = 65536 - 3
    a = Asm().mov64(0, 0)
    for i in range(k):
        a.add64(0, (i % 5) + 1)
    a.alu64("add", 0, "r2").exit()                  # + the unit length (r2)
    code = a.assemble()
    assert len(code) // 8 == 65536
    n = 256
    units = np.zeros((n, 16), np.uint8)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_raw(units.copy(), 16)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 16, fixed_len=16, rets=dr) == 0
    got = dr.download(np.uint64)
    np.testing.assert_array_equal(got, want)
    too_big = Asm().mov64(0, 0)
    for _ in range(65536):
        too_big.add64(0, 1)
    too_big = too_big.exit().assemble()
    with pytest.raises(Exception, match="too many instructions"):
        dev.VM().load(too_big)
