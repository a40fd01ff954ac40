"""ebpf_set_unwind_function_index (vm/vm-core/include/ebpf-vm.h:181-191,
compat_ubpf.cpp:239-241 -> ubpf's unwind-on-success): a call of the helper
registered under that ubpf id which returns 0 ends the program with r0 = 0.
The oracle restates it (oracle/interp.c, the 0x85 case); the device ends the
unit in its C++ tier (interp.hip R_CALL), map_lookup_elem leaving its asm
handlers when it is the unwind helper.  ubpf ids follow the registration
order of the default helpers, the same on both sides (vm_api.cpp
bpftime_amd_register_default_helpers, oracle/helpers.c)."""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa
from bpftime_amd.isa import Asm

from _helpers import make_maps

UBPF_LOOKUP, UBPF_UPDATE, UBPF_CPU = 12, 13, 1   # registration order (1-based)


def prog(fd):
    """key = word & 7; v = lookup(key): hit -> 100 + *v; miss ->
    update(key, {key}) and 500 + its result."""
    a = Asm().ldx(4, 6, 1, 0).alu64("and", 6, 7).stx(4, 10, -4, "r6").stx(8, 10, -16, "r6")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(1)
    a.jmp("jeq", 0, 0, "miss").ldx(8, 0, 0, 0).add64(0, 100).exit()
    a.label("miss").ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -16)
    a.mov64(4, 0).call(2).add64(0, 500).exit()
    return a.assemble()


def _units(n):
    return gen.sm64(21, np.arange(n, dtype=np.uint64)).view(np.uint8).reshape(n, 8)


def test_oracle_unwind(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)
    for k in range(4):
        m.update(struct.pack("<I", k), struct.pack("<Q", 10 * k))
    u = _units(64)
    keys = u.view(np.uint32)[:, 0] & 7
    v = po.OracleVM()
    v.load(prog(m.fd))
    plain = v.run_raw(u.copy(), 8)
    np.testing.assert_array_equal(plain, np.where(keys < 4, 100 + 10 * keys, 499))
    v.set_unwind(UBPF_LOOKUP)                      # a miss returns 0: unwind
    np.testing.assert_array_equal(v.run_raw(u.copy(), 8), np.where(keys < 4, 100 + 10 * keys, 0))


@pytest.mark.gpu
@pytest.mark.parametrize("mtype,unwind,ordered", [
    (isa.BPF_MAP_TYPE_ARRAY, UBPF_LOOKUP, False),    # lookup (asm-tier helper) misses unwind
    (isa.BPF_MAP_TYPE_ARRAY, UBPF_UPDATE, False),    # failing updates (E2BIG) do not
    (isa.BPF_MAP_TYPE_HASH, UBPF_UPDATE, True),      # the inserting unit of each key unwinds
    (isa.BPF_MAP_TYPE_ARRAY, UBPF_CPU, False),       # a helper the program never calls
    (isa.BPF_MAP_TYPE_HASH, -1, True),
])
def test_device_unwind(fresh_oracle, fresh_runtime, mtype, unwind, ordered):
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(mtype, 4, 8, 4 if mtype == isa.BPF_MAP_TYPE_ARRAY else 64)], po, dev)
    if mtype == isa.BPF_MAP_TYPE_ARRAY:
        for k in range(4):
            for m in (om, dm):
                m.update(struct.pack("<I", k), struct.pack("<Q", 10 * k))
    n = 5000
    u = _units(n)
    code = prog(dm.fd)
    ovm, vm = po.OracleVM(), dev.VM()
    ovm.load(code)
    vm.load(code)
    if unwind >= 0:
        ovm.set_unwind(unwind)
        assert vm.set_unwind(unwind) == 0
    want = ovm.run_raw(u.copy(), 8)
    d = dev.DeviceBuffer.from_array(u)
    dr = dev.DeviceBuffer(8 * n)
    flags = dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr, flags=flags) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), want)
    if unwind == UBPF_LOOKUP:
        assert (want == 0).sum() > n // 4
    # ebpf_exec (one unit, the same kernel)
    rc, r0 = vm.exec(bytearray(u[3].tobytes()))
    assert rc == 0


def test_unwind_index_range():
    """ubpf ids below 64 (MAX_EXT_FUNCS) are accepted, no GPU needed"""
    from bpftime_amd import vm as dev
    vm = dev.VM()
    assert vm.set_unwind(63) == 0 and vm.set_unwind(64) == -1
