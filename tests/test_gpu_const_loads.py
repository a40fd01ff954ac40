"""Constant-address loads through the scalar cache (loader.cpp const_loads,
gen_fast.py ldxk): loads from an ARRAY map value at an lddw map_val address
that nothing in the program writes -- libbpf's .rodata globals -- are read
with s_load; a program that may write the location keeps the vector load.
Both against the oracle."""
import struct

import numpy as np
import pytest

from bpftime_amd import isa
from bpftime_amd.isa import Asm

from _helpers import make_maps

pytestmark = pytest.mark.gpu


def _reader(fd):
    """r0 = u8 @1 + u16 @2 + u32 @4 + u64 @8 + u32 @20 + (the unit's first
    u64 & 7): constant loads of every width at aligned offsets."""
    a = Asm().ldx(8, 6, 1, 0).alu64("and", 6, 7)
    a.ld_map_value(2, fd, 0)
    a.ldx(1, 3, 2, 1).alu64("add", 6, "r3")
    a.ldx(2, 3, 2, 2).alu64("add", 6, "r3")
    a.ldx(4, 3, 2, 4).alu64("add", 6, "r3")
    a.ldx(8, 3, 2, 8).alu64("add", 6, "r3")
    a.ld_map_value(4, fd, 16)
    a.ldx(4, 3, 4, 4).alu64("add", 6, "r3")
    return a.mov64(0, "r6").exit().assemble()


def test_rodata_loads(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 32, 1)], po, dev)
    val = struct.pack("<BBHIQIIQ", 0, 0xA5, 0xBEEF, 0x12345678, 0x1122334455667788, 9, 0xCAFE, 0)
    om.update(b"\0" * 4, val)
    dm.update(b"\0" * 4, val)
    code = _reader(dm.fd)
    n = 1 << 16
    units = np.random.default_rng(1).integers(0, 255, size=(n, 64), dtype=np.uint8)
    v = po.OracleVM()
    v.load(code)
    want = v.run_raw(units.copy(), 64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    r = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 64, fixed_len=64, rets=r) == 0
    assert (r.download(np.uint64) == want).all()
    # a host update reaches the next launch
    val2 = val[:1] + b"\x5a" + val[2:]
    om.update(b"\0" * 4, val2)
    dm.update(b"\0" * 4, val2)
    want = v.run_raw(units.copy(), 64)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 64, fixed_len=64, rets=r) == 0
    assert (r.download(np.uint64) == want).all()


def test_written_location_keeps_vector_loads(fresh_oracle, fresh_runtime):
    """r0 = *c; *c += 1 through the same constant address: in an ORDERED
    batch unit i reads i (a scalar-cache load would read 0 every time)."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 1)], po, dev)
    code = (Asm().ld_map_value(2, dm.fd, 0).ldx(8, 0, 2, 0).mov64(3, "r0").add64(3, 1).stx(8, 2, 0, "r3")
            .exit().assemble())
    n = 4096
    units = np.zeros((n, 16), np.uint8)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    r = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 16, fixed_len=16, rets=r, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED) == 0
    assert (r.download(np.uint64) == np.arange(n, dtype=np.uint64)).all()
    v = po.OracleVM()
    v.load(code)
    v.run_raw(units.copy(), 16)
    assert dm.lookup(b"\0" * 4) == om.lookup(b"\0" * 4)
