"""Lane groups of a hash-table XDP launch (k_interp G, interp.hip `groups`):
divergent lanes insert into a HASH map (lookup miss -> update NOEXIST ->
lookup, the lookup_or_try_init idiom of syscount maps.bpf.h:10-38), call a
helper the asm tier does not run (bpf_csum_diff, helper 28: C++ with other
groups pending) or add a counter, and meet again at exit.  Run with lane
groups scheduled through the asm tier (default), with the C++ divergent
loop (BPFTIME_AMD_DBG=4) and with the asm's own groups off
(BPFTIME_AMD_NO_ASM_DIVERGENCE): verdicts and every map element bit-exact
against the oracle."""
import struct

import numpy as np
import pytest

from bpftime_amd import isa
from bpftime_amd.isa import ATOMIC_ADD, Asm

from _helpers import make_maps

pytestmark = pytest.mark.gpu


def _program(fd: int) -> bytes:
    a = Asm()
    a.ldx(8, 2, 1, 0).ldx(8, 3, 1, 8)
    a.mov64(0, isa.XDP_PASS)
    a.mov64(4, "r2").add64(4, 16).jmp("jgt", 4, "r3", "out")
    a.ldx(1, 7, 2, 0)                             # r7 = selector byte
    a.ldx(4, 8, 2, 4).alu64("and", 8, 255)        # 256 keys
    a.stx(4, 10, -4, "r8")
    a.stx(8, 10, -16, "r2")                       # data, across the calls
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.jmp("jne", 0, 0, "have")
    a.st(8, 10, -32, 0).st(8, 10, -24, 0)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -32)
    a.mov64(4, isa.BPF_NOEXIST).call(isa.BPF_FUNC_map_update_elem)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.mov64(1, "r0").mov64(0, isa.XDP_ABORTED).jmp("jeq", 1, 0, "out").mov64(0, "r1")
    a.label("have")
    a.mov64(9, "r0")
    a.alu64("and", 7, 3)
    a.jmp("jeq", 7, 0, "csum")
    a.jmp("jeq", 7, 1, "cnt")
    a.mov64(0, isa.XDP_PASS).ja("out")
    a.label("csum")                               # C++ helper, other groups pending
    a.ldx(8, 3, 10, -16).add64(3, 8)
    a.mov64(1, 0).mov64(2, 0).mov64(4, 4).mov64(5, 0).call(isa.BPF_FUNC_csum_diff)
    a.atomic(8, ATOMIC_ADD, 9, 0, "r0")
    a.mov64(0, isa.XDP_TX).ja("out")
    a.label("cnt")
    a.mov64(1, 1).atomic(8, ATOMIC_ADD, 9, 8, "r1")
    a.mov64(0, isa.XDP_DROP)
    a.label("out").exit()
    return a.assemble()


@pytest.mark.parametrize("mode", ["asm-groups", "cpp-divergent", "no-asm-divergence"])
@pytest.mark.parametrize("n", [4096, 1 << 17])
def test_hash_xdp_lane_groups(fresh_oracle, fresh_runtime, monkeypatch, mode, n):
    if mode == "cpp-divergent":
        monkeypatch.setenv("BPFTIME_AMD_DBG", "4")
    elif mode == "no-asm-divergence":
        monkeypatch.setenv("BPFTIME_AMD_NO_ASM_DIVERGENCE", "1")
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 4, 16, 256)], po, dev)
    code = _program(dm.fd)
    rng = np.random.default_rng(n)
    slots = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    ovm = po.OracleVM()
    ovm.load(code)
    ov = ovm.run_xdp(slots.copy(), fixed_len=64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    got, want = dm.hash_items(), om.items()
    assert len(want) == 256 and got == want
    # every selector class took its path
    sel = slots[:, 0] & 3
    assert sum(struct.unpack("<QQ", v)[1] for v in want.values()) == int((sel == 1).sum())
