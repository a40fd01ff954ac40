"""The oracle's XDP helpers against analytic expectations of
runtime/src/bpf_helper.cpp:713-788 (CPU only; the device is compared with
the oracle in test_gpu_xdp_helpers.py)."""
import numpy as np
import pytest

from bpftime_amd import isa
from bpftime_amd.isa import Asm

STRIDE = 256
EINVAL32 = 2 ** 32 - 22


def _run(po, code, slot, length, head=0, load_bytes=False):
    vm = po.OracleVM()
    if load_bytes:
        vm.register_xdp_load_bytes()
    vm.load(code)
    slots = slot.reshape(1, STRIDE).copy()
    v, off, ln = vm.run_xdp(slots, lens=np.array([length], np.uint32), want_meta=True, head=head)
    return int(v[0]), int(off[0]), int(ln[0]), slots[0]


@pytest.mark.parametrize("off,length,head", [(-20, 64, 0), (-64, 100, 16), (10, 64, 0), (50, 64, 0),
                                             (51, 64, 0), (-8, 64, 8), (-200, 40, 0)])
def test_adjust_head(fresh_oracle, off, length, head):
    slot = (np.arange(STRIDE) * 7 % 251).astype(np.uint8)
    v, doff, ln, out = _run(fresh_oracle, Asm().mov64(2, off).call(44).exit().assemble(), slot, length, head)
    data = head + off
    if data > head + length - 14:
        assert v == EINVAL32 and doff == head and ln == length
        np.testing.assert_array_equal(out, slot)
    elif data < 0:
        # memmove(buffer_start + (buffer_start - data), data, data_end - data); data = buffer_start
        want = slot.copy()
        want[-data:-data + length] = slot[head:head + length]
        assert v == 0 and doff == 0 and ln == length + head
        np.testing.assert_array_equal(out, want)
    else:
        assert v == 0 and doff == data and ln == length + head - data
        np.testing.assert_array_equal(out, slot)


@pytest.mark.parametrize("delta,length,head", [(-10, 64, 0), (-64, 64, 0), (-65, 64, 0), (192, 64, 0),
                                               (193, 64, 0), (-49, 32, 16)])
def test_adjust_tail(fresh_oracle, delta, length, head):
    v, doff, ln, _ = _run(fresh_oracle, Asm().mov64(2, delta).call(65).exit().assemble(),
                          np.zeros(STRIDE, np.uint8), length, head)
    end = head + length + delta
    ok = head <= end <= STRIDE
    assert v == (0 if ok else EINVAL32) and ln == (length + delta if ok else length) and doff == head


@pytest.mark.parametrize("fsz,tsz", [(4, 8), (3, 8), (8, 6), (0, 0), (28, 28)])
def test_csum_diff(fresh_oracle, fsz, tsz):
    a = Asm().ldx(8, 6, 1, 0).mov64(1, "r6").mov64(2, fsz).mov64(3, "r6").add64(3, 32)
    a.mov64(4, tsz).mov64(5, 0x1234).call(28).exit()
    slot = (np.arange(STRIDE) * 13 % 256).astype(np.uint8)
    v, _, _, _ = _run(fresh_oracle, a.assemble(), slot, 128)
    if fsz % 4 or tsz % 4:
        assert v == EINVAL32
    else:
        w = slot.view(np.uint16)
        assert v == 0x1234 + int(w[16:16 + tsz // 2].sum()) + int((0xFFFF - w[:fsz // 2]).sum())


@pytest.mark.parametrize("off,ln", [(0, 8), (56, 8), (57, 8), (64, 0), (65, 0)])
def test_xdp_load_bytes(fresh_oracle, off, ln):
    a = Asm().st(8, 10, -8, 0).mov64(2, off).mov64(3, "r10").add64(3, -8).mov64(4, ln).call(189)
    a.alu64("and", 0, 0xFF).ldx(4, 1, 10, -8).alu64("lsh", 1, 8).alu64("or", 0, "r1").exit()
    slot = (np.arange(STRIDE) + 1).astype(np.uint8)
    v, _, _, _ = _run(fresh_oracle, a.assemble(), slot, 64, load_bytes=True)
    if off + ln > 64:
        assert v & 0xFF == 0xEA and v >> 8 == 0
    else:
        got = bytes(slot[off:off + min(ln, 4)]) + bytes(4)
        assert v & 0xFF == 0 and v >> 8 == int.from_bytes(got[:4], "little") & 0xFFFFFF


def test_load_bytes_not_in_default_group(fresh_oracle):
    """bpf_helper.cpp:778 defines bpf_xdp_load_bytes but no default group
    registers it: loading a program that calls it fails."""
    rc, msg = fresh_oracle.OracleVM().try_load(Asm().call(189).exit().assemble())
    assert rc < 0 and msg == "invalid call immediate at PC 0"  # compat_ubpf.cpp:83-94
