"""XDP helpers on the device vs the oracle: bpf_xdp_adjust_head (44),
bpf_xdp_adjust_tail (65), bpf_csum_diff (28) and bpf_xdp_load_bytes (189)
(runtime/src/bpf_helper.cpp:713-788), with the batch outputs data_off_out /
len_out.  Bit-exact on verdicts, packet bytes (the adjust_head memmove
included), returned codes and the out arrays."""
import numpy as np
import pytest

from bpftime_amd import gen, isa
from bpftime_amd.isa import Asm

pytestmark = pytest.mark.gpu

STRIDE = 256


def _sext8(a, r):
    return a.alu64("lsh", r, 56).alu64("arsh", r, 56)


def helper_mix_program() -> bytes:
    """Per packet: adjust_head(ctx, (s8)b[20]); adjust_tail(ctx, (s8)b[21]);
    csum_diff(data, b[22] & 31, data + 8, b[23] & 28, u32 b[24..27]) when
    40 bytes remain; xdp_load_bytes(ctx, b[25] & 63, fp-96, b[26] & 31);
    r0 packs the four results and the first loaded word."""
    a = Asm().mov64(6, "r1")
    a.ldx(8, 2, 6, 0).ldx(8, 3, 6, 8).mov64(4, "r2").add64(4, 32).mov64(0, 1).jmp("jgt", 4, "r3", "out")
    a.ldx(1, 7, 2, 20)
    _sext8(a, 7)
    a.ldx(1, 8, 2, 21)
    _sext8(a, 8)
    a.ldx(1, 9, 2, 22).stx(8, 10, -8, "r9")        # csum sizes byte
    a.ldx(1, 9, 2, 23).stx(8, 10, -16, "r9")
    a.ldx(4, 9, 2, 24).stx(8, 10, -24, "r9")       # seed
    a.ldx(1, 9, 2, 25).stx(8, 10, -32, "r9")       # load_bytes offset
    a.ldx(1, 9, 2, 26).stx(8, 10, -40, "r9")       # load_bytes len
    for off in (-96, -88, -80, -72):
        a.st(8, 10, off, 0)
    a.mov64(1, "r6").mov64(2, "r7").call(isa.BPF_FUNC_xdp_adjust_head).stx(8, 10, -48, "r0")
    a.mov64(1, "r6").mov64(2, "r8").call(isa.BPF_FUNC_xdp_adjust_tail).stx(8, 10, -56, "r0")
    a.mov64(0, 0x55).stx(8, 10, -64, "r0")
    a.ldx(8, 2, 6, 0).ldx(8, 3, 6, 8).mov64(4, "r2").add64(4, 40).jmp("jgt", 4, "r3", "nocsum")
    a.mov64(1, "r2").ldx(8, 2, 10, -8).alu64("and", 2, 31)
    a.mov64(3, "r1").add64(3, 8).ldx(8, 4, 10, -16).alu64("and", 4, 28)
    a.ldx(8, 5, 10, -24).call(isa.BPF_FUNC_csum_diff).stx(8, 10, -64, "r0")
    a.label("nocsum")
    a.mov64(1, "r6").ldx(8, 2, 10, -32).alu64("and", 2, 63).mov64(3, "r10").add64(3, -96)
    a.ldx(8, 4, 10, -40).alu64("and", 4, 31).call(isa.BPF_FUNC_xdp_load_bytes)
    # the loaded bytes land at buffer_start + 224 .. 255 (ctx->buffer_start)
    a.ldx(8, 2, 6, 32)
    for k in range(4):
        a.ldx(8, 1, 10, -96 + 8 * k).stx(8, 2, 224 + 8 * k, "r1")
    # r0 = rc4 & 0xf | (rc1 & 0xf) << 4 | (rc2 & 0xf) << 8 | (csum & 0xffff) << 12
    a.alu64("and", 0, 0xF)
    a.ldx(8, 1, 10, -48).alu64("and", 1, 0xF).alu64("lsh", 1, 4).alu64("or", 0, "r1")
    a.ldx(8, 1, 10, -56).alu64("and", 1, 0xF).alu64("lsh", 1, 8).alu64("or", 0, "r1")
    a.ldx(8, 1, 10, -64).alu64("and", 1, 0xFFFF).alu64("lsh", 1, 12).alu64("or", 0, "r1")
    a.label("out").exit()
    return a.assemble()


def _frames(n, seed, head):
    """Random bytes in 256-B slots, lengths 32..120 (+ head <= 128): the
    adjust_head memmove of at most 128 + 120 bytes stays inside the slot's
    first 248 bytes; the program stores what it loads at 224..255 (the same
    on both sides, in its own slot)."""
    slots = gen.sm64(seed, np.arange(n * STRIDE // 8, dtype=np.uint64)).view(np.uint8).reshape(n, STRIDE).copy()
    lens = (32 + gen.sm64(seed ^ 0x77, np.arange(n, dtype=np.uint64)) % np.uint64(89)).astype(np.uint32)
    return slots, lens


def _run_both(po, dev, code, slots, lens, head, flags):
    n = slots.shape[0]
    ovm = po.OracleVM()
    ovm.register_xdp_load_bytes()
    ovm.load(code)
    oslots = slots.copy()
    ov, ooff, olen = ovm.run_xdp(oslots, lens=lens, want_meta=True, head=head)
    vm = dev.VM()
    assert vm.register(isa.BPF_FUNC_xdp_load_bytes, "bpf_xdp_load_bytes") == 0
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens)
    dv, doff, dln = dev.DeviceBuffer(4 * n), dev.DeviceBuffer(4 * n), dev.DeviceBuffer(4 * n)
    failed = vm.exec_batch(dev.CTX_XDP, d, n, STRIDE, lens=dl, verdicts=dv, data_off_out=doff, len_out=dln,
                           head=head, flags=flags)
    return (ov, oslots, ooff, olen), (dv.download(np.uint32), d.download().reshape(n, STRIDE),
                                      doff.download(np.int32), dln.download(np.uint32)), failed


@pytest.mark.parametrize("head", [0, 32, 128])
@pytest.mark.parametrize("n", [1, 257, 20000])
@pytest.mark.parametrize("ordered", [False, True])
def test_xdp_helper_mix_matches_oracle(fresh_oracle, fresh_runtime, head, n, ordered):
    po, dev = fresh_oracle, fresh_runtime
    if ordered and n > 257:
        pytest.skip("ordered: small batches")
    slots, lens = _frames(n, 0xA11CE + head + n, head)
    code = helper_mix_program()
    (ov, os_, ooff, olen), (dv, ds, doff, dln), failed = _run_both(
        po, dev, code, slots, lens, head, dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0))
    assert failed == 0
    np.testing.assert_array_equal(dv, ov)
    np.testing.assert_array_equal(doff, ooff)
    np.testing.assert_array_equal(dln, olen)
    np.testing.assert_array_equal(ds, os_)
    if n >= 20000:
        # every branch of the helpers ran: -EINVAL and success for each, the
        # memmove branch of adjust_head (data below buffer_start) when head < 128
        rc_head, rc_tail = (ov >> 4) & 0xF, (ov >> 8) & 0xF
        assert set(np.unique(rc_head)) >= {0, 0xA} and set(np.unique(rc_tail)) >= {0, 0xA}
        assert ((ov & 0xF) == 0).any() and ((ov & 0xF) == 0xA).any()
        if head < 128:
            assert (ooff == 0).any() and ((ooff == 0) & (rc_head == 0)).sum() > 0


def _one(po, dev, prog, slot, length, head=0):
    slots = slot.reshape(1, STRIDE).copy()
    lens = np.array([length], dtype=np.uint32)
    return _run_both(po, dev, prog, slots, lens, head, dev.BATCH_SYNC)


@pytest.mark.parametrize("off,length,head", [(-20, 64, 0), (-64, 100, 16), (10, 64, 0), (50, 64, 0),
                                             (51, 64, 0), (-8, 64, 8), (-200, 40, 0), (200, 64, 0)])
def test_adjust_head_cases(fresh_oracle, fresh_runtime, off, length, head):
    """bpf_helper.cpp:748-764: data > data_end - 14 or > buffer_end ->
    -EINVAL; data < buffer_start -> memmove to buffer_start + (buffer_start -
    data) and data = buffer_start; else data moves."""
    po, dev = fresh_oracle, fresh_runtime
    code = Asm().mov64(2, off).call(isa.BPF_FUNC_xdp_adjust_head).exit().assemble()
    slot = (np.arange(STRIDE) * 7 % 251).astype(np.uint8)
    (ov, os_, ooff, olen), (dv, ds, doff, dln), failed = _one(po, dev, code, slot, length, head)
    assert failed == 0
    assert (dv == ov).all() and (doff == ooff).all() and (dln == olen).all()
    np.testing.assert_array_equal(ds, os_)
    data = head + off
    if data > head + length - 14 or data > STRIDE:
        assert dv[0] == (2 ** 32 - 22)
    else:
        assert dv[0] == 0 and doff[0] == max(data, 0)


@pytest.mark.parametrize("delta,length,head", [(-10, 64, 0), (-64, 64, 0), (-65, 64, 0), (100, 64, 0),
                                               (192, 64, 0), (193, 64, 0), (-40, 32, 16), (-49, 32, 16)])
def test_adjust_tail_cases(fresh_oracle, fresh_runtime, delta, length, head):
    """bpf_helper.cpp:766-776: data_end + delta below data / buffer_start or
    above buffer_end -> -EINVAL."""
    po, dev = fresh_oracle, fresh_runtime
    code = Asm().mov64(2, delta).call(isa.BPF_FUNC_xdp_adjust_tail).exit().assemble()
    slot = np.zeros(STRIDE, dtype=np.uint8)
    (ov, _, ooff, olen), (dv, _, doff, dln), failed = _one(po, dev, code, slot, length, head)
    assert failed == 0 and (dv == ov).all() and (dln == olen).all() and (doff == ooff).all()
    end = head + length + delta
    ok = head <= end <= STRIDE
    assert dv[0] == (0 if ok else 2 ** 32 - 22)
    assert dln[0] == (length + delta if ok else length)


@pytest.mark.parametrize("fsz,tsz,null_from,null_to", [(4, 8, False, False), (3, 8, False, False),
                                                       (8, 6, False, False), (0, 0, False, False),
                                                       (16, 16, True, False), (16, 16, False, True),
                                                       (28, 28, False, False)])
def test_csum_diff_cases(fresh_oracle, fresh_runtime, fsz, tsz, null_from, null_to):
    """bpf_helper.cpp:713-744: sizes not multiples of 4 -> -EINVAL; a NULL
    buffer contributes nothing; from words are complemented."""
    po, dev = fresh_oracle, fresh_runtime
    a = Asm().ldx(8, 6, 1, 0)
    a.mov64(1, 0) if null_from else a.mov64(1, "r6")
    a.mov64(2, fsz)
    a.mov64(3, 0) if null_to else a.mov64(3, "r6").add64(3, 32)
    a.mov64(4, tsz).mov64(5, 0x1234).call(isa.BPF_FUNC_csum_diff).exit()
    slot = (np.arange(STRIDE) * 13 % 256).astype(np.uint8)
    (ov, _, _, _), (dv, _, _, _), failed = _one(po, dev, a.assemble(), slot, 128)
    assert failed == 0 and (dv == ov).all()
    if fsz % 4 or tsz % 4:
        assert dv[0] == 2 ** 32 - 22
    else:
        w = slot.view(np.uint16)
        want = 0x1234 + (0 if null_to else int(w[16:16 + tsz // 2].sum())) + \
            (0 if null_from else int((0xFFFF - w[:fsz // 2]).sum()))
        assert dv[0] == want


@pytest.mark.parametrize("off,ln", [(0, 8), (56, 8), (57, 8), (60, 4), (61, 4), (0, 0), (64, 0), (65, 0)])
def test_xdp_load_bytes_cases(fresh_oracle, fresh_runtime, off, ln):
    """bpf_helper.cpp:778-788: data + off + len > data_end -> -EINVAL, else
    a copy into the buffer (64-B packet)."""
    po, dev = fresh_oracle, fresh_runtime
    a = Asm().mov64(6, "r1").st(8, 10, -8, 0).mov64(2, off).mov64(3, "r10").add64(3, -8).mov64(4, ln)
    a.call(isa.BPF_FUNC_xdp_load_bytes).alu64("and", 0, 0xFF)
    a.ldx(4, 1, 10, -8).alu64("lsh", 1, 8).alu64("or", 0, "r1").exit()
    slot = (np.arange(STRIDE) + 1).astype(np.uint8)
    (ov, _, _, _), (dv, _, _, _), failed = _one(po, dev, a.assemble(), slot, 64)
    assert failed == 0 and (dv == ov).all()
