"""Device parity tests: the HIP interpreter (through the C ABI in
libbpftime_amd.so) against the CPU oracle on the same seeded inputs.
Bit-exact for verdicts / r0, packet bytes and map contents."""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs
from bpftime_amd.isa import Asm

from _helpers import make_maps, u64s, xdp_counter_maps

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def run_xdp_both(po, dev, code, slots, lens=None, fixed_len=64, ncpu=0, flags=None):
    """Runs `code` as XDP over `slots` on oracle and device; returns
    (oracle verdicts, oracle slots, device verdicts, device slots, failed)."""
    n, stride = slots.shape
    ovm = po.OracleVM()
    ovm.load(code)
    oslots = slots.copy()
    ov = ovm.run_xdp(oslots, lens=lens, fixed_len=fixed_len, ncpu=ncpu)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens) if lens is not None else None
    dv = dev.DeviceBuffer(4 * n)
    failed = vm.exec_batch(dev.CTX_XDP, d, n, stride, fixed_len=fixed_len, lens=dl, verdicts=dv,
                           flags=flags if flags is not None else dev.BATCH_SYNC)
    return ov, oslots, dv.download(np.uint32), d.download().reshape(n, stride), failed, vm


@pytest.mark.parametrize("n", [1, 63, 4096, 100003])
def test_xdp_counter_parity(fresh_oracle, fresh_runtime, n):
    po, dev = fresh_oracle, fresh_runtime
    (octl, obss), (dctl, dbss) = xdp_counter_maps(po, dev)
    code = programs.xdp_counter(dctl.fd, dbss.fd)
    slots = gen.xdp_packets(n, seed=gen.SEED_CFG2)
    ov, os_, dv, ds, failed, vm = run_xdp_both(po, dev, code, slots)
    assert failed == 0
    assert vm.info()["fused_rmw"] == 1
    # stack store, bound-map lookup, flag load through the non-null value,
    # constant-address counter, ctx data/data_end, 6 packet loads, 6 stores
    assert vm.fast_specialized(dev.CTX_XDP) == 18
    np.testing.assert_array_equal(dv, ov)
    np.testing.assert_array_equal(ds, os_)
    assert (dv == isa.XDP_TX).all()
    assert dbss.lookup(b"\0\0\0\0") == obss.lookup(b"\0\0\0\0")
    assert u64s(dbss.lookup(b"\0\0\0\0"))[0] == n
    # analytic: MACs swapped, rest untouched
    assert (ds[:, :6] == slots[:, 6:12]).all() and (ds[:, 6:12] == slots[:, :6]).all()
    assert (ds[:, 12:] == slots[:, 12:]).all()


def test_xdp_counter_ctl_flag(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    (octl, obss), (dctl, dbss) = xdp_counter_maps(po, dev, ctl_flag=1)
    code = programs.xdp_counter(dctl.fd, dbss.fd)
    slots = gen.xdp_packets(2000)
    ov, os_, dv, ds, failed, _ = run_xdp_both(po, dev, code, slots)
    assert failed == 0 and (dv == isa.XDP_PASS).all() and (ov == dv).all()
    np.testing.assert_array_equal(ds, slots)
    assert u64s(dbss.lookup(b"\0\0\0\0"))[0] == 0


def test_xdp_counter_config1_pcap(fresh_oracle, fresh_runtime):
    """config 1 frames (990 x 64 B + 10 runts) with per-packet lengths."""
    po, dev = fresh_oracle, fresh_runtime
    (octl, obss), (dctl, dbss) = xdp_counter_maps(po, dev)
    code = programs.xdp_counter(dctl.fd, dbss.fd)
    slots, lens = gen.frames_to_slots(gen.config1_frames(), stride=128)
    ov, os_, dv, ds, failed, _ = run_xdp_both(po, dev, code, slots, lens=lens)
    assert failed == 0
    np.testing.assert_array_equal(dv, ov)
    np.testing.assert_array_equal(ds, os_)
    assert (dv == isa.XDP_TX).sum() == 990 and (dv == isa.XDP_DROP).sum() == 10
    assert u64s(dbss.lookup(b"\0\0\0\0"))[0] == 1000


def _raw_both(po, dev, code, units, length, flags=None):
    n, stride = units.shape
    ovm = po.OracleVM()
    ovm.load(code)
    ou = units.copy()
    orets = ovm.run_raw(ou, length)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    failed = vm.exec_batch(dev.CTX_RAW, d, n, stride, fixed_len=length, rets=dr,
                           flags=flags if flags is not None else dev.BATCH_SYNC)
    return orets, ou, dr.download(np.uint64), d.download().reshape(n, stride), failed


ALU = ["add", "sub", "mul", "or", "and", "xor", "mov", "div", "mod", "lsh", "rsh", "arsh", "neg"]
JMP = ["jeq", "jne", "jgt", "jge", "jlt", "jle", "jset", "jsgt", "jsge", "jslt", "jsle"]


def _operands(n, seed):
    r = gen.sm64(seed, np.arange(2 * n, dtype=np.uint64)).reshape(n, 2)
    # mix in small / boundary values so div-by-zero, shifts >= 32, signs all occur
    small = (r % np.uint64(70)).astype(np.uint64)
    pick = (gen.sm64(seed + 1, np.arange(2 * n, dtype=np.uint64)) % np.uint64(3)).reshape(n, 2)
    r = np.where(pick == 0, small, r)
    r[pick == 1] = r[pick == 1] | np.uint64(0xFFFFFFFF00000000)
    return r


@pytest.mark.parametrize("w32", [False, True])
def test_alu_ops_random(fresh_oracle, fresh_runtime, w32):
    po, dev = fresh_oracle, fresh_runtime
    units = _operands(4096, 11 + w32).view(np.uint8).reshape(4096, 16)
    for op in ALU:
        a = Asm().ldx(8, 0, 1, 0).ldx(8, 2, 1, 8)
        if op == "neg":
            a.neg32(0) if w32 else a.neg64(0)
        else:
            (a.alu32 if w32 else a.alu64)(op, 0, "r2")
        code = a.exit().assemble()
        o, _, d, _, failed = _raw_both(po, dev, code, units, 16)
        assert failed == 0
        np.testing.assert_array_equal(d, o, err_msg=op)
        # immediate forms
        for imm in (0, 1, -1, 31, 33, -0x80000000):
            if op == "neg":
                continue
            code = (Asm().ldx(8, 0, 1, 0).__getattribute__("alu32" if w32 else "alu64")(op, 0, imm)
                    .exit().assemble())
            o, _, d, _, failed = _raw_both(po, dev, code, units[:256], 16)
            assert failed == 0
            np.testing.assert_array_equal(d, o, err_msg=f"{op} imm {imm}")


@pytest.mark.parametrize("w32", [False, True])
def test_jumps_divergent(fresh_oracle, fresh_runtime, w32):
    """Random operands make every conditional branch split the wave."""
    po, dev = fresh_oracle, fresh_runtime
    units = _operands(4096, 21 + w32).view(np.uint8).reshape(4096, 16)
    for op in JMP:
        a = Asm().ldx(8, 3, 1, 0).ldx(8, 4, 1, 8).mov64(0, 7)
        (a.jmp32 if w32 else a.jmp)(op, 3, "r4", "t")
        a.mov64(0, 1).alu64("add", 0, "r3").exit().label("t").mov64(0, 2).alu64("xor", 0, "r4").exit()
        o, _, d, _, failed = _raw_both(po, dev, a.assemble(), units, 16)
        assert failed == 0
        np.testing.assert_array_equal(d, o, err_msg=op)


def test_endian_and_memory(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    units = gen.sm64(5, np.arange(2048 * 4, dtype=np.uint64)).view(np.uint8).reshape(2048, 32)
    a = Asm().ldx(8, 0, 1, 0).mov64(2, "r0").be(2, 16).mov64(3, "r0").be(3, 32).mov64(4, "r0").be(4, 64)
    a.mov64(5, "r0").le(5, 16).add64(2, "r3").add64(2, "r4").add64(2, "r5")
    # unaligned loads / stores of every size into the unit and the stack
    a.ldx(4, 6, 1, 3).ldx(2, 7, 1, 9).ldx(1, 8, 1, 17).stx(4, 1, 21, "r2").stx(8, 10, -13, "r6")
    a.ldx(8, 9, 10, -13).st(2, 1, 27, -2).stx(1, 1, 30, "r8")
    a.mov64(0, "r2").alu64("xor", 0, "r9").add64(0, "r7").exit()
    o, ou, d, du, failed = _raw_both(po, dev, a.assemble(), units, 32)
    assert failed == 0
    np.testing.assert_array_equal(d, o)
    np.testing.assert_array_equal(du, ou)


def test_atomics_per_unit(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    units = gen.sm64(9, np.arange(1024 * 4, dtype=np.uint64)).view(np.uint8).reshape(1024, 32)
    a = Asm().ldx(8, 2, 1, 8).mov64(3, "r2")
    a.atomic(8, isa.ATOMIC_ADD | isa.ATOMIC_FETCH, 1, 0, "r2")
    a.atomic(8, isa.ATOMIC_XOR, 1, 16, "r3")
    a.atomic(4, isa.ATOMIC_OR | isa.ATOMIC_FETCH, 1, 24, "r3")
    a.ldx(8, 0, 1, 0).mov64(4, 5).atomic(8, isa.ATOMIC_CMPXCHG, 1, 16, "r4")
    a.add64(0, "r2").add64(0, "r3").exit()
    o, ou, d, du, failed = _raw_both(po, dev, a.assemble(), units, 32)
    assert failed == 0
    np.testing.assert_array_equal(d, o)
    np.testing.assert_array_equal(du, ou)


def test_divergent_loops_sum(fresh_oracle, fresh_runtime):
    """sum.bpf.o-style loop with a different trip count on every lane."""
    po, dev = fresh_oracle, fresh_runtime
    n = 3000
    rng = np.random.default_rng(4)
    arr = rng.integers(-1000, 1000, size=(n, 64)).astype(np.int32)
    arr[:, 0] = rng.integers(0, 63, size=n)
    units = arr.view(np.uint8).reshape(n, 256)
    o, _, d, _, failed = _raw_both(po, dev, programs.kat_sum(), units, 256)
    assert failed == 0
    np.testing.assert_array_equal(d, o)
    exp = np.array([arr[i, 1:1 + arr[i, 0]].sum() for i in range(n)], dtype=np.int64).view(np.uint64)
    np.testing.assert_array_equal(d, exp)


def _random_program(rng, nins=60):
    """Random straight-line/forward-branch program over r0..r9 + stack."""
    a = Asm()
    a.ldx(8, 6, 1, 0).ldx(8, 7, 1, 8).ldx(8, 8, 1, 16).ldx(8, 9, 1, 24)
    for r in range(6):
        a.mov64(r, "r%d" % (6 + r % 4))
    labels = 0
    pending = []
    for i in range(nins):
        k = rng.integers(0, 10)
        dst = int(rng.integers(0, 10))
        src = "r%d" % int(rng.integers(0, 10))
        if dst == 10:
            continue
        if k < 5:
            op = ALU[int(rng.integers(0, len(ALU)))]
            w32 = bool(rng.integers(0, 2))
            if op == "neg":
                a.neg32(dst) if w32 else a.neg64(dst)
            elif rng.integers(0, 2):
                (a.alu32 if w32 else a.alu64)(op, dst, src)
            else:
                (a.alu32 if w32 else a.alu64)(op, dst, int(rng.integers(-50, 50)))
        elif k < 7:
            off = -8 * int(rng.integers(1, 8))
            a.stx(8, 10, off, src)
            a.ldx([1, 2, 4, 8][int(rng.integers(0, 4))], dst, 10, off + int(rng.integers(0, 8)) // 8 * 0)
        elif k < 9:
            name = f"L{labels}"
            labels += 1
            op = JMP[int(rng.integers(0, len(JMP)))]
            (a.jmp32 if rng.integers(0, 2) else a.jmp)(op, dst, src, name)
            pending.append((name, i + int(rng.integers(1, 8))))
        else:
            a.mov64(dst, int(rng.integers(-1000, 1000)))
        for name, at in list(pending):
            if at <= i:
                a.label(name)
                pending.remove((name, at))
    for name, _ in pending:
        a.label(name)
    a.mov64(0, "r0").alu64("xor", 0, "r1").alu64("add", 0, "r2").alu64("xor", 0, "r3")
    a.alu64("add", 0, "r4").alu64("xor", 0, "r5").exit()
    return a.assemble()


@pytest.mark.parametrize("asm_groups", [True, False])
def test_random_programs(fresh_oracle, fresh_runtime, monkeypatch, asm_groups):
    """Random forward-branch programs: lane groups scheduled inside the asm
    fast path, and (BPFTIME_AMD_NO_ASM_DIVERGENCE) by the C++ loop alone."""
    if not asm_groups:
        monkeypatch.setenv("BPFTIME_AMD_NO_ASM_DIVERGENCE", "1")
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(1234)
    units = _operands(2048, 77).view(np.uint8).reshape(2048, 16)
    units = np.concatenate([units, units[::-1]], axis=1).copy()
    for t in range(40):
        code = _random_program(rng)
        o, _, d, _, failed = _raw_both(po, dev, code, units, 32)
        assert failed == 0, t
        np.testing.assert_array_equal(d, o, err_msg=f"program {t}")


def test_exec_single_kats(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    vm = dev.VM()
    vm.load(programs.kat_add_mem())
    rc, r = vm.exec(bytearray(struct.pack("<II", 40, 2)))
    assert rc == 0 and r == 42
    vm = dev.VM()
    vm.load(programs.kat_mul())
    assert vm.exec(bytearray(8)) == (0, 2)
    arr = [5, 1, -2, 30, 4, -100, 999]
    vm = dev.VM()
    vm.load(programs.kat_sum())
    rc, r = vm.exec(bytearray(struct.pack("<7i", *arr)))
    assert rc == 0 and r == (sum(arr[1:6]) & M64)


def test_oob_access_fails_lane_not_gpu(fresh_oracle, fresh_runtime):
    """A wild pointer fails its lane (verdict 0, like a failed exec) instead
    of faulting the GPU; other lanes are unaffected."""
    dev = fresh_runtime
    a = Asm().ldx(8, 2, 1, 0).jmp("jeq", 2, 0, "ok").lddw(3, 0x1000).ldx(8, 0, 3, 0).exit()
    a.label("ok").mov64(0, 5).exit()
    vm = dev.VM()
    vm.load(a.assemble())
    units = np.zeros((256, 8), dtype=np.uint8)
    units[::2, 0] = 1
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * 256)
    failed = vm.exec_batch(dev.CTX_RAW, d, 256, 8, fixed_len=8, rets=dr)
    r = dr.download(np.uint64)
    assert failed == 128
    assert (r[1::2] == 5).all() and (r[::2] == 0).all()


def test_step_limit_stops_infinite_loop(fresh_runtime):
    dev = fresh_runtime
    vm = dev.VM()
    vm.load(Asm().label("top").add64(0, 1).ja("top").exit().assemble())
    vm.set_step_limit(10000)
    d = dev.DeviceBuffer(64 * 8)
    dr = dev.DeviceBuffer(8 * 64)
    assert vm.exec_batch(dev.CTX_RAW, d, 64, 8, fixed_len=8, rets=dr) == 64


def test_ordered_mode_matches_sequential(fresh_oracle, fresh_runtime):
    """A last-writer-wins program (plain store of packet bytes into a shared
    map value) is order dependent: EBPF_BATCH_ORDERED reproduces the
    reference's sequential result exactly."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 1)], po, dev)
    a = Asm().ldx(8, 6, 1, 0).ld_map_value(2, dm.fd, 0).ldx(8, 3, 2, 0).add64(3, "r6").stx(8, 2, 0, "r3")
    a.mov64(7, "r3").mov64(0, "r7").exit()  # loaded value stays live -> not fused
    code = a.assemble()
    units = gen.sm64(3, np.arange(500, dtype=np.uint64)).view(np.uint8).reshape(500, 8)
    o, _, d, _, failed = _raw_both(po, dev, code, units, 8, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED)
    assert failed == 0
    np.testing.assert_array_equal(d, o)
    assert dm.lookup(b"\0\0\0\0") == om.lookup(b"\0\0\0\0")


def test_load_errors_match_oracle(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    cases = [Asm().call(99).exit().assemble(), Asm().mov64(0, 0).call(60).exit().assemble(),
             Asm().lddw(0, 1, src=3).exit().assemble(), b"\x95" + b"\0" * 6,
             Asm().raw(0xff).exit().assemble(), Asm().ja(5).exit().assemble()]
    for c in cases:
        o_rc, o_msg = po.OracleVM().try_load(c)
        d_rc, d_msg = dev.VM().try_load(c)
        assert (o_rc < 0) == (d_rc < 0) and o_msg == d_msg, (o_msg, d_msg)


@pytest.mark.parametrize("first", [0, 12345])
def test_device_generators_match_numpy(fresh_runtime, first):
    """csrc/gen.hip regenerates gen.py's config-3/5 inputs word for word, so
    full-size device-resident runs use the same inputs as the parity tests."""
    dev = fresh_runtime
    L = dev.lib()
    n = 3000
    cdf = gen.zipf_cdf(65536, 1.1)
    dc = dev.DeviceBuffer.from_array(cdf)
    fb, fl = dev.DeviceBuffer(n * 2048), dev.DeviceBuffer(4 * n)
    assert L.bpftime_amd_gen_flow(fb.ptr, fl.ptr, n, 2048, gen.SEED_CFG3, first, dc.ptr, 65536, None) == 0
    slots, lens = gen.flow_packets(n, first=first)
    np.testing.assert_array_equal(fb.download(np.uint8).reshape(n, 2048), slots)
    np.testing.assert_array_equal(fl.download(np.uint32), lens)
    cdf5 = gen.zipf_cdf(335, 1.2)
    dc5 = dev.DeviceBuffer.from_array(cdf5)
    sb = dev.DeviceBuffer(n * 64)
    assert L.bpftime_amd_gen_syscall(sb.ptr, n, gen.SEED_CFG5, first, dc5.ptr, 335, None) == 0
    np.testing.assert_array_equal(sb.download(np.uint8).reshape(n, 64), gen.syscall_records(n, first=first))


def _staged_mix():
    """Packet / stack / ctx accesses of every size at aligned, unaligned,
    dword-straddling and window-edge offsets, reads after writes, and one
    store the staged path cannot take (straddling) — the fast path's typed
    handlers against the oracle."""
    a = Asm()
    a.mov64(6, "r1").ldx(8, 2, 6, 0).ldx(8, 3, 6, 8)
    a.mov64(4, "r2").add64(4, 64).jmp("jgt", 4, "r3", "short")
    a.mov64(0, 0)
    for sz, off in [(1, 63), (2, 1), (4, 2), (8, 5), (8, 56), (2, 62), (1, 0), (4, 60)]:
        a.ldx(sz, 5, 2, off).alu64("xor", 0, "r5").alu64("lsh", 0, 3).alu64("add", 0, "r5")
    a.stx(1, 2, 7, "r0").stx(2, 2, 3, "r0").stx(4, 2, 8, "r0").stx(8, 2, 16, "r0")
    a.st(4, 2, 40, 0x1234567).st(2, 2, 62, -2).st(1, 2, 33, 7).st(8, 2, 48, -5)
    a.ldx(4, 5, 2, 8).alu64("add", 0, "r5").ldx(2, 5, 2, 3).alu64("add", 0, "r5")
    a.ldx(8, 5, 2, 14).alu64("xor", 0, "r5")
    a.stx(8, 10, -8, "r0").stx(4, 10, -12, "r5").st(1, 10, -13, 9).st(2, 10, -16, 300)
    a.ldx(4, 5, 10, -8).alu64("add", 0, "r5").ldx(1, 5, 10, -13).alu64("add", 0, "r5")
    a.ldx(2, 5, 10, -16).alu64("add", 0, "r5").ldx(8, 5, 10, -16).alu64("xor", 0, "r5")
    a.ldx(4, 5, 6, 20).alu64("add", 0, "r5")          # ifindex: the LDS ctx field load (LDX4_CTX)
    a.alu64("and", 0, 0xffff).exit()
    a.label("short").mov64(0, 1).exit()
    return a.assemble()


@pytest.mark.parametrize("stride,n", [(64, 5000), (128, 3001), (2048, 700)])
def test_staged_typed_accesses(fresh_oracle, fresh_runtime, stride, n):
    po, dev = fresh_oracle, fresh_runtime
    code = _staged_mix()
    slots = gen.xdp_packets(n, stride=stride, seed=77)
    lens = np.full(n, stride, dtype=np.uint32)
    lens[::7] = 40                                     # short units take the other path
    ov, os_, dv, ds, failed, vm = run_xdp_both(po, dev, code, slots, lens=lens, fixed_len=0)
    assert failed == 0
    assert vm.fast_specialized(dev.CTX_XDP) == 30
    np.testing.assert_array_equal(dv, ov)
    np.testing.assert_array_equal(ds, os_)


def test_staged_raw_slot_accesses(fresh_oracle, fresh_runtime):
    """RAW units (r1 = the slot itself): slot-typed accesses read the staged
    copy and see earlier stores."""
    po, dev = fresh_oracle, fresh_runtime
    a = Asm().mov64(0, 0)
    for sz, off in [(8, 0), (4, 12), (2, 30), (1, 63)]:
        a.ldx(sz, 3, 1, off).alu64("add", 0, "r3")
    a.stx(4, 1, 12, "r0").ldx(4, 3, 1, 12).alu64("xor", 0, "r3").stx(8, 1, 40, "r0").exit()
    code = a.assemble()
    n = 4000
    units = gen.xdp_packets(n, stride=64, seed=5)
    ovm = po.OracleVM()
    ovm.load(code)
    ou = units.copy()
    orets = ovm.run_raw(ou, 64)
    vm = dev.VM()
    vm.load(code)
    assert vm.fast_specialized(dev.CTX_RAW) == 7
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 64, fixed_len=64, rets=dr) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), orets)
    np.testing.assert_array_equal(d.download().reshape(n, 64), ou)


def test_atomics_shared_map_and_own_bytes(fresh_oracle, fresh_runtime):
    """Device-scope atomics from every lane onto shared array-map values
    (commutative, so any interleaving gives the oracle's totals), fetch
    forms with the fetched value discarded, and an atomic on the unit's own
    staged bytes (the C++ path, after write-back)."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 16, 4)], po, dev)
    a = Asm()
    a.ldx(8, 6, 1, 0).mov64(7, "r6").alu64("and", 7, 3).stx(4, 10, -4, "r7")
    a.mov64(9, "r1").ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).call(1)
    a.jmp("jeq", 0, 0, "out")
    a.atomic(8, isa.ATOMIC_ADD, 0, 0, "r6")
    a.mov64(8, "r6").atomic(8, isa.ATOMIC_ADD | isa.ATOMIC_FETCH, 0, 0, "r8")
    a.mov64(8, "r6").atomic(4, isa.ATOMIC_XOR, 0, 8, "r8")
    a.mov64(8, "r6").atomic(4, isa.ATOMIC_OR | isa.ATOMIC_FETCH, 0, 12, "r8")
    a.stx(8, 9, 16, "r6").atomic(8, isa.ATOMIC_ADD, 9, 16, "r7")   # own staged bytes
    a.label("out").mov64(0, "r7").exit()
    code = a.assemble()
    n = 20000
    units = gen.xdp_packets(n, stride=64, seed=31)
    ovm = po.OracleVM()
    ovm.load(code)
    ou = units.copy()
    orets = ovm.run_raw(ou, 64)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(units)
    dr = dev.DeviceBuffer(8 * n)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 64, fixed_len=64, rets=dr) == 0
    np.testing.assert_array_equal(dr.download(np.uint64), orets)
    np.testing.assert_array_equal(d.download().reshape(n, 64), ou)
    for k in range(4):
        assert dm.lookup(struct.pack("<I", k)) == om.lookup(struct.pack("<I", k)), k


def test_fused_counter_per_lane_addresses(fresh_oracle, fresh_runtime):
    """ldx/add/stx fused counters whose address differs per lane (hash of
    the unit): one atomic per lane in the fast path."""
    po, dev = fresh_oracle, fresh_runtime
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 64)], po, dev)
    a = Asm()
    a.ldx(4, 6, 1, 4).alu64("and", 6, 63).stx(4, 10, -4, "r6")
    a.ld_map_fd(1, dm.fd).mov64(2, "r10").add64(2, -4).call(1)
    a.jmp("jeq", 0, 0, "out")
    a.ldx(8, 1, 0, 0).add64(1, "r6").stx(8, 0, 0, "r1")
    a.label("out").mov64(0, 2).exit()
    code = a.assemble()
    n = 30000
    units = gen.xdp_packets(n, stride=64, seed=32)
    ovm = po.OracleVM()
    ovm.load(code)
    ovm.run_raw(units.copy(), 64)
    vm = dev.VM()
    vm.load(code)
    assert vm.info()["fused_rmw"] == 1
    d = dev.DeviceBuffer.from_array(units)
    assert vm.exec_batch(dev.CTX_RAW, d, n, 64, fixed_len=64) == 0
    for k in range(64):
        assert dm.lookup(struct.pack("<I", k)) == om.lookup(struct.pack("<I", k)), k


@pytest.mark.parametrize("asm_groups", [True, False])
def test_ctx_reads_after_divergence(fresh_oracle, fresh_runtime, monkeypatch, asm_groups):
    """ctx->data / data_end read only after lanes split (the loader keeps the
    ctx out of LDS when every ctx read is a specialised data / data_end
    load): the C++ tier must see the same values as the asm tier."""
    if not asm_groups:
        monkeypatch.setenv("BPFTIME_AMD_NO_ASM_DIVERGENCE", "1")
    po, dev = fresh_oracle, fresh_runtime
    a = Asm().mov64(6, "r1").ldx(8, 2, 1, 0).ldx(1, 3, 2, 0)
    for k in range(5):                         # up to six lane groups
        a.jmp("jeq", 3, k, f"g{k}")
    a.mov64(0, 9).ja("tail")
    for k in range(5):
        a.label(f"g{k}").mov64(0, k).ja("tail")
    a.label("tail")
    a.ldx(8, 2, 6, 0).ldx(8, 4, 6, 8)          # ctx->data, ctx->data_end again
    a.alu64("sub", 4, "r2").alu64("lsh", 4, 8).alu64("or", 0, "r4")
    a.ldx(1, 5, 2, 1).alu64("lsh", 5, 16).alu64("or", 0, "r5").exit()
    code = a.assemble()
    n = 4096
    pk = gen.xdp_packets(n, seed=77)
    pk[:, 0] %= 7
    lens = (np.arange(n) % 50 + 14).astype(np.uint32)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), lens=lens)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, lens=dl, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), want)


@pytest.mark.parametrize("asm_groups", [True, False])
def test_ctx_reads_inside_divergent_groups(fresh_oracle, fresh_runtime, monkeypatch, asm_groups):
    """ctx->data read inside each of six lane groups (before they
    reconverge), so the C++ tier executes ctx loads itself."""
    if not asm_groups:
        monkeypatch.setenv("BPFTIME_AMD_NO_ASM_DIVERGENCE", "1")
    po, dev = fresh_oracle, fresh_runtime
    a = Asm().mov64(6, "r1").ldx(8, 2, 1, 0).ldx(1, 3, 2, 0)
    for k in range(5):
        a.jmp("jeq", 3, k, f"g{k}")
    a.mov64(0, 9).ja("tail")
    for k in range(5):
        a.label(f"g{k}").ldx(8, 2, 6, 0).ldx(8, 4, 6, 8).alu64("sub", 4, "r2")
        a.ldx(1, 5, 2, k + 1).alu64("lsh", 5, 8).alu64("or", 5, "r4").mov64(0, "r5").add64(0, k).ja("tail")
    a.label("tail").exit()
    code = a.assemble()
    n = 4096
    pk = gen.xdp_packets(n, seed=78)
    pk[:, 0] %= 7
    lens = (np.arange(n) % 50 + 14).astype(np.uint32)
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(pk.copy(), lens=lens)
    vm = dev.VM()
    vm.load(code)
    d = dev.DeviceBuffer.from_array(pk)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, lens=dl, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), want)


def _random_xdp_program(rng, map_fd, nins=50):
    """Random XDP program of the shapes a verifier accepts: scalars in
    r0-r5, r6 = ctx, r7 / r8 = data / data_end (re-read from the ctx at
    random points), 64 B bounds-checked once, packet loads / stores at
    constant offsets, stack traffic, forward branches on scalars, and
    array-map counters (lookup + fused add)."""
    a = Asm().mov64(6, "r1").ldx(8, 7, 1, 0).ldx(8, 8, 1, 8)
    a.mov64(9, "r7").add64(9, 64).mov64(0, 1).jmp("jgt", 9, "r8", "out")
    for r in range(6):
        a.mov64(r, int(rng.integers(-100, 100)))
    labels, pending = 0, []
    for i in range(nins):
        k = int(rng.integers(0, 12))
        dst = int(rng.integers(0, 6))
        src = "r%d" % int(rng.integers(0, 6))
        if k < 3:
            op = ["add", "sub", "xor", "or", "and", "lsh", "rsh", "mul"][int(rng.integers(0, 8))]
            v = src if rng.integers(0, 2) else int(rng.integers(0, 31))
            (a.alu32 if rng.integers(0, 2) else a.alu64)(op, dst, v)
        elif k < 5:
            sz = [1, 2, 4, 8][int(rng.integers(0, 4))]
            a.ldx(sz, dst, 7, int(rng.integers(0, 64 - sz + 1)))
        elif k < 6:
            sz = [1, 2, 4, 8][int(rng.integers(0, 4))]
            a.stx(sz, 7, int(rng.integers(0, 64 - sz + 1)), src)
        elif k < 7:
            a.ldx(8, 7, 6, 0) if rng.integers(0, 2) else a.ldx(8, 8, 6, 8)
        elif k < 8:
            off = -8 * int(rng.integers(1, 6))
            a.stx(8, 10, off, src).ldx(8, dst, 10, off)
        elif k < 10:
            name = f"L{labels}"
            labels += 1
            op = JMP[int(rng.integers(0, len(JMP)))]
            v = src if rng.integers(0, 2) else int(rng.integers(-5, 5))
            (a.jmp32 if rng.integers(0, 2) else a.jmp)(op, dst, v, name)
            pending.append((name, i + int(rng.integers(1, 6))))
        else:
            # counters[(dst & 3)] += 1 (lookup_elem, fused ldx / add / stx)
            skip = f"M{labels}"
            labels += 1
            a.mov64(9, f"r{dst}").alu64("and", 9, 3).stx(4, 10, -48, "r9")
            a.ld_map_fd(1, map_fd).mov64(2, "r10").add64(2, -48).call(1)
            a.jmp("jeq", 0, 0, skip).ldx(8, 1, 0, 0).add64(1, int(rng.integers(1, 9))).stx(8, 0, 0, "r1")
            a.label(skip)
            for r in range(6):
                a.mov64(r, int(rng.integers(-100, 100)))
        for name, at in list(pending):
            if at <= i:
                a.label(name)
                pending.remove((name, at))
    for name, _ in pending:
        a.label(name)
    a.alu64("xor", 0, "r1").alu64("add", 0, "r2").alu64("xor", 0, "r3").alu64("add", 0, "r4")
    a.alu64("xor", 0, "r5").ldx(8, 2, 6, 8).ldx(8, 3, 6, 0).alu64("sub", 2, "r3").alu64("add", 0, "r2")
    a.label("out").exit()
    return a.assemble()


@pytest.mark.parametrize("asm_groups", [True, False])
def test_random_xdp_programs(fresh_oracle, fresh_runtime, monkeypatch, asm_groups):
    """Random verifier-shaped XDP programs: verdicts, packet bytes and map
    counters bit-exact against the oracle, with lane groups in asm and in
    the C++ tier."""
    if not asm_groups:
        monkeypatch.setenv("BPFTIME_AMD_NO_ASM_DIVERGENCE", "1")
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(2024)
    n = 2048
    for t in range(64):
        po.reset()
        dev.reset_runtime()
        (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)], po, dev)
        code = _random_xdp_program(rng, dm.fd)
        pk = gen.xdp_packets(n, seed=100 + t)
        lens = np.where(np.arange(n) % 13 == 0, 40, 64).astype(np.uint32)
        ovm = po.OracleVM()
        ovm.load(code)
        opk = pk.copy()
        want = ovm.run_xdp(opk, lens=lens)
        vm = dev.VM()
        vm.load(code)
        d = dev.DeviceBuffer.from_array(pk)
        dl = dev.DeviceBuffer.from_array(lens)
        dv = dev.DeviceBuffer(4 * n)
        assert vm.exec_batch(dev.CTX_XDP, d, n, 64, lens=dl, verdicts=dv) == 0, t
        np.testing.assert_array_equal(dv.download(np.uint32), want, err_msg=f"program {t}")
        np.testing.assert_array_equal(d.download().reshape(n, 64), opk, err_msg=f"program {t}")
        for k in range(4):
            key = struct.pack("<I", k)
            assert dm.lookup(key) == om.lookup(key), (t, k)


def test_random_programs_unfused(fresh_oracle, fresh_runtime, monkeypatch):
    """The same random programs with the loader's superinstructions off
    (loader.cpp fuse_pairs: `mov; add` and `mov imm; jump / exit` pairs run
    as two dispatches): the fused and unfused forms both match the oracle."""
    monkeypatch.setenv("BPFTIME_AMD_NO_FUSE", "1")
    test_random_xdp_programs(fresh_oracle, fresh_runtime, monkeypatch, True)
    test_random_programs(fresh_oracle, fresh_runtime, monkeypatch, True)
