"""Random sys_enter / sys_exit program pairs that pass state from one to the
other, through the thread-ordered dispatch (csrc/vm_api.cpp seq_dispatch,
interp.hip k_sys_seq) in both of its tiers -- the asm tier (LDS stacks,
caller / clock beside the ctx copy, lane groups in asm) and the C++ tier
(BPFTIME_AMD_SEQ_ASM=0) -- against the oracle's record-by-record
dispatch_syscall (attach/syscall_trace_attach_impl/src/
syscall_trace_attach_impl.cpp:18-95; oracle/drivers.c orc_sys_dispatch):
every map and every return bit-exact.

Each enter program computes a value from the call's arguments, its caller
and its recorded clock through random ALU operations and forward branches,
stores it in start[tid] (HASH) and, for some pairs, in an ARRAY slot at a
constant address; each exit program reads both back (the ARRAY slot
through the constant-address load the loader would send through the scalar
cache, were no other program writing it), mixes them with the return value
and adds the result into per-bucket counters (an ARRAY, BPF_ATOMIC add).
The pairs that share the ARRAY slot across threads run EBPF_BATCH_ORDERED
(the serial run): between threads the reference fixes no order."""
import numpy as np
import pytest

from bpftime_amd import gen, isa
from bpftime_amd.isa import Asm

from _helpers import make_maps

pytestmark = pytest.mark.gpu

TRACEPOINT = 5
HASH, ARRAY = isa.BPF_MAP_TYPE_HASH, isa.BPF_MAP_TYPE_ARRAY
ALU = ["add", "sub", "mul", "or", "and", "xor", "lsh", "rsh", "arsh"]
JMP = ["jeq", "jne", "jgt", "jge", "jlt", "jle", "jsgt", "jsge", "jslt", "jsle", "jset"]


def _mix(a, rng, n):
    """n random ALU / forward-branch instructions over r0..r5."""
    pending, labels = [], 0
    for i in range(n):
        k = int(rng.integers(0, 10))
        dst = int(rng.integers(0, 6))
        src = "r%d" % int(rng.integers(0, 6))
        if k < 6:
            op = ALU[int(rng.integers(0, len(ALU)))]
            alu = a.alu32 if rng.integers(0, 2) else a.alu64
            if op in ("lsh", "rsh", "arsh") or rng.integers(0, 2):
                alu(op, dst, int(rng.integers(0, 31)) if op in ("lsh", "rsh", "arsh") else int(rng.integers(-99, 99)))
            else:
                alu(op, dst, src)
        elif k < 9:
            name = "L%d" % labels
            labels += 1
            (a.jmp32 if rng.integers(0, 2) else a.jmp)(JMP[int(rng.integers(0, len(JMP)))], dst, src, name)
            pending.append((name, i + int(rng.integers(1, 6))))
        else:
            a.mov64(dst, int(rng.integers(-1000, 1000)))
        for name, at in list(pending):
            if at <= i:
                a.label(name)
                pending.remove((name, at))
    for name, _ in pending:
        a.label(name)


def _pair(rng, start_fd, arr_fd, acc_fd, use_arr):
    slot = 8 * int(rng.integers(0, 4))
    e = Asm()
    e.mov64(6, "r1")
    e.call(isa.BPF_FUNC_get_current_pid_tgid).mov64(7, "r0").stx(4, 10, -4, "r0")
    e.call(isa.BPF_FUNC_ktime_get_ns).mov64(5, "r0")
    e.ldx(8, 0, 6, 16).ldx(8, 1, 6, 24).ldx(8, 2, 6, 32).ldx(8, 3, 6, 40).mov64(4, "r7")
    _mix(e, rng, int(rng.integers(8, 30)))
    e.alu64("xor", 0, "r1").alu64("add", 0, "r2").alu64("xor", 0, "r5")
    e.stx(8, 10, -16, "r0")
    if use_arr:
        e.ld_map_value(8, arr_fd, 0).stx(8, 8, slot, "r0")
    e.ld_map_fd(1, start_fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -16).mov64(4, 0)
    e.call(isa.BPF_FUNC_map_update_elem)
    e.mov64(0, 0).exit()
    x = Asm()
    x.mov64(6, "r1")
    x.call(isa.BPF_FUNC_get_current_pid_tgid).stx(4, 10, -4, "r0").mov64(7, "r0")
    x.ld_map_fd(1, start_fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    x.mov64(9, 0)
    x.jmp("jeq", 0, 0, "nostart")
    x.ldx(8, 9, 0, 0)
    x.label("nostart")
    x.call(isa.BPF_FUNC_ktime_get_ns).mov64(5, "r0")
    x.ldx(8, 1, 6, 16).mov64(0, "r9").mov64(2, "r7").mov64(3, "r9").mov64(4, 3)
    if use_arr:
        x.ld_map_value(8, arr_fd, 0).ldx(8, 4, 8, slot)
    _mix(x, rng, int(rng.integers(8, 30)))
    x.alu64("xor", 0, "r3").alu64("add", 0, "r4").alu64("xor", 0, "r5")
    x.mov64(8, "r0")
    x.mov64(1, "r9").alu64("and", 1, 7).stx(4, 10, -8, "r1")
    x.ld_map_fd(1, acc_fd).mov64(2, "r10").add64(2, -8).call(isa.BPF_FUNC_map_lookup_elem)
    x.jmp("jeq", 0, 0, "out")
    x.atomic(8, isa.ATOMIC_ADD, 0, 0, 8)
    x.mov64(1, 1).atomic(8, isa.ATOMIC_ADD, 0, 8, 1)
    x.label("out").mov64(0, 0).exit()
    return e.assemble(), x.assemble()


@pytest.mark.parametrize("tier", ["asm", "cpp"])
def test_random_state_pairs(fresh_oracle, fresh_runtime, monkeypatch, tier):
    po, dev = fresh_oracle, fresh_runtime
    monkeypatch.setenv("BPFTIME_AMD_SEQ_ASM", "1" if tier == "asm" else "0")
    rng = np.random.default_rng(606)
    n = 1 << 13
    recs = gen.syscall_records_timed(n, threads=96)
    for t in range(12):
        po.reset()
        dev.reset_runtime()
        d = dev.DeviceBuffer.from_array(recs)
        (ostart, oarr, oacc), (dstart, darr, dacc) = make_maps(
            [(HASH, 4, 8, 1024), (ARRAY, 4, 32, 1), (ARRAY, 4, 16, 8)], po, dev)
        enter, exit_ = _pair(rng, dstart.fd, darr.fd, dacc.fd, use_arr=bool(t % 2))
        o = po.OracleSyscallDispatch()
        for code, e in ((enter, True), (exit_, False)):
            dev.syscall_attach(dev.prog_create(code, "p", TRACEPOINT), -1, e)
            o.attach(code, -1, e)
        assert dev.syscall_dispatch_plan() == 1, t
        out = dev.DeviceBuffer(8 * n)
        # the ARRAY slot is shared by every thread: only the serial run
        # (EBPF_BATCH_ORDERED, one lane in record order) has one answer
        flags = dev.BATCH_SYNC | (dev.BATCH_ORDERED if t % 2 else 0)
        assert dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, out=out, flags=flags) == 0, t
        want = o.dispatch(recs)
        assert (out.download(np.int64) == want).all(), t
        assert dstart.hash_items() == ostart.items(), t
        for k in range(8):
            key = k.to_bytes(4, "little")
            assert dacc.lookup(key) == oacc.lookup(key), (t, k)
        assert darr.lookup(b"\0" * 4) == oarr.lookup(b"\0" * 4), t
