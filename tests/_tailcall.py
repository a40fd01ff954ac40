"""Programs for the bpf_tail_call / PROG_ARRAY parity tests (shared by the
oracle KATs and the device tests).  Semantics under test
(runtime/src/bpf_helper.cpp:568-650, the interpreter backend): the target
runs as a nested exec over a 64-B copy of the ctx (r2 = 64), its r0 comes
back to the caller as the helper's result, the caller's registers, stack and
ctx are unchanged, packet bytes written through ctx->data stay written, a
missing slot / non-prog-array map returns -1, and depth stops at 32."""
from bpftime_amd import isa
from bpftime_amd.isa import Asm

TAIL = isa.BPF_FUNC_tail_call
XADD = 0x00  # BPF_ADD atomic


def ref_kat_caller(pa_fd: int, tail_then_exit: bool) -> bytes:
    """runtime/unit-test/tailcall/test_user_to_user_tailcall.cpp caller:
    lddw r2 = the prog array fd as a plain immediate, r3 = 0, call 0x0c.
    With tail_then_exit the program exits with the helper's r0 (the callee's
    0x1234 under both VM backends); otherwise it then returns 0xdead as in
    the reference test body."""
    a = Asm().lddw(2, pa_fd).mov64(3, 0).call(TAIL)
    if not tail_then_exit:
        a.mov64(0, 0xdead)
    return a.exit().assemble()


def ref_kat_target() -> bytes:
    return Asm().mov64(0, 0x1234).exit().assemble()


def xdp_caller(pa_fd: int, cnt_fd: int) -> bytes:
    """idx = data[0] & 3; a canary on the stack; r0 = tail_call(ctx, pa, idx);
    counts per idx; returns r0 + 1000 * (canary intact) + ctx->ingress_ifindex
    read after the call (the target rewrites its copy)."""
    a = Asm()
    a.mov64(6, "r1")
    a.ldx(8, 2, 6, 0).ldx(8, 3, 6, 8)               # data, data_end
    a.mov64(4, "r2").add64(4, 1).jmp("jgt", 4, "r3", "short")
    a.ldx(1, 7, 2, 0).alu64("and", 7, 3)             # r7 = idx
    a.lddw(8, 0x1111222233334444).stx(8, 10, -8, 8)  # canary
    a.st(4, 10, -16, 0).stx(4, 10, -16, 7)           # key = idx
    a.mov64(1, "r6").ld_map_fd(2, pa_fd).mov64(3, "r7").call(TAIL)
    a.mov64(9, "r0")
    # cnt[idx] += 1
    a.ld_map_fd(1, cnt_fd).mov64(2, "r10").add64(2, -16).call(isa.BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "nocnt")
    a.mov64(1, 1).atomic(8, XADD, 0, 0, 1)
    a.label("nocnt")
    a.mov64(0, "r9")
    a.ldx(8, 1, 10, -8).lddw(2, 0x1111222233334444).jmp("jne", 1, "r2", "bad")
    a.add64(0, 1000)
    a.label("bad")
    a.ldx(4, 1, 6, 20).alu64("add", 0, "r1")         # ctx->ingress_ifindex
    a.exit()
    a.label("short").mov64(0, 1).exit()
    return a.assemble()


def target_write(tag: int) -> bytes:
    """Writes data[1] = tag through its ctx copy's data pointer, clobbers its
    ctx copy's ingress_ifindex and its own stack, returns r2 (= 64) + tag."""
    a = Asm()
    a.ldx(8, 3, 1, 0).ldx(8, 4, 1, 8)
    a.mov64(5, "r3").add64(5, 2).jmp("jgt", 5, "r4", "out")
    a.st(1, 3, 1, tag)
    a.label("out")
    a.st(4, 1, 20, 0x7777)
    a.lddw(6, 0x5555555555555555).stx(8, 10, -8, 6)
    a.mov64(0, "r2").add64(0, tag).exit()
    return a.assemble()


def target_count(cnt_fd: int) -> bytes:
    """cnt[1] += 1, returns 2."""
    a = Asm()
    a.st(4, 10, -4, 1)
    a.ld_map_fd(1, cnt_fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "out")
    a.mov64(1, 1).atomic(8, XADD, 0, 0, 1)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def target_recurse(pa_fd: int, cnt_fd: int, slot: int) -> bytes:
    """cnt[2] += 1; r0 = tail_call(ctx, pa, slot) + 1 (itself: the depth limit
    of 32 ends the chain with -1, so the outermost returns 31)."""
    a = Asm()
    a.mov64(6, "r1")
    a.st(4, 10, -4, 2)
    a.ld_map_fd(1, cnt_fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "skip")
    a.mov64(1, 1).atomic(8, XADD, 0, 0, 1)
    a.label("skip")
    a.mov64(1, "r6").ld_map_fd(2, pa_fd).mov64(3, slot).call(TAIL)
    a.add64(0, 1).exit()
    return a.assemble()
