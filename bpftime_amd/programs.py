"""Hand-assembled eBPF programs for the hot path and its parity tests.

No BPF clang exists in this image, so the programs below are
*hand-assembled equivalents* of the reference sources they cite -- the same
semantics after libbpf relocation / CO-RE, not byte-identical clang output.

* :func:`xdp_counter` -- ``example/xdp-counter/xdp-counter.bpf.c:50-70`` after
  relocation against ``base.btf``.
* :func:`flow_hash` -- the "deepflow-style" 5-tuple flow accounting program of
  BASELINE.json configs[2] (written here).
* :func:`syscall_agg` -- syscount-style per-syscall aggregation
  (``example/tracing/syscount/syscount.bpf.c:53-81`` + ``maps.bpf.h:10-38``)
  for BASELINE.json configs[4].
* KATs from ``vm/example/bpf_progs.h:6-119`` and ``.github/assets/sum.bpf.o``
  restated from their documented semantics (expected values are analytic).
"""
from __future__ import annotations

import struct

from .isa import (Asm, BPF_ANY, BPF_FUNC_get_current_pid_tgid, BPF_FUNC_ktime_get_ns, BPF_FUNC_map_lookup_elem,
                  BPF_FUNC_map_update_elem, BPF_FUNC_override_return, BPF_FUNC_set_retval,
                  BPF_FUNC_ringbuf_output, BPF_NOEXIST, ATOMIC_ADD, XDP_DROP, XDP_PASS, XDP_TX, XDP_ABORTED)

ETH_P_IP_LE = 0x0008  # htons(0x0800) as read by a little-endian ldxh
IPPROTO_TCP, IPPROTO_UDP = 6, 17


def xdp_counter(ctl_fd: int, bss_fd: int) -> bytes:
    """``xdp_pass`` of example/xdp-counter (SURVEY.md Appendix A, 38 insns).

    ctl_array: ARRAY key 4 value 4 max 2; .bss: ARRAY key 4 value 4096 max 1
    holding ``__u64 cntrs_array[512]`` (xdp-counter.bpf.c:24-32).
    """
    a = Asm()
    a.mov64(6, "r1")                      # 0  r6 = ctx
    a.mov64(1, 0)                         # 1
    a.stx(4, 10, -4, "r1")                # 2  *(u32*)(fp-4) = 0 (ctl_flag_pos)
    a.mov64(2, "r10")                     # 3
    a.add64(2, -4)                        # 4
    a.ld_map_fd(1, ctl_fd)                # 5,6 r1 = &ctl_array
    a.call(BPF_FUNC_map_lookup_elem)      # 7
    a.mov64(1, "r0")                      # 8
    a.mov64(0, XDP_PASS)                  # 9
    a.jmp("jeq", 1, 0, "out")             # 10 if (!flag) return XDP_PASS
    a.ldx(4, 1, 1, 0)                     # 11 r1 = *flag
    a.jmp("jne", 1, 0, "out")             # 12 if (*flag != 0) return XDP_PASS
    a.ld_map_value(1, bss_fd, 0)          # 13,14 r1 = &cntrs_array[0]
    a.ldx(8, 2, 1, 0)                     # 15  cntrs_array[0]++  (ldx/add/stx RMW)
    a.add64(2, 1)                         # 16
    a.stx(8, 1, 0, "r2")                  # 17
    a.ldx(8, 1, 6, 8)                     # 18 r1 = ctx->data_end
    a.ldx(8, 2, 6, 0)                     # 19 r2 = ctx->data
    a.mov64(3, "r2")                      # 20
    a.add64(3, 14)                        # 21
    a.mov64(0, XDP_DROP)                  # 22
    a.jmp("jgt", 3, "r1", "out")          # 23 if (data + 14 > data_end) return XDP_DROP
    a.ldx(2, 1, 2, 0)                     # 24 swap_src_dst_mac
    a.ldx(2, 3, 2, 6)                     # 25
    a.stx(2, 2, 0, "r3")                  # 26
    a.ldx(2, 3, 2, 2)                     # 27
    a.ldx(2, 4, 2, 8)                     # 28
    a.stx(2, 2, 2, "r4")                  # 29
    a.ldx(2, 4, 2, 4)                     # 30
    a.ldx(2, 5, 2, 10)                    # 31
    a.stx(2, 2, 4, "r5")                  # 32
    a.stx(2, 2, 6, "r1")                  # 33
    a.stx(2, 2, 8, "r3")                  # 34
    a.stx(2, 2, 10, "r4")                 # 35
    a.mov64(0, XDP_TX)                    # 36
    a.label("out")
    a.exit()                              # 37
    code = a.assemble()
    assert len(code) == 38 * 8
    return code


def flow_hash(flows_fd: int) -> bytes:
    """5-tuple flow accounting over Eth/IPv4/{TCP,UDP} (BASELINE configs[2]).

    flows: HASH key 16 B {u32 saddr, u32 daddr, u16 sport, u16 dport, u8 proto,
    u8 pad[3]}, value 16 B {u64 pkts, u64 bytes}.  Uses the
    ``bpf_map_lookup_or_try_init`` idiom (syscount maps.bpf.h:10-38) and
    ``__sync_fetch_and_add`` (BPF_ATOMIC add).  Verdicts: runt -> DROP,
    non-IPv4 / ihl!=5 / other L4 -> PASS, TCP -> TX, UDP -> PASS.
    """
    a = Asm()
    a.ldx(8, 2, 1, 0)                     # r2 = data
    a.ldx(8, 3, 1, 8)                     # r3 = data_end
    a.mov64(6, "r3")
    a.alu64("sub", 6, "r2")               # r6 = len
    a.mov64(4, "r2")
    a.add64(4, 14)
    a.mov64(0, XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")          # runt ethernet
    a.ldx(2, 4, 2, 12)                    # h_proto
    a.mov64(0, XDP_PASS)
    a.jmp("jne", 4, ETH_P_IP_LE, "out")   # not IPv4
    a.mov64(4, "r2")
    a.add64(4, 34)
    a.mov64(0, XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")          # runt IPv4
    a.ldx(1, 4, 2, 14)                    # ver/ihl
    a.mov64(0, XDP_PASS)
    a.jmp("jne", 4, 0x45, "out")
    a.ldx(1, 7, 2, 23)                    # r7 = proto
    a.jmp("jeq", 7, IPPROTO_TCP, "l4")
    a.jmp("jne", 7, IPPROTO_UDP, "out")
    a.label("l4")
    a.mov64(4, "r2")
    a.add64(4, 38)
    a.mov64(0, XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")          # runt L4
    # key on stack at fp-16 .. fp-1
    a.ldx(4, 4, 2, 26)                    # saddr (unaligned packet load)
    a.stx(4, 10, -16, "r4")
    a.ldx(4, 4, 2, 30)                    # daddr
    a.stx(4, 10, -12, "r4")
    a.ldx(4, 4, 2, 34)                    # sport|dport
    a.stx(4, 10, -8, "r4")
    a.stx(4, 10, -4, "r7")                # proto + 3 zero pad bytes
    # zero value at fp-32
    a.st(8, 10, -32, 0)
    a.st(8, 10, -24, 0)
    # v = lookup(flows, &key)
    a.ld_map_fd(1, flows_fd)
    a.mov64(2, "r10")
    a.add64(2, -16)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jne", 0, 0, "have")
    a.ld_map_fd(1, flows_fd)
    a.mov64(2, "r10")
    a.add64(2, -16)
    a.mov64(3, "r10")
    a.add64(3, -32)
    a.mov64(4, BPF_NOEXIST)
    a.call(BPF_FUNC_map_update_elem)
    a.ld_map_fd(1, flows_fd)
    a.mov64(2, "r10")
    a.add64(2, -16)
    a.call(BPF_FUNC_map_lookup_elem)
    a.mov64(1, "r0")
    a.mov64(0, XDP_ABORTED)
    a.jmp("jeq", 1, 0, "out")
    a.mov64(0, "r1")
    a.label("have")
    a.mov64(1, 1)
    a.atomic(8, ATOMIC_ADD, 0, 0, "r1")   # __sync_fetch_and_add(&v->pkts, 1)
    a.atomic(8, ATOMIC_ADD, 0, 8, "r6")   # __sync_fetch_and_add(&v->bytes, len)
    a.mov64(0, XDP_TX)
    a.jmp("jeq", 7, IPPROTO_TCP, "out")
    a.mov64(0, XDP_PASS)
    a.label("out")
    a.exit()
    return a.assemble()


def syscall_agg(counts_fd: int) -> bytes:
    """syscount-style aggregation over ``trace_event_raw_sys_enter`` (64 B ctx:
    id@8, args[6]@16; attach/syscall_trace_attach_impl/include/
    syscall_trace_attach_impl.hpp:17-29).

    counts: HASH key u32 id, value data_t 32 B {u64 count, u64 total_ns,
    char comm[16]} (syscount.h).  ``count = count + 1`` is the plain RMW of
    syscount.bpf.c:81; for ids 0/1 ``total_ns += args[2]``.  Returns 0.
    """
    a = Asm()
    a.ldx(8, 6, 1, 8)                     # r6 = id
    a.ldx(8, 7, 1, 32)                    # r7 = args[2]
    a.stx(4, 10, -4, "r6")                # key = (u32)id
    a.ld_map_fd(1, counts_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jne", 0, 0, "have")
    a.st(8, 10, -40, 0)                   # static const struct data_t zero
    a.st(8, 10, -32, 0)
    a.st(8, 10, -24, 0)
    a.st(8, 10, -16, 0)
    a.ld_map_fd(1, counts_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.mov64(3, "r10")
    a.add64(3, -40)
    a.mov64(4, BPF_NOEXIST)
    a.call(BPF_FUNC_map_update_elem)
    a.ld_map_fd(1, counts_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "ret")
    a.label("have")
    a.ldx(8, 1, 0, 0)                     # val->count = val->count + 1
    a.add64(1, 1)
    a.stx(8, 0, 0, "r1")
    a.jmp("jgt", 6, 1, "ret")             # only read/write (nr 0/1) accumulate
    a.ldx(8, 2, 0, 8)                     # val->total_ns += args[2]
    a.add64(2, "r7")
    a.stx(8, 0, 8, "r2")
    a.label("ret")
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


# syscount's const volatile options (example/tracing/syscount/syscount.bpf.c:
# 12-17) as its .rodata: bool filter_cg @0, count_by_process @1,
# measure_latency @2, filter_failed @3, int filter_errno @4, pid_t
# filter_pid @8 (12 B, an ARRAY map of one value, read through lddw map_val)
SYSCOUNT_RODATA = 12
EEXIST = 17


def syscount_rodata(count_by_process: bool = False, filter_failed: bool = False, filter_errno: int = 0,
                    filter_pid: int = 0, measure_latency: bool = False) -> bytes:
    return struct.pack("<BBBBii", 0, int(count_by_process), int(measure_latency), int(filter_failed),
                       filter_errno, filter_pid)


def syscount_enter(start_fd: int, rodata_fd: int) -> bytes:
    """syscount's sys_enter program (example/tracing/syscount/syscount.bpf.c:
    33-47): the caller's pid_tgid; filter_pid on the pid (.rodata @8); ``ts =
    bpf_ktime_get_ns()``; ``bpf_map_update_elem(&start, &tid, &ts, 0)``.
    start: HASH u32 tid -> u64 ns.  Returns 0."""
    a = Asm()
    a.call(BPF_FUNC_get_current_pid_tgid)
    a.stx(4, 10, -4, "r0")                # u32 tid = id
    a.mov64(6, "r0").alu64("rsh", 6, 32)  # pid = id >> 32
    a.ld_map_value(9, rodata_fd, 0)
    a.ldx(4, 2, 9, 8)                     # filter_pid
    a.jmp("jeq", 2, 0, "nopid")
    a.jmp32("jne", 6, "r2", "ret")        # (pid_t) pid != filter_pid
    a.label("nopid")
    a.call(BPF_FUNC_ktime_get_ns)
    a.stx(8, 10, -16, "r0")               # ts
    a.ld_map_fd(1, start_fd)
    a.mov64(2, "r10").add64(2, -4)
    a.mov64(3, "r10").add64(3, -16)
    a.mov64(4, BPF_ANY)
    a.call(BPF_FUNC_map_update_elem)
    a.label("ret")
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


def syscount_exit(data_fd: int, rodata_fd: int, start_fd: int = -1) -> bytes:
    """syscount's sys_exit program (example/tracing/syscount/syscount.bpf.c:
    49-87) over ``trace_event_raw_sys_exit`` {ent, id@8, ret@16}: skip id == -1
    (an interrupt), filter_pid on the caller's pid, filter_failed (ret >= 0
    skipped) and filter_errno (ret != -filter_errno skipped) from .rodata;
    with ``start_fd`` (the sys_enter program's start map) the measure_latency
    path: ``start_ts = lookup(&start, &tid)``, none -> return, ``lat =
    bpf_ktime_get_ns() - *start_ts``; key = count_by_process ? pid : id;
    ``bpf_map_lookup_or_try_init`` of data (maps.bpf.h: lookup, NOEXIST update
    of a zeroed data_t, an error other than -EEXIST gives up, lookup again);
    ``count = count + 1`` and, measuring latency, ``total_ns = total_ns +
    lat``.  data: HASH u32 -> data_t 32 B {u64 count, u64 total_ns, char
    comm[16]}.  Returns 0."""
    a = Asm()
    a.mov64(6, "r1")
    a.call(BPF_FUNC_get_current_pid_tgid)
    a.stx(4, 10, -8, "r0")                # u32 tid = id
    a.mov64(8, "r0").alu64("rsh", 8, 32)  # pid = id >> 32
    a.ldx(8, 7, 6, 8)                     # args->id
    a.jmp("jeq", 7, -1, "ret")
    a.ld_map_value(9, rodata_fd, 0)
    a.ldx(4, 2, 9, 8)                     # filter_pid
    a.jmp("jeq", 2, 0, "nopid")
    a.jmp32("jne", 8, "r2", "ret")        # (pid_t) pid != filter_pid
    a.label("nopid")
    a.ldx(8, 3, 6, 16)                    # args->ret
    a.ldx(1, 2, 9, 3)                     # filter_failed
    a.jmp("jeq", 2, 0, "nofail")
    a.jmp("jsge", 3, 0, "ret")
    a.label("nofail")
    a.ldx(4, 2, 9, 4)                     # filter_errno
    a.jmp("jeq", 2, 0, "noerr")
    a.alu64("lsh", 2, 32).alu64("arsh", 2, 32).neg64(2)  # (long) -filter_errno
    a.jmp("jne", 3, "r2", "ret")
    a.label("noerr")
    a.st(8, 10, -48, 0)                   # lat = 0
    if start_fd >= 0:
        a.ldx(1, 2, 9, 2)                 # measure_latency
        a.jmp("jeq", 2, 0, "nolat")
        a.ld_map_fd(1, start_fd)
        a.mov64(2, "r10").add64(2, -8)
        a.call(BPF_FUNC_map_lookup_elem)  # start_ts = lookup(&start, &tid)
        a.jmp("jeq", 0, 0, "ret")
        a.ldx(8, 1, 0, 0)
        a.stx(8, 10, -48, "r1")
        a.call(BPF_FUNC_ktime_get_ns)
        a.ldx(8, 1, 10, -48)
        a.alu64("sub", 0, "r1")           # lat = now - *start_ts
        a.stx(8, 10, -48, "r0")
        a.label("nolat")
    a.ldx(1, 2, 9, 1)                     # count_by_process
    a.mov64(1, "r7")
    a.jmp("jeq", 2, 0, "key")
    a.mov64(1, "r8")
    a.label("key")
    a.stx(4, 10, -4, "r1")                # u32 key
    a.ld_map_fd(1, data_fd)
    a.mov64(2, "r10").add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jne", 0, 0, "have")
    a.st(8, 10, -40, 0)                   # static const struct data_t zero
    a.st(8, 10, -32, 0)
    a.st(8, 10, -24, 0)
    a.st(8, 10, -16, 0)
    a.ld_map_fd(1, data_fd)
    a.mov64(2, "r10").add64(2, -4)
    a.mov64(3, "r10").add64(3, -40)
    a.mov64(4, BPF_NOEXIST)
    a.call(BPF_FUNC_map_update_elem)
    a.jmp("jeq", 0, 0, "again")
    a.jmp("jne", 0, -EEXIST, "ret")       # err && err != -EEXIST: give up
    a.label("again")
    a.ld_map_fd(1, data_fd)
    a.mov64(2, "r10").add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "ret")
    a.label("have")
    a.ldx(8, 1, 0, 0)                     # val->count = val->count + 1
    a.add64(1, 1)
    a.stx(8, 0, 0, "r1")
    if start_fd >= 0:
        a.ldx(1, 2, 9, 2)                 # measure_latency
        a.jmp("jeq", 2, 0, "ret")
        a.ldx(8, 2, 10, -48)
        a.ldx(8, 1, 0, 8)                 # val->total_ns = val->total_ns + lat
        a.add64(1, "r2")
        a.stx(8, 0, 8, "r1")
    a.label("ret")
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


def tid_state_enter(start_fd: int) -> bytes:
    """A sys_enter program that keeps per-thread state: ``start[tid] =
    args[0]`` (start: HASH u32 tid -> u64), the shape of syscount's latency
    pair with the argument in place of the clock."""
    a = Asm()
    a.mov64(6, "r1")
    a.call(BPF_FUNC_get_current_pid_tgid)
    a.stx(4, 10, -4, "r0")
    a.ldx(8, 1, 6, 16)                    # args[0]
    a.stx(8, 10, -16, "r1")
    a.ld_map_fd(1, start_fd)
    a.mov64(2, "r10").add64(2, -4)
    a.mov64(3, "r10").add64(3, -16)
    a.mov64(4, BPF_ANY)
    a.call(BPF_FUNC_map_update_elem)
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


def tid_state_exit(start_fd: int, sum_fd: int) -> bytes:
    """Its sys_exit partner: ``sum += start[tid]`` (sum: an ARRAY u64 @0),
    ``sum2 += start[tid] * ret`` (@8): the value the same call's sys_enter
    stored."""
    a = Asm()
    a.mov64(6, "r1")
    a.call(BPF_FUNC_get_current_pid_tgid)
    a.stx(4, 10, -4, "r0")
    a.ld_map_fd(1, start_fd)
    a.mov64(2, "r10").add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "out")
    a.ldx(8, 3, 0, 0)
    a.ld_map_value(2, sum_fd, 0)
    a.atomic(8, ATOMIC_ADD, 2, 0, 3)
    a.ldx(8, 4, 6, 16)                    # ret
    a.alu64("mul", 3, "r4")
    a.atomic(8, ATOMIC_ADD, 2, 8, 3)
    a.label("out")
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


def inject_enter(mod: int, value: int = -1) -> bytes:
    """error-inject's sys_enter program (example/error-inject/
    error_inject_syscall.bpf.c:12-22) made deterministic for replays (B.11):
    ``bpf_override_return(ctx, value)`` when args[2] % mod == 0 instead of on
    an even ``bpf_get_prandom_u32``.  Returns 0."""
    a = Asm()
    a.ldx(8, 2, 1, 32)                    # args[2]
    a.alu64("mod", 2, mod)
    a.jmp("jne", 2, 0, "ret")
    a.mov64(2, value)
    a.call(BPF_FUNC_override_return)
    a.label("ret")
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


def exit_clamp(value: int = 0) -> bytes:
    """A sys_exit program that turns a failed call's return into ``value``
    with ``bpf_set_retval`` (bpf_helper.cpp:1282-1286) when ret < 0 and id
    is odd.  Returns 0."""
    a = Asm()
    a.ldx(8, 3, 1, 16)                    # args->ret
    a.jmp("jsge", 3, 0, "ret")
    a.ldx(8, 2, 1, 8)
    a.jmp("jset", 2, 1, "set")
    a.ja("ret")
    a.label("set")
    a.mov64(1, value)
    a.call(BPF_FUNC_set_retval)
    a.label("ret")
    a.mov64(0, 0)
    a.exit()
    return a.assemble()


def lpm_route(routes_fd: int) -> bytes:
    """XDP routing: verdict = u32 value of the longest prefix (LPM_TRIE,
    key {u32 prefixlen = 32, be32 daddr}) containing the IPv4 destination;
    PASS when there is no route or the frame is not IPv4."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, XDP_PASS)
    a.mov64(4, "r2").add64(4, 34).jmp("jgt", 4, "r3", "out")
    a.ldx(2, 4, 2, 12).jmp("jne", 4, ETH_P_IP_LE, "out")
    a.st(4, 10, -8, 32).ldx(4, 4, 2, 30).stx(4, 10, -4, "r4")
    a.ld_map_fd(1, routes_fd).mov64(2, "r10").add64(2, -8).call(BPF_FUNC_map_lookup_elem)
    a.mov64(1, "r0").mov64(0, XDP_PASS).jmp("jeq", 1, 0, "out").ldx(4, 0, 1, 0)
    a.label("out").exit()
    return a.assemble()


def ringbuf_sampler(rb_fd: int, every_log2: int = 4) -> bytes:
    """XDP sampler: frames whose first byte is 0 modulo 2^every_log2 send
    their first 12 bytes (the MACs) to a ring buffer with
    bpf_ringbuf_output (bpf_helper.cpp:451-467); verdict PASS, DROP when
    the ring had no room."""
    a = Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, XDP_PASS)
    a.mov64(4, "r2").add64(4, 14).jmp("jgt", 4, "r3", "out")
    a.ldx(1, 4, 2, 0).alu64("and", 4, (1 << every_log2) - 1).jmp("jne", 4, 0, "out")
    a.ld_map_fd(1, rb_fd).mov64(3, 12).mov64(4, 0).call(BPF_FUNC_ringbuf_output)
    a.mov64(1, "r0").mov64(0, XDP_PASS).jmp("jeq", 1, 0, "out").mov64(0, XDP_DROP)
    a.label("out").exit()
    return a.assemble()


# ---------------------------------------------------------------------------
# Interpreter known-answer programs (analytic expectations).
# ---------------------------------------------------------------------------

def lru_track(lru_fd: int) -> bytes:
    """Connection-tracking style use of an LRU hash (key u32, value 16 B {u64
    hits, u64 tag}) over 16-B raw units {u32 key, u32 op, u64 tag}:
      op 0: lookup; a hit adds 1 to hits and returns the element's tag, a
            miss inserts {0, tag} with BPF_ANY, looks up again, adds 1 to
            hits and returns 100 + the insert's result
      op 1: update {0, tag} with BPF_NOEXIST, returns 200 + its result
      op 2: delete, returns 300 + its result
      op 3: update {0, tag} with BPF_EXIST, returns 400 + its result"""
    a = Asm()
    a.mov64(6, "r1")
    a.ldx(4, 2, 6, 0)
    a.stx(4, 10, -4, "r2")                # key at fp-4
    a.ldx(4, 7, 6, 4)                     # r7 = op
    a.ldx(8, 8, 6, 8)                     # r8 = tag
    a.st(8, 10, -24, 0)                   # value {0, tag} at fp-24
    a.stx(8, 10, -16, "r8")
    a.jmp("jeq", 7, 1, "noexist")
    a.jmp("jeq", 7, 2, "delete")
    a.jmp("jeq", 7, 3, "exist")
    a.ld_map_fd(1, lru_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "miss")
    a.mov64(1, 1)
    a.atomic(8, ATOMIC_ADD, 0, 0, "r1")   # __sync_fetch_and_add(&v->hits, 1)
    a.ldx(8, 0, 0, 8)                     # return v->tag
    a.exit()
    a.label("miss")                       # bpf_map_lookup_or_try_init (BPF_ANY), then count
    a.ld_map_fd(1, lru_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.mov64(3, "r10")
    a.add64(3, -24)
    a.mov64(4, BPF_ANY)
    a.call(BPF_FUNC_map_update_elem)
    a.mov64(9, "r0")
    a.add64(9, 100)
    a.ld_map_fd(1, lru_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "ret9")
    a.mov64(1, 1)
    a.atomic(8, ATOMIC_ADD, 0, 0, "r1")
    a.label("ret9")
    a.mov64(0, "r9")
    a.exit()
    a.label("noexist")
    a.mov64(9, 200)
    a.mov64(4, BPF_NOEXIST)
    a.ja("upd")
    a.label("exist")
    a.mov64(9, 400)
    a.mov64(4, 2)                         # BPF_EXIST
    a.label("upd")
    a.ld_map_fd(1, lru_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.mov64(3, "r10")
    a.add64(3, -24)
    a.call(BPF_FUNC_map_update_elem)
    a.add64(0, "r9")
    a.exit()
    a.label("delete")
    a.ld_map_fd(1, lru_fd)
    a.mov64(2, "r10")
    a.add64(2, -4)
    a.call(3)                             # bpf_map_delete_elem
    a.add64(0, 300)
    a.exit()
    return a.assemble()


def kat_add_mem() -> bytes:
    """vm/example/bpf_progs.h:6-11 ``bpf_add_mem_64_bit_minimal``: return
    ``(u32)mem[0..4) + (u32)mem[4..8)`` (64-bit add of two zero-extended words)."""
    a = Asm()
    a.ldx(4, 2, 1, 0)
    a.ldx(4, 0, 1, 4)
    a.add64(0, "r2")
    a.exit()
    return a.assemble()


def kat_add_mem_stack() -> bytes:
    """vm/example/bpf_progs.h:44-57 ``bpf_add_mem_64_bit``: spill r1/r2 to the
    stack, reload, return ``d->a + d->b``."""
    a = Asm()
    a.stx(8, 10, -8, "r1")
    a.stx(4, 10, -12, "r2")
    a.ldx(8, 1, 10, -8)
    a.ldx(4, 0, 1, 0)
    a.ldx(4, 1, 1, 4)
    a.add64(0, "r1")
    a.exit()
    return a.assemble()


def kat_mul() -> bytes:
    """vm/example/bpf_progs.h:66-77 ``bpf_mul_64_bit``: 1*2 through the stack -> 2."""
    a = Asm()
    a.mov64(1, 1)
    a.stx(4, 10, -4, "r1")
    a.mov64(1, 2)
    a.stx(4, 10, -8, "r1")
    a.ldx(4, 1, 10, -4)
    a.ldx(4, 2, 10, -8)
    a.alu32("mul", 1, "r2")
    a.stx(4, 10, -12, "r1")
    a.ldx(4, 0, 10, -12)
    a.exit()
    return a.assemble()


def kat_sum() -> bytes:
    """``.github/assets/sum.bpf.o`` ``int test(int *arr)``: return
    ``sum(arr[1..arr[0]])`` over signed 32-bit ints (loop with jsgt, arsh
    sign extension and stack spills), restated from its documented semantics."""
    a = Asm()
    a.stx(8, 10, -8, "r1")                # spill arr
    a.ldx(4, 2, 1, 0)                     # n = arr[0]
    a.alu64("lsh", 2, 32)
    a.alu64("arsh", 2, 32)                # sign-extend n
    a.mov64(0, 0)                         # sum
    a.mov64(3, 1)                         # i = 1
    a.label("loop")
    a.jmp("jsgt", 3, "r2", "done")
    a.ldx(8, 1, 10, -8)
    a.mov64(4, "r3")
    a.alu64("lsh", 4, 2)
    a.add64(1, "r4")
    a.ldx(4, 5, 1, 0)
    a.alu64("lsh", 5, 32)
    a.alu64("arsh", 5, 32)
    a.add64(0, "r5")
    a.add64(3, 1)
    a.ja("loop")
    a.label("done")
    a.alu64("lsh", 0, 32)                 # return (int)sum
    a.alu64("arsh", 0, 32)
    a.exit()
    return a.assemble()


def kat_div64_call(helper_id: int = 3) -> bytes:
    """vm/example/bpf_progs.h:101-119 ``bpf_div64_code`` shape: r0 = helper(1, 5);
    r2 = 8 / r0 (64-bit, div-by-zero -> 0); returns r0 (the helper result)."""
    a = Asm()
    a.ldx(8, 3, 1, 0)
    a.mov64(1, 1)
    a.mov64(2, 5)
    a.call(helper_id)
    a.stx(8, 10, -8, "r0")
    a.ldx(8, 1, 10, -8)
    a.mov64(2, 8)
    a.alu64("div", 2, "r1")
    a.stx(8, 10, -16, "r2")
    a.exit()
    return a.assemble()


# ---- bpf_tail_call programs (runtime/src/bpf_helper.cpp:568-650) -----------
# A jump-table XDP caller and its targets; tests/test_*_tailcall.py and the
# tail-call bench workload use them.

_TAIL = 12  # BPF_FUNC_tail_call
_XADD = 0x00  # BPF_ADD atomic


def tail_ref_kat_caller(pa_fd: int, tail_then_exit: bool) -> bytes:
    """runtime/unit-test/tailcall/test_user_to_user_tailcall.cpp caller:
    lddw r2 = the prog array fd as a plain immediate, r3 = 0, call 0x0c.
    With tail_then_exit the program exits with the helper's r0 (the callee's
    0x1234 under both VM backends); otherwise it then returns 0xdead as in
    the reference test body."""
    a = Asm().lddw(2, pa_fd).mov64(3, 0).call(_TAIL)
    if not tail_then_exit:
        a.mov64(0, 0xdead)
    return a.exit().assemble()


def tail_ref_kat_target() -> bytes:
    return Asm().mov64(0, 0x1234).exit().assemble()


def tail_xdp_caller(pa_fd: int, cnt_fd: int) -> bytes:
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
    a.mov64(1, "r6").ld_map_fd(2, pa_fd).mov64(3, "r7").call(_TAIL)
    a.mov64(9, "r0")
    # cnt[idx] += 1
    a.ld_map_fd(1, cnt_fd).mov64(2, "r10").add64(2, -16).call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "nocnt")
    a.mov64(1, 1).atomic(8, _XADD, 0, 0, 1)
    a.label("nocnt")
    a.mov64(0, "r9")
    a.ldx(8, 1, 10, -8).lddw(2, 0x1111222233334444).jmp("jne", 1, "r2", "bad")
    a.add64(0, 1000)
    a.label("bad")
    a.ldx(4, 1, 6, 20).alu64("add", 0, "r1")         # ctx->ingress_ifindex
    a.exit()
    a.label("short").mov64(0, 1).exit()
    return a.assemble()


def tail_target_write(tag: int) -> bytes:
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


def tail_target_count(cnt_fd: int) -> bytes:
    """cnt[1] += 1, returns 2."""
    a = Asm()
    a.st(4, 10, -4, 1)
    a.ld_map_fd(1, cnt_fd).mov64(2, "r10").add64(2, -4).call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "out")
    a.mov64(1, 1).atomic(8, _XADD, 0, 0, 1)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def tail_target_recurse(pa_fd: int, cnt_fd: int, slot: int) -> bytes:
    """cnt[2] += 1; r0 = tail_call(ctx, pa, slot) + 1 (itself: the depth limit
    of 32 ends the chain with -1, so the outermost returns 31)."""
    a = Asm()
    a.mov64(6, "r1")
    a.st(4, 10, -4, 2)
    a.ld_map_fd(1, cnt_fd).mov64(2, "r10").add64(2, -4).call(BPF_FUNC_map_lookup_elem)
    a.jmp("jeq", 0, 0, "skip")
    a.mov64(1, 1).atomic(8, _XADD, 0, 0, 1)
    a.label("skip")
    a.mov64(1, "r6").ld_map_fd(2, pa_fd).mov64(3, slot).call(_TAIL)
    a.add64(0, 1).exit()
    return a.assemble()
