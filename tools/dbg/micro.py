"""Micro-benchmarks of interpreter building blocks (device-resident, 2^24 XDP units)."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from bpftime_amd import gen, isa, programs
from bpftime_amd import vm as dev
from bpftime_amd.isa import Asm

N = 1 << 24


def run(name, build, steps=10):
    dev.reset_runtime()
    ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2)
    bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)
    code = build(ctl.fd, bss.fd)
    vm = dev.VM(); vm.load(code)
    pk = dev.DeviceBuffer(N * 64)
    dev.lib().bpftime_amd_gen_xdp(pk.ptr, N, 64, 64, gen.SEED_CFG2, 0, None)
    vd = dev.DeviceBuffer(4 * N)
    for _ in range(2):
        vm.exec_batch(dev.CTX_XDP, pk, N, 64, fixed_len=64, verdicts=vd, flags=0)
    dev.lib().bpftime_amd_sync()
    e0, e1 = dev.Event(), dev.Event()
    e0.record()
    for _ in range(steps):
        vm.exec_batch(dev.CTX_XDP, pk, N, 64, fixed_len=64, verdicts=vd, flags=0)
    e1.record()
    ms = e0.elapsed_ms(e1) / steps
    n_insn = len(code) // 8
    print(f"{name:28s} insns={n_insn:3d} {ms:8.3f} ms  {N / ms / 1e3:9.1f} Mpps", flush=True)


def exit_only(c, b):
    return Asm().mov64(0, 2).exit().assemble()


def alu(k):
    def f(c, b):
        a = Asm().mov64(0, 2)
        for i in range(k):
            a.add64(3, 1)
        return a.exit().assemble()
    return f


def ctx_loads(c, b):
    return Asm().ldx(8, 2, 1, 0).ldx(8, 3, 1, 8).mov64(0, 2).exit().assemble()


def pkt_loads(k):
    def f(c, b):
        a = Asm().ldx(8, 2, 1, 0)
        for i in range(k):
            a.ldx(2, 3, 2, 2 * i)
        return a.mov64(0, 2).exit().assemble()
    return f


def pkt_ldst(c, b):
    a = Asm().ldx(8, 2, 1, 0)
    for i in range(6):
        a.ldx(2, 3, 2, 2 * i).stx(2, 2, 2 * i + 20, "r3")
    return a.mov64(0, 2).exit().assemble()


def lookup(c, b):
    a = Asm().mov64(1, 0).stx(4, 10, -4, "r1").mov64(2, "r10").add64(2, -4).ld_map_fd(1, c).call(1)
    return a.mov64(0, 2).exit().assemble()


def counter(c, b):
    a = Asm().ld_map_value(1, b, 0).ldx(8, 2, 1, 0).add64(2, 1).stx(8, 1, 0, "r2")
    return a.mov64(0, 2).exit().assemble()


run("exit only", exit_only)
run("10 alu", alu(10))
run("30 alu", alu(30))
run("2 ctx loads", ctx_loads)
run("1 pkt load", pkt_loads(1))
run("6 pkt loads", pkt_loads(6))
run("6 pkt ld+st", pkt_ldst)
run("array lookup", lookup)
run("fused counter", counter)
run("xdp-counter", programs.xdp_counter)
