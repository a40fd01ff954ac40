"""Interpreter cost model on the GPU: kernel time of tiny XDP programs over
2^24 64-B frames (fixed per-unit cost, cost per dispatched instruction of a
few handler classes).  python tools/experiments/micro.py [log2n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench_workloads as bw  # noqa: E402
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

PKT = 64


def ret_only():
    a = isa.Asm()
    a.mov64(0, isa.XDP_PASS)
    a.exit()
    return a.assemble()


def alu(n):
    a = isa.Asm()
    for i in range(n):
        a.add64(3, i + 1)
    a.mov64(0, isa.XDP_PASS)
    a.exit()
    return a.assemble()


def alu_rr(n):
    a = isa.Asm()
    a.mov64(4, 7)
    for i in range(n):
        a.add64(3, "r4")
    a.mov64(0, isa.XDP_PASS)
    a.exit()
    return a.assemble()


def staged_loads(n):
    a = isa.Asm()
    a.ldx(8, 2, 1, 0)
    a.ldx(8, 3, 1, 8)
    a.mov64(4, "r2")
    a.add64(4, 32)
    a.mov64(0, isa.XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")
    for i in range(n):
        a.ldx(2, 5, 2, 2 * (i % 16))
    a.mov64(0, isa.XDP_PASS)
    a.label("out")
    a.exit()
    return a.assemble()


def jumps(n):
    a = isa.Asm()
    for i in range(n):
        a.jmp("jeq", 3, 12345, "out")
    a.mov64(0, isa.XDP_PASS)
    a.label("out")
    a.exit()
    return a.assemble()


def xc(ctl_fd, bss_fd, lookup=True, counter=True, loads=True, stores=True):
    """xdp-counter (programs.xdp_counter) with parts left out."""
    a = isa.Asm()
    a.mov64(6, "r1")
    if lookup:
        a.mov64(1, 0)
        a.stx(4, 10, -4, "r1")
        a.mov64(2, "r10")
        a.add64(2, -4)
        a.ld_map_fd(1, ctl_fd)
        a.call(1)
        a.mov64(1, "r0")
        a.mov64(0, isa.XDP_PASS)
        a.jmp("jeq", 1, 0, "out")
        a.ldx(4, 1, 1, 0)
        a.jmp("jne", 1, 0, "out")
    if counter:
        a.ld_map_value(1, bss_fd, 0)
        a.ldx(8, 2, 1, 0)
        a.add64(2, 1)
        a.stx(8, 1, 0, "r2")
    a.ldx(8, 1, 6, 8)
    a.ldx(8, 2, 6, 0)
    a.mov64(3, "r2")
    a.add64(3, 14)
    a.mov64(0, isa.XDP_DROP)
    a.jmp("jgt", 3, "r1", "out")
    if loads:
        a.ldx(2, 1, 2, 0)
        a.ldx(2, 3, 2, 6)
    if stores:
        a.stx(2, 2, 0, "r3")
    if loads:
        a.ldx(2, 3, 2, 2)
        a.ldx(2, 4, 2, 8)
    if stores:
        a.stx(2, 2, 2, "r4")
    if loads:
        a.ldx(2, 4, 2, 4)
        a.ldx(2, 5, 2, 10)
    if stores:
        a.stx(2, 2, 4, "r5")
        a.stx(2, 2, 6, "r1")
        a.stx(2, 2, 8, "r3")
        a.stx(2, 2, 10, "r4")
    a.mov64(0, isa.XDP_TX)
    a.label("out")
    a.exit()
    return a.assemble()


def stores(load_at, store_ats):
    """Staged window sized by a load at load_at; 2-byte stores at store_ats."""
    a = isa.Asm()
    a.ldx(8, 2, 1, 0)
    a.ldx(8, 3, 1, 8)
    a.mov64(4, "r2")
    a.add64(4, 64)
    a.mov64(0, isa.XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")
    a.ldx(2, 5, 2, load_at)
    for at in store_ats:
        a.stx(2, 2, at, "r5")
    a.mov64(0, isa.XDP_PASS)
    a.label("out")
    a.exit()
    return a.assemble()


def flow(flows_fd, lookup=True, adds=True, split=True):
    """programs.flow_hash with parts left out (split=False: no TCP/UDP
    divergence)."""
    from bpftime_amd.isa import BPF_NOEXIST
    a = isa.Asm()
    a.ldx(8, 2, 1, 0)
    a.ldx(8, 3, 1, 8)
    a.mov64(6, "r3")
    a.alu64("sub", 6, "r2")
    a.mov64(4, "r2")
    a.add64(4, 14)
    a.mov64(0, isa.XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")
    a.ldx(2, 4, 2, 12)
    a.mov64(0, isa.XDP_PASS)
    a.jmp("jne", 4, 0x0008, "out")
    a.mov64(4, "r2")
    a.add64(4, 34)
    a.mov64(0, isa.XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")
    a.ldx(1, 4, 2, 14)
    a.mov64(0, isa.XDP_PASS)
    a.jmp("jne", 4, 0x45, "out")
    a.ldx(1, 7, 2, 23)
    if split:
        a.jmp("jeq", 7, 6, "l4")
        a.jmp("jne", 7, 17, "out")
    a.label("l4")
    a.mov64(4, "r2")
    a.add64(4, 38)
    a.mov64(0, isa.XDP_DROP)
    a.jmp("jgt", 4, "r3", "out")
    a.ldx(4, 4, 2, 26)
    a.stx(4, 10, -16, "r4")
    a.ldx(4, 4, 2, 30)
    a.stx(4, 10, -12, "r4")
    a.ldx(4, 4, 2, 34)
    a.stx(4, 10, -8, "r4")
    a.stx(4, 10, -4, "r7")
    a.st(8, 10, -32, 0)
    a.st(8, 10, -24, 0)
    if lookup:
        a.ld_map_fd(1, flows_fd)
        a.mov64(2, "r10")
        a.add64(2, -16)
        a.call(1)
        a.jmp("jne", 0, 0, "have")
        a.ld_map_fd(1, flows_fd)
        a.mov64(2, "r10")
        a.add64(2, -16)
        a.mov64(3, "r10")
        a.add64(3, -32)
        a.mov64(4, BPF_NOEXIST)
        a.call(2)
        a.ld_map_fd(1, flows_fd)
        a.mov64(2, "r10")
        a.add64(2, -16)
        a.call(1)
        a.mov64(1, "r0")
        a.mov64(0, isa.XDP_ABORTED)
        a.jmp("jeq", 1, 0, "out")
        a.mov64(0, "r1")
        a.label("have")
        if adds:
            a.mov64(1, 1)
            a.atomic(8, isa.ATOMIC_ADD, 0, 0, "r1")
            a.atomic(8, isa.ATOMIC_ADD, 0, 8, "r6")
    a.mov64(0, isa.XDP_TX)
    if split:
        a.jmp("jeq", 7, 6, "out")
        a.mov64(0, isa.XDP_PASS)
    a.label("out")
    a.exit()
    return a.assemble()


def flow_cases(n, zipf_s=1.1, only=None):
    """flow-hash variants over the bench's frames (2048-B slots)."""
    nflows, stride = 65536, 2048
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(nflows, zipf_s))
    pk = dev.DeviceBuffer(n * stride)
    dl = dev.DeviceBuffer(4 * n)
    if dev.lib().bpftime_amd_gen_flow(pk.ptr, dl.ptr, n, stride, gen.SEED_CFG3, 0, cdf.ptr, nflows, None):
        raise SystemExit("flow generator failed")
    dv = dev.DeviceBuffer(4 * n)
    for name, kw in [("flow", {}), ("flow-noadds", {"adds": False}), ("flow-nolookup", {"lookup": False}),
                     ("flow-nosplit", {"split": False}), ("flow-nosplit-nolk", {"split": False, "lookup": False})]:
        if only and name not in only:
            continue
        flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, nflows, name="flows")
        vm = dev.VM()
        vm.load(flow(flows.fd, **kw))

        def step():
            vm.exec_batch(dev.CTX_XDP, pk, n, stride, lens=dl, verdicts=dv, flags=0)
        _, k = bw._timed(dev, step, 10, 3)
        print("%-18s kernel %.4f ms  %.2f ps/pkt" % (name, k * 1e3, k / n * 1e12), flush=True)


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    n = 1 << log2n
    ngpu = dev.lib().bpftime_amd_device_count()
    if ngpu <= 0 or dev.lib().bpftime_amd_set_device(0) != 0:
        raise SystemExit("no GPU")
    dev.reset_runtime()
    ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array")
    bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, flags=isa.BPF_F_MMAPABLE, name=".bss")
    pkts = dev.DeviceBuffer(n * PKT)
    if dev.lib().bpftime_amd_gen_xdp(pkts.ptr, n, PKT, PKT, gen.SEED_CFG2, 0, None) != 0:
        raise SystemExit("generator failed")
    verd = dev.DeviceBuffer(4 * n)
    cases = [("ret", ret_only(), 2), ("alu8", alu(8), 10), ("alu32", alu(32), 34), ("alurr32", alu_rr(32), 35),
             ("ld8", staged_loads(8), 15), ("ld32", staged_loads(32), 39), ("jmp32", jumps(32), 34),
             ("xdp-counter", programs.xdp_counter(ctl.fd, bss.fd), 37),
             ("xc-nolookup", xc(ctl.fd, bss.fd, lookup=False), 26),
             ("xc-nocounter", xc(ctl.fd, bss.fd, counter=False), 33),
             ("xc-nostores", xc(ctl.fd, bss.fd, stores=False), 31),
             ("xc-noswap", xc(ctl.fd, bss.fd, loads=False, stores=False), 25),
             ("xc-bare", xc(ctl.fd, bss.fd, lookup=False, counter=False, loads=False, stores=False), 8),
             ("st-none16", stores(0, []), 9), ("st-none64", stores(60, []), 9),
             ("st-1of16", stores(0, [0]), 10), ("st-1of64", stores(60, [0]), 10),
             ("st-2of64", stores(60, [0, 16]), 11), ("st-4of64", stores(60, [0, 16, 32, 48]), 13),
             ("st-6of16", stores(0, [0, 2, 4, 6, 8, 10]), 15)]
    if os.environ.get("MICRO_FLOW"):
        del pkts
        s = float(os.environ.get("MICRO_ZIPF", "1.1"))
        flow_cases(n, s, os.environ.get("MICRO_ONLY", "").split(",") if os.environ.get("MICRO_ONLY") else None)
        return
    for name, code, ninsn in cases:
        vm = dev.VM()
        vm.load(code)

        def step():
            vm.exec_batch(dev.CTX_XDP, pkts, n, PKT, fixed_len=PKT, verdicts=verd, flags=0)
        _, k = bw._timed(dev, step, 10, 3)
        print("%-12s insns %3d  kernel %.4f ms  %.2f ps/pkt  %.3f ps/pkt/insn" %
              (name, ninsn, k * 1e3, k / n * 1e12, k / n / ninsn * 1e12), flush=True)


if __name__ == "__main__":
    main()
