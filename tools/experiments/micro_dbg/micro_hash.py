"""Where the time goes in the hash workloads (configs 3 and 5 shapes, 2^22
units, device-resident, maps warmed by one full run first)."""
import os
import sys
sys.path.insert(0, os.getcwd())
import numpy as np
from bpftime_amd import gen, isa, programs
from bpftime_amd import vm as dev
from bpftime_amd.isa import Asm
from bpftime_amd.programs import BPF_FUNC_map_lookup_elem

N = 1 << int(os.environ.get("LOG2N", "22"))


def timeit(vm, kind, buf, stride, steps=10, **kw):
    for _ in range(2):
        vm.exec_batch(kind, buf, N, stride, flags=0, **kw)
    dev.lib().bpftime_amd_sync()
    e0, e1 = dev.Event(), dev.Event()
    e0.record()
    for _ in range(steps):
        vm.exec_batch(kind, buf, N, stride, flags=0, **kw)
    e1.record()
    return e0.elapsed_ms(e1) / steps


def syscall():
    dev.reset_runtime()
    m = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192)
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(335, 1.2))
    recs = dev.DeviceBuffer(N * 64)
    dev.lib().bpftime_amd_gen_syscall(recs.ptr, N, gen.SEED_CFG5, 0, cdf.ptr, 335, None)
    dr = dev.DeviceBuffer(8 * N)
    full = programs.syscall_agg(m.fd)
    variants = {
        "r0=0": Asm().mov64(0, 0).exit().assemble(),
        "ids+lookup": Asm().ldx(8, 6, 1, 8).stx(4, 10, -4, "r6").ld_map_fd(1, m.fd).mov64(2, "r10")
                           .add64(2, -4).call(BPF_FUNC_map_lookup_elem).mov64(0, 0).exit().assemble(),
        "lookup+count": Asm().ldx(8, 6, 1, 8).stx(4, 10, -4, "r6").ld_map_fd(1, m.fd).mov64(2, "r10")
                             .add64(2, -4).call(BPF_FUNC_map_lookup_elem).jmp("jeq", 0, 0, "o")
                             .ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, "r1").label("o").mov64(0, 0).exit()
                             .assemble(),
        "full": full,
    }
    vm = dev.VM(); vm.load(full)
    vm.exec_batch(dev.CTX_SYSCALL, recs, N, 64, rets=dr)
    for name, code in variants.items():
        vm = dev.VM(); vm.load(code)
        ms = timeit(vm, dev.CTX_SYSCALL, recs, 64, rets=dr)
        print(f"syscall {name:14s} {ms:8.3f} ms {N / ms / 1e3:9.1f} Mrec/s", flush=True)


def flow():
    dev.reset_runtime()
    m = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, 65536)
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(65536, 1.1))
    stride = 2048
    pk = dev.DeviceBuffer(N * stride)
    dl = dev.DeviceBuffer(4 * N)
    dev.lib().bpftime_amd_gen_flow(pk.ptr, dl.ptr, N, stride, gen.SEED_CFG3, 0, cdf.ptr, 65536, None)
    dv = dev.DeviceBuffer(4 * N)
    full = programs.flow_hash(m.fd)
    code = bytearray(full)
    # truncations of flow_hash: stop right before the lookup (r0 = verdict so far)
    n_ins = len(full) // 8
    look = next(i for i in range(n_ins) if full[8 * i] == 0x85)
    parse = bytes(full[:8 * (look - 3)]) + Asm().mov64(0, 3).exit().assemble()
    vm = dev.VM(); vm.load(full)
    vm.exec_batch(dev.CTX_XDP, pk, N, stride, lens=dl, verdicts=dv)
    def patch(code, nop_atomics, no_lookup):
        c = bytearray(code)
        first_call = True
        for i in range(0, len(c), 8):
            if nop_atomics and c[i] == 0xDB:
                c[i:i + 8] = bytes([0xBF, 0x00, 0, 0, 0, 0, 0, 0])      # mov64 r0, r0
            if no_lookup and c[i] == 0x85 and first_call:
                c[i:i + 8] = bytes([0xB7, 0x00, 0, 0, 1, 0, 0, 0])      # mov64 r0, 1
                first_call = False
        return bytes(c)
    for name, c in (("r0=2", Asm().mov64(0, 2).exit().assemble()),
                    ("parse+key", patch(full, True, True)),
                    ("+lookup", patch(full, True, False)),
                    ("full", full)):
        vm = dev.VM(); vm.load(c)
        try:
            ms = timeit(vm, dev.CTX_XDP, pk, stride, lens=dl, verdicts=dv)
        except Exception as e:  # noqa
            print(name, "failed", e)
            continue
        print(f"flow    {name:14s} {ms:8.3f} ms {N / ms / 1e3:9.1f} Mpps", flush=True)


if len(sys.argv) < 2 or sys.argv[1] == "syscall":
    syscall()
if len(sys.argv) < 2 or sys.argv[1] == "flow":
    flow()
