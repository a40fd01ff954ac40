"""Where the counter-add time goes in syscall-agg (2^22 records, maps warm):
the same lookup with and without the combining table, a value load, a
fused add, an atomic add."""
import os
import sys
sys.path.insert(0, os.getcwd())
from bpftime_amd import gen, isa, programs
from bpftime_amd import vm as dev
from bpftime_amd.isa import Asm
from bpftime_amd.programs import BPF_FUNC_map_lookup_elem

N = 1 << 22


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


def main():
    dev.reset_runtime()
    m = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192)
    side = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 64, 1)
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(335, 1.2))
    recs = dev.DeviceBuffer(N * 64)
    dev.lib().bpftime_amd_gen_syscall(recs.ptr, N, gen.SEED_CFG5, 0, cdf.ptr, 335, None)
    dr = dev.DeviceBuffer(8 * N)

    def look(a):
        return a.ldx(8, 6, 1, 8).stx(4, 10, -4, "r6").ld_map_fd(1, m.fd).mov64(2, "r10") \
                .add64(2, -4).call(BPF_FUNC_map_lookup_elem)

    def dead_comb(a):
        # an add never executed whose target is a map value: forces the table
        a.jmp("jne", 6, 0x7fffffff, "skip").ld_map_fd(1, side.fd).mov64(2, "r10").add64(2, -4) \
         .call(BPF_FUNC_map_lookup_elem).jmp("jeq", 0, 0, "skip").mov64(3, 1) \
         .atomic(8, isa.ATOMIC_ADD, 0, 0, 3).label("skip")
        return a

    variants = {
        "lookup": look(Asm()).mov64(0, 0).exit().assemble(),
        "lookup+table": dead_comb(look(Asm()).mov64(7, "r0")).mov64(0, 0).exit().assemble(),
        "lookup+load": look(Asm()).jmp("jeq", 0, 0, "o").ldx(8, 1, 0, 0).label("o").mov64(0, 0).exit()
                                  .assemble(),
        "lookup+load+table": dead_comb(look(Asm()).jmp("jeq", 0, 0, "o").ldx(8, 1, 0, 0).label("o"))
                             .mov64(0, 0).exit().assemble(),
        "lookup+rmw": look(Asm()).jmp("jeq", 0, 0, "o").ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, "r1")
                                 .label("o").mov64(0, 0).exit().assemble(),
        "lookup+atomic": look(Asm()).jmp("jeq", 0, 0, "o").mov64(1, 1).atomic(8, isa.ATOMIC_ADD, 0, 0, 1)
                                    .label("o").mov64(0, 0).exit().assemble(),
        "full": programs.syscall_agg(m.fd),
    }
    vm = dev.VM()
    vm.load(programs.syscall_agg(m.fd))
    vm.exec_batch(dev.CTX_SYSCALL, recs, N, 64, rets=dr)
    for name, code in variants.items():
        vm = dev.VM()
        vm.load(code)
        ms = timeit(vm, dev.CTX_SYSCALL, recs, 64, rets=dr)
        print(f"syscall {name:18s} {ms:8.3f} ms {N / ms / 1e3:9.1f} Mrec/s  counters {vm.counter_info(dev.CTX_SYSCALL)}",
              flush=True)


main()


def conflicts():
    """Atomic adds through the table with 1, 4, 64 and 1024 distinct
    addresses (array map, key = args[0] & mask): the cost of LDS
    same-address serialization vs set probing."""
    dev.reset_runtime()
    arr = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 1024)
    cdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(335, 1.2))
    recs = dev.DeviceBuffer(N * 64)
    dev.lib().bpftime_amd_gen_syscall(recs.ptr, N, gen.SEED_CFG5, 0, cdf.ptr, 335, None)
    dr = dev.DeviceBuffer(8 * N)
    for mask in (0, 3, 63, 1023):
        a = Asm().ldx(8, 6, 1, 16).alu64("and", 6, mask).stx(4, 10, -4, "r6").ld_map_fd(1, arr.fd)
        a.mov64(2, "r10").add64(2, -4).call(BPF_FUNC_map_lookup_elem).jmp("jeq", 0, 0, "o")
        a.mov64(1, 1).atomic(8, isa.ATOMIC_ADD, 0, 0, 1).label("o").mov64(0, 0).exit()
        vm = dev.VM()
        vm.load(a.assemble())
        ms = timeit(vm, dev.CTX_SYSCALL, recs, 64, rets=dr)
        print(f"conflict mask {mask:5d} {ms:8.3f} ms {N / ms / 1e3:9.1f} Mrec/s", flush=True)


conflicts()
