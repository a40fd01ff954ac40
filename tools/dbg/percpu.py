import sys, os, struct
sys.path.insert(0, os.getcwd())
import numpy as np
from bpftime_amd import gen, isa
from bpftime_amd import vm as dev
from bpftime_amd.isa import Asm

def run(fuse, ordered, uniform_key, ncpu=8, n=5000):
    dev.reset_runtime(); dev.set_ncpu(ncpu)
    m = dev.Map(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 4)
    a = Asm()
    a.ldx(8, 6, 1, 0)
    a.alu64("and", 6, 0 if uniform_key else 3).stx(4, 10, -4, "r6")
    a.ld_map_fd(1, m.fd).mov64(2, "r10").add64(2, -4).call(1)
    a.jmp("jeq", 0, 0, "out")
    a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, "r1")
    if not fuse:
        a.mov64(7, "r1")
    a.call(isa.BPF_FUNC_get_smp_processor_id)
    a.label("out").exit()
    vm = dev.VM(); vm.load(a.assemble())
    units = gen.sm64(8, np.arange(n, dtype=np.uint64)).view(np.uint8).reshape(n, 8)
    d = dev.DeviceBuffer.from_array(units); dr = dev.DeviceBuffer(8 * n)
    fl = dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0)
    f = vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr, flags=fl)
    tot = sum(sum(struct.unpack("<%dQ" % ncpu, m.lookup(struct.pack("<i", k)))) for k in range(4))
    print(f"fuse={fuse} ordered={ordered} ukey={uniform_key} fused={vm.info()['fused_rmw']} failed={f} total={tot} (expect {n})", flush=True)

for fuse in (True, False):
    for ordered in (False, True):
        for uk in (True, False):
            run(fuse, ordered, uk)
