"""Debug timing: flow-hash over a PERCPU_HASH map on the device."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
import numpy as np
from bpftime_amd import vm as dev, isa, gen, programs

dev.lib().bpftime_amd_set_device(0)
for log2n, nflows in ((14, 65536), (16, 65536), (18, 65536), (18, 4096)):
    n = 1 << log2n
    slots, lens = gen.flow_packets(n, nflows=nflows, stride=2048)
    for mtype in (isa.BPF_MAP_TYPE_HASH, isa.BPF_MAP_TYPE_PERCPU_HASH):
        dev.reset_runtime()
        dev.set_ncpu(64)
        m = dev.Map(mtype, 16, 16, 65536)
        vm = dev.VM()
        vm.load(programs.flow_hash(m.fd))
        d = dev.DeviceBuffer.from_array(slots)
        dl = dev.DeviceBuffer.from_array(lens)
        dv = dev.DeviceBuffer(4 * n)
        t = time.time()
        vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=dl, verdicts=dv)
        t1 = time.time() - t
        t = time.time()
        vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=dl, verdicts=dv)
        t2 = time.time() - t
        t = time.time()
        it = m.hash_items()
        print(f"n=2^{log2n} flows={nflows} type={mtype}: first {t1*1e3:.1f} ms, second {t2*1e3:.1f} ms, "
              f"items {len(it)} in {time.time()-t:.2f} s", flush=True)
