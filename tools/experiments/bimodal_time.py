"""Headline kernel time over wall time in one process, one allocation
(does the rate change as the GPU keeps running?).
    python tools/experiments/bimodal_time.py [blocks] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 20
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
PKT, n = 64, 1 << 24
dev.lib().bpftime_amd_set_device(0)
dev.reset_runtime()
ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array")
bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, flags=isa.BPF_F_MMAPABLE, name=".bss")
vm = dev.VM()
vm.load(programs.xdp_counter(ctl.fd, bss.fd))
pkts = dev.DeviceBuffer(n * PKT)
verd = dev.DeviceBuffer(4 * n)
dev.lib().bpftime_amd_gen_xdp(pkts.ptr, n, PKT, PKT, gen.SEED_CFG2, 0, None)
t0 = time.perf_counter()
idle = float(os.environ.get("IDLE_S", "0"))
for b in range(blocks):
    e0, e1 = dev.Event(), dev.Event()
    e0.record()
    for _ in range(steps):
        vm.exec_batch(dev.CTX_XDP, pkts, n, PKT, fixed_len=PKT, verdicts=verd)
    e1.record()
    dev.lib().bpftime_amd_sync()
    print(f"t {time.perf_counter() - t0:7.3f} s  ms {e0.elapsed_ms(e1) / steps:.4f}", flush=True)
    if idle and b == blocks // 2:
        time.sleep(idle)
