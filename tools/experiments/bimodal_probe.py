"""Headline kernel time per fresh packet-buffer allocation in one process
(is the fast / slow mode a property of the buffer's placement?).
    python tools/experiments/bimodal_probe.py [allocs] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

allocs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
PKT, n = 64, 1 << 24
dev.lib().bpftime_amd_set_device(0)
dev.reset_runtime()
ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array")
bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, flags=isa.BPF_F_MMAPABLE, name=".bss")
vm = dev.VM()
vm.load(programs.xdp_counter(ctl.fd, bss.fd))
keep = []
pad = int(os.environ.get("PAD_MB", "0"))
pre = int(os.environ.get("PRE_MB", "0"))
if pre:
    keep.append(dev.DeviceBuffer(pre << 20))  # allocated before every packet buffer
for a in range(allocs):
    if pad:
        keep.append(dev.DeviceBuffer(pad << 20))  # shift the next allocation
    pkts = dev.DeviceBuffer(n * PKT)
    verd = dev.DeviceBuffer(4 * n)
    dev.lib().bpftime_amd_gen_xdp(pkts.ptr, n, PKT, PKT, gen.SEED_CFG2, 0, None)
    for _ in range(5):
        vm.exec_batch(dev.CTX_XDP, pkts, n, PKT, fixed_len=PKT, verdicts=verd)
    dev.lib().bpftime_amd_sync()
    res = []
    for rep in range(3):
        e0, e1 = dev.Event(), dev.Event()
        e0.record()
        for _ in range(steps):
            vm.exec_batch(dev.CTX_XDP, pkts, n, PKT, fixed_len=PKT, verdicts=verd)
        e1.record()
        dev.lib().bpftime_amd_sync()
        res.append(e0.elapsed_ms(e1) / steps)
    print(f"alloc {a} pkts 0x{pkts.ptr:x} verd 0x{verd.ptr:x} ms " + " ".join(f"{x:.4f}" for x in res), flush=True)
    keep.append((pkts, verd))
