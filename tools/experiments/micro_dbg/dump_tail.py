import os, struct, sys
sys.path.insert(0, "/root/repo")
os.environ["BPFTIME_AMD_DUMP_FAST"] = "1"
import numpy as np
from bpftime_amd import isa, programs
from bpftime_amd import vm as dev
dev.reset_runtime()
pa = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, name="jmp_table")
cnt = dev.Map(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 4, name="counts")
targets = {0: programs.tail_target_write(0xA1), 1: programs.tail_target_count(cnt.fd),
           3: programs.tail_target_recurse(pa.fd, cnt.fd, 0)}
for k, code in targets.items():
    pa.update(struct.pack("<i", k), struct.pack("<i", dev.prog_create(code, "t%d" % k, 6)))
vm = dev.VM()
vm.load(programs.tail_xdp_caller(pa.fd, cnt.fd))
n = 64
pk = dev.DeviceBuffer.from_array(np.zeros((n, 64), np.uint8))
dv = dev.DeviceBuffer(4 * n)
vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0, ifindex=5)
