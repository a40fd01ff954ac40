"""The linked threaded forms of syscall-agg's sys_enter program and
syscount's sys_exit program (BPFTIME_AMD_DUMP_FAST)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
os.environ["BPFTIME_AMD_DUMP_FAST"] = "1"
import numpy as np  # noqa: E402
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

dev.reset_runtime()
counts = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192)
vm = dev.VM()
vm.load(programs.syscall_agg(counts.fd))
n = 1 << 16
recs = dev.DeviceBuffer.from_array(gen.syscall_records(n))
print("---- syscall-agg", file=sys.stderr)
vm.exec_batch(dev.CTX_SYSCALL, recs, n, 64, flags=dev.BATCH_SYNC)
data = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192)
ro = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1)
ro.update(b"\0" * 4, programs.syscount_rodata())
pfd = dev.prog_create(programs.syscount_exit(data.fd, ro.fd), "sys_exit", 5)
dev.syscall_attach(pfd, -1, enter=False)
full = dev.DeviceBuffer.from_array(gen.syscall_records_full(n))
print("---- syscount", file=sys.stderr)
dev.syscall_dispatch(full, n, flags=dev.BATCH_SYNC)
