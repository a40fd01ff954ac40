"""The linked threaded form of the flow-hash program (BPFTIME_AMD_DUMP_FAST)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
os.environ["BPFTIME_AMD_DUMP_FAST"] = "1"
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

dev.reset_runtime()
flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, 65536)
vm = dev.VM()
vm.load(programs.flow_hash(flows.fd))
n = 4096
pk, lens = gen.flow_packets(n, nflows=4096, stride=2048)
d = dev.DeviceBuffer.from_array(pk)
ld = dev.DeviceBuffer.from_array(lens)
v = dev.DeviceBuffer(4 * n)
vm.exec_batch(dev.CTX_XDP, d, n, 2048, lens=ld, verdicts=v)
