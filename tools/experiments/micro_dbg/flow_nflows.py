"""flow-hash steady-state kernel time by flow count (the lookup cache's
reach): the bench's program and frames with 256 .. 65536 Zipf(1.1) flows in a
65536-entry table; BPFTIME_AMD_DBG=512 lookup-cache hit rate beside.
python tools/experiments/micro_dbg/flow_nflows.py [log2n]"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
import bench_workloads as bw  # noqa: E402
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 24)
stride = 2048
pk = dev.DeviceBuffer(n * stride)
dl = dev.DeviceBuffer(4 * n)
dv = dev.DeviceBuffer(4 * n)
for nflows in (256, 2048, 8192, 65536):
    dev.reset_runtime()
    flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, 65536, name="flows")
    vm = dev.VM()
    vm.load(programs.flow_hash(flows.fd))
    dcdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(nflows, 1.1))
    if dev.lib().bpftime_amd_gen_flow(pk.ptr, dl.ptr, n, stride, gen.SEED_CFG3, 0, dcdf.ptr, nflows, None):
        raise SystemExit("flow generator failed")

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, stride, lens=dl, verdicts=dv, flags=0)

    step()
    _, k = bw._timed(dev, step, 5, 2)
    print("flows %6d kernel %.4f ms (%d in the table)" % (nflows, k * 1e3, flows.count()), flush=True)
