"""Insert-path counters of flow-hash's cold launch (an experiment build made
with -DBPFTIME_AMD_INSERT_STATS, dev_helpers.hpp ISTAT):
    BPFTIME_AMD_LIB=ab/istats.so python tools/experiments/insert_stats.py [log2n]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bpftime_amd import gen, isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n, stride, nflows = 1 << log2n, 2048, 65536
dev.lib().bpftime_amd_set_device(0)
dev.reset_runtime()
names = ["inserts", "bitmap_words", "claim_fail", "res_wait_trips", "max_words", "find_insert_calls",
         "find_lookup_calls", "index_steps"]
f = dev.lib().bpftime_amd_insert_stats
f.argtypes = [C.POINTER(C.c_uint64)]
out = (C.c_uint64 * 8)()
for rep in range(2):
    flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, nflows, name="flows")
    vm = dev.VM()
    vm.load(programs.flow_hash(flows.fd))
    dcdf = dev.DeviceBuffer.from_array(gen.zipf_cdf(nflows, 1.1))
    pk = dev.DeviceBuffer(n * stride)
    dl = dev.DeviceBuffer(4 * n)
    dev.lib().bpftime_amd_gen_flow(pk.ptr, dl.ptr, n, stride, gen.SEED_CFG3, 0, dcdf.ptr, nflows, None)
    dv = dev.DeviceBuffer(4 * n)
    f(out)
    vm.exec_batch(dev.CTX_XDP, pk, n, stride, lens=dl, verdicts=dv, flags=dev.BATCH_TIMED)
    cold = vm.last_batch_ms()
    f(out)
    print("cold ms %.3f flows %d" % (cold, flows.count()), {k: out[i] for i, k in enumerate(names)}, flush=True)
    vm.exec_batch(dev.CTX_XDP, pk, n, stride, lens=dl, verdicts=dv, flags=dev.BATCH_TIMED)
    warm = vm.last_batch_ms()
    f(out)
    print("warm ms %.3f" % warm, {k: out[i] for i, k in enumerate(names)}, flush=True)
    for b in (pk, dl, dv, dcdf):
        b.free()
    vm.close()
    flows.close()
