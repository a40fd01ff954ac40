"""Debug: per-CPU flow-hash, 8 shards vs one batch vs the oracle (first differences)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
import numpy as np
from bpftime_amd import vm as dev, isa, gen, programs, shard
from oracle import pyoracle as po

dev.lib().bpftime_amd_set_device(0)
LOG2N = int(os.environ.get("LOG2N", "18"))
n = 1 << LOG2N
ncpu = 64
slots, lens = gen.flow_packets(n, nflows=65536, stride=2048)
for mtype in (isa.BPF_MAP_TYPE_HASH, isa.BPF_MAP_TYPE_PERCPU_HASH):
    def run(first, cnt):
        dev.reset_runtime()
        dev.set_ncpu(ncpu)
        flows = dev.Map(mtype, 16, 16, 65536, fd=5)
        vm = dev.VM()
        vm.load(programs.flow_hash(flows.fd))
        d = dev.DeviceBuffer.from_array(slots[first:first + cnt])
        dl = dev.DeviceBuffer.from_array(lens[first:first + cnt])
        dv = dev.DeviceBuffer(4 * cnt)
        vm.exec_batch(dev.CTX_XDP, d, cnt, 2048, lens=dl, verdicts=dv, first_unit=first)
        return dv.download(np.uint32), flows.hash_items()
    items = [run(f, c)[1] for f, c in (shard.shard_range(n, 8, g) for g in range(8))]
    merged = shard.merge_hash_additive({}, items, 65536, width=8)
    _, full = run(0, n)
    po.reset(); po.set_ncpu(ncpu)
    om = po.OracleMap(mtype, 16, 16, 65536, fd=5)
    ovm = po.OracleVM(); ovm.load(programs.flow_hash(om.fd))
    ovm.run_xdp(slots.copy(), lens=lens, ncpu=ncpu)
    oi = om.items()
    print(mtype, "keys merged/full/oracle", len(merged), len(full), len(oi),
          "merged==full", merged == full, "full==oracle", full == oi, "merged==oracle", merged == oi, flush=True)
    for name, a, b in (("merged-full", merged, full), ("full-oracle", full, oi), ("merged-oracle", merged, oi)):
        bad = [k for k in set(a) | set(b) if a.get(k) != b.get(k)]
        print(" ", name, "differing keys", len(bad))
        for k in bad[:3]:
            va = np.frombuffer(a.get(k, b""), np.uint64)
            vb = np.frombuffer(b.get(k, b""), np.uint64)
            if len(va) == len(vb):
                idx = np.nonzero(va != vb)[0]
                print("    key", k.hex(), "words", idx[:8].tolist(), "a", va[idx[:8]].tolist(), "b", vb[idx[:8]].tolist())
            else:
                print("    key", k.hex(), "sizes", len(va), len(vb))
