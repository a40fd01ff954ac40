"""Tail-call line cost by lane pattern: the bench's jump table over 2^24
64-B frames whose first byte (the slot) is the same for every frame (u0..u3),
the same within each wave but random across waves (wave), or random per frame
(rand, the bench).  Kernel ms per launch (HIP events).
python tools/experiments/micro_dbg/tail_cost.py [log2n]"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
import bench_workloads as bw  # noqa: E402
from bpftime_amd import isa, programs  # noqa: E402
from bpftime_amd import vm as dev  # noqa: E402

n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 24)
dev.reset_runtime()
pa = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, name="jmp_table")
cnt = dev.Map(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 4, name="counts")
targets = {0: programs.tail_target_write(0xA1), 1: programs.tail_target_count(cnt.fd),
           3: programs.tail_target_recurse(pa.fd, cnt.fd, 0)}
for k, code in targets.items():
    pa.update(struct.pack("<i", k), struct.pack("<i", dev.prog_create(code, "t%d" % k, 6)))
vm = dev.VM()
vm.load(programs.tail_xdp_caller(pa.fd, cnt.fd))
rng = np.random.default_rng(5)
pats = {"u0": np.zeros(n, np.uint8), "u1": np.ones(n, np.uint8), "u2": np.full(n, 2, np.uint8),
        "u3": np.full(n, 3, np.uint8), "wave": np.repeat(rng.integers(0, 4, n // 64).astype(np.uint8), 64),
        "rand": rng.integers(0, 4, n).astype(np.uint8)}
frames = np.zeros((n, 64), np.uint8)
pk = dev.DeviceBuffer(n * 64)
dv = dev.DeviceBuffer(4 * n)


class A:
    steps, warmup = 5, 2


for name, b0 in pats.items():
    frames[:, 0] = b0
    pk = dev.DeviceBuffer.from_array(frames)

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0, ifindex=5)

    wall, kern_s = bw._timed(dev, step, A.steps, A.warmup)
    print("%-5s kernel %.4f ms" % (name, kern_s * 1e3), flush=True)

# slot 0 -> a two-instruction target: the push / pop round trip alone
triv = isa.Asm().mov64(0, 0).exit().assemble()
pa.update(struct.pack("<i", 0), struct.pack("<i", dev.prog_create(triv, "triv", 6)))
for name in ("u0", "rand"):
    frames[:, 0] = pats[name]
    pk = dev.DeviceBuffer.from_array(frames)

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0, ifindex=5)

    wall, kern_s = bw._timed(dev, step, A.steps, A.warmup)
    print("%-5s trivial slot 0: kernel %.4f ms" % (name, kern_s * 1e3), flush=True)
