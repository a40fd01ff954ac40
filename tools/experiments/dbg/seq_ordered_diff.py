"""Debug: the EBPF_BATCH_ORDERED cross-thread pair (test_gpu_syscall_threads
_shared_last) through the asm / C++ tiers vs the oracle, by batch size."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import numpy as np  # noqa: E402

from bpftime_amd import gen, isa, vm as dev  # noqa: E402
from bpftime_amd.isa import Asm  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

ARRAY = isa.BPF_MAP_TYPE_ARRAY


def run(asm, n, variant):
    os.environ["BPFTIME_AMD_SEQ_ASM"] = asm
    dev.reset_runtime()
    po.reset()
    dlast = dev.Map(ARRAY, 4, 16, 1)
    olast = po.OracleMap(ARRAY, 4, 16, 1, fd=dlast.fd)
    enter = Asm().ldx(8, 3, 1, 24).ld_map_value(2, dlast.fd, 0).stx(8, 2, 0, "r3").mov64(0, 0).exit().assemble()
    if variant == "atomic":
        exit_ = (Asm().ldx(8, 4, 1, 16).alu64("or", 4, 1).ld_map_value(2, dlast.fd, 0).ldx(8, 3, 2, 0)
                 .alu64("mul", 3, "r4").atomic(8, isa.ATOMIC_ADD, 2, 8, 3).mov64(0, 0).exit().assemble())
    elif variant == "store":   # exit stores last * (ret | 1) at +8 (no atomic)
        exit_ = (Asm().ldx(8, 4, 1, 16).alu64("or", 4, 1).ld_map_value(2, dlast.fd, 0).ldx(8, 3, 2, 0)
                 .alu64("mul", 3, "r4").stx(8, 2, 8, "r3").mov64(0, 0).exit().assemble())
    else:                      # exit copies last to +8
        exit_ = (Asm().ld_map_value(2, dlast.fd, 0).ldx(8, 3, 2, 0)
                 .stx(8, 2, 8, "r3").mov64(0, 0).exit().assemble())
    o = po.OracleSyscallDispatch()
    for c, e in ((enter, True), (exit_, False)):
        dev.syscall_attach(dev.prog_create(c, "p", 5), -1, e)
        o.attach(c, -1, e)
    recs = gen.syscall_records_timed(n, threads=16)
    d = dev.DeviceBuffer.from_array(recs)
    rc = dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED,
                              flags=dev.BATCH_SYNC | dev.BATCH_ORDERED)
    o.dispatch(recs)
    g, w = dlast.lookup(b"\0" * 4), olast.lookup(b"\0" * 4)
    return rc, g == w, g.hex(), w.hex()


if __name__ == "__main__":
    for variant in ("copy", "store", "atomic"):
        for asm in ("0", "1"):
            first = None
            for n in (1, 2, 3, 4, 5, 8, 16, 64, 256, 4096):
                rc, ok, g, w = run(asm, n, variant)
                if not ok and first is None:
                    first = (n, g, w)
            print(variant, "asm", asm, "first mismatch", first, flush=True)
