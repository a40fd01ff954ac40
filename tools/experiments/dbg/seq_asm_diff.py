"""Debug: the thread-ordered syscount pair with the asm tier vs the C++ tier
vs the oracle, at a small size; prints the first mismatching records."""
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))), "tests"))
import numpy as np  # noqa: E402

from bpftime_amd import gen, isa, programs, vm as dev  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

HASH, ARRAY = isa.BPF_MAP_TYPE_HASH, isa.BPF_MAP_TYPE_ARRAY


def run(asm, n, threads, progs):
    os.environ["BPFTIME_AMD_SEQ_ASM"] = asm
    dev.reset_runtime()
    po.reset()
    maps = []
    for t, k, v, m in [(HASH, 4, 8, 10240), (HASH, 4, 32, 10240), (ARRAY, 4, programs.SYSCOUNT_RODATA, 1)]:
        d = dev.Map(t, k, v, m)
        o = po.OracleMap(t, k, v, m, fd=d.fd)
        maps.append((o, d))
    (ostart, dstart), (odata, ddata), (oro, dro) = maps
    ro = programs.syscount_rodata(measure_latency=True)
    oro.update(b"\0" * 4, ro)
    dro.update(b"\0" * 4, ro)
    o = po.OracleSyscallDispatch()
    if progs == "syscount":
        codes = [(programs.syscount_enter(dstart.fd, dro.fd), True),
                 (programs.syscount_exit(ddata.fd, dro.fd, dstart.fd), False)]
    else:
        codes = [(isa.Asm().mov64(0, 0).exit().assemble(), True), (isa.Asm().mov64(0, 0).exit().assemble(), False)]
    for c, e in codes:
        dev.syscall_attach(dev.prog_create(c, "p", 5), -1, e)
        o.attach(c, -1, e)
    recs = gen.syscall_records_timed(n, threads=threads)
    d = dev.DeviceBuffer.from_array(recs)
    out = dev.DeviceBuffer(8 * n)
    rc = dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, out=out,
                              flags=dev.BATCH_SYNC | dev.DISPATCH_THREADS)
    got = out.download(np.int64)
    want = o.dispatch(recs)
    w = recs.view(np.int64).reshape(n, 16)
    bad = np.nonzero(got != want)[0]
    print("asm", asm, progs, "rc", rc, "out mismatches", len(bad), "of", n)
    for i in bad[:8]:
        print("  rec", i, "nr", w[i, 1], "exit nr", w[i, 9], "ret", w[i, 10], "pid", hex(w[i, 11]), "got", got[i],
              "want", want[i])
    di, oi = ddata.hash_items(), odata.items()
    print("  data equal", di == oi, len(di), len(oi))
    for k in sorted(set(oi) | set(di))[:6]:
        if di.get(k) != oi.get(k):
            print("   key", k.hex(), "dev", (di.get(k) or b"")[:16].hex(), "ora", (oi.get(k) or b"")[:16].hex())
    si, so = dstart.hash_items(), ostart.items()
    print("  start equal", si == so, len(si), len(so))


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 12
    for progs in ("trivial", "syscount"):
        for asm in ("0", "1"):
            run(asm, n, 64, progs)
