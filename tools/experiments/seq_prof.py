"""Where a thread-ordered syscall dispatch spends its time: k_sys_seq built
with -DBPFTIME_AMD_SEQ_PROF (interp.hip: clock64 sums per region, per wave),
run through BPFTIME_AMD_LIB=ab/seqprof.so over syscount's latency pair (or
the tools/sys_threads_time.py probes), printed as cycles per record of a
wave.

  BPFTIME_AMD_LIB=$PWD/ab/seqprof.so python tools/experiments/seq_prof.py --threads 64 --n 18
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from bpftime_amd import _lib, gen, isa, programs, vm as dev  # noqa: E402

NAMES = ["wave total", "record + ctx build", "interpret (run_loop)", "helper 1 lookup", "helper 2 update",
         "helper 5/14 (registers)", "other helpers", "record tail", "callbacks", "uniform runs",
         "divergent runs", "n lookup", "n update", "n 5/14", "n other", "steps (lane 0)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=18)
    ap.add_argument("--threads", type=int, default=64)
    ap.add_argument("--progs", default="syscount", choices=["syscount", "trivial"])
    a = ap.parse_args()
    n = 1 << a.n
    lib = _lib.lib()
    fn = lib.bpftime_amd_seq_prof
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev.reset_runtime()
    dev.set_ncpu(64)
    start = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 8, max(10240, 2 * a.threads))
    data = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 10240)
    ro = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1)
    ro.update(b"\0" * 4, programs.syscount_rodata(measure_latency=True))
    if a.progs == "syscount":
        enter_c = programs.syscount_enter(start.fd, ro.fd)
        exit_c = programs.syscount_exit(data.fd, ro.fd, start.fd)
    else:
        enter_c = exit_c = isa.Asm().mov64(0, 0).exit().assemble()
    dev.syscall_attach(dev.prog_create(enter_c, "e", 5), -1, True)
    dev.syscall_attach(dev.prog_create(exit_c, "x", 5), -1, False)
    recs = gen.syscall_records_timed(n, threads=a.threads)
    d = dev.DeviceBuffer.from_array(recs)
    flags = dev.BATCH_SYNC | dev.DISPATCH_THREADS
    dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, flags=flags)
    buf = (ctypes.c_ulonglong * 32)()
    fn(buf, 1)
    dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED, flags=flags)
    fn(buf, 0)
    waves = buf[16]
    per_rec = n / max(1, a.threads)
    out = {"progs": a.progs, "records": n, "threads": a.threads, "waves": waves,
           "records_per_lane": per_rec}
    for i, nm in enumerate(NAMES):
        v = buf[i] / max(1, waves)
        out[nm] = round(v / per_rec, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
