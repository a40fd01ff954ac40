"""Times the syscall dispatch plans on the device: syscount's latency pair
(thread-ordered: sys_enter writes start[tid], sys_exit reads it) over 128-B
records from T threads, and the same records with syscount's exit program
alone (program-major).  One JSON line per case: records / s of the whole
dispatch (grouping included), and of the k_sys_seq launch alone.

  python tools/sys_threads_time.py [--n 22] [--threads 64,4096,65536]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from bpftime_amd import _lib, gen, isa, programs, vm as dev  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=22)
    ap.add_argument("--threads", default="64,1024,65536")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--progs", default="syscount", choices=["syscount", "trivial", "pid", "lookup"],
                    help="trivial: r0 = 0 programs (the per-call overhead); pid: + a helper call; lookup: + "
                         "one hash lookup")
    a = ap.parse_args()
    n = 1 << a.n
    for t in [int(x) for x in a.threads.split(",")]:
        for pair in (True, False):
            dev.reset_runtime()
            dev.set_ncpu(64)
            start = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 8, max(10240, 2 * t))
            data = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 10240)
            ro = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1)
            ro.update(b"\0" * 4, programs.syscount_rodata(measure_latency=pair))
            if a.progs == "syscount":
                enter_c = programs.syscount_enter(start.fd, ro.fd)
                exit_c = programs.syscount_exit(data.fd, ro.fd, start.fd if pair else -1)
            else:
                from bpftime_amd.isa import Asm
                body = {"trivial": lambda x: x,
                        "pid": lambda x: x.call(isa.BPF_FUNC_get_current_pid_tgid),
                        "lookup": lambda x: x.call(isa.BPF_FUNC_get_current_pid_tgid).stx(4, 10, -4, "r0")
                        .ld_map_fd(1, start.fd).mov64(2, "r10").add64(2, -4).call(isa.BPF_FUNC_map_lookup_elem)}
                enter_c = body[a.progs](Asm()).mov64(0, 0).exit().assemble()
                # (the exit writes start: the pair does not commute, thread-ordered)
                exit_c = body[a.progs](Asm()).st(4, 10, -4, 1).st(8, 10, -16, 0).ld_map_fd(1, start.fd) \
                    .mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -16).mov64(4, 0) \
                    .call(isa.BPF_FUNC_map_update_elem).mov64(0, 0).exit().assemble() if a.progs != "trivial" \
                    else Asm().mov64(0, 0).exit().assemble()
            if pair:
                dev.syscall_attach(dev.prog_create(enter_c, "e", 5), -1, True)
            dev.syscall_attach(dev.prog_create(exit_c, "x", 5), -1, False)
            recs = gen.syscall_records_timed(n, threads=t)
            d = dev.DeviceBuffer.from_array(recs)
            plan = dev.syscall_dispatch_plan(dev.DISPATCH_THREADS if a.progs != "syscount" else 0)
            best = 1e9
            for _ in range(a.reps):
                _lib.lib().bpftime_amd_sync()
                t0 = time.perf_counter()
                dev.syscall_dispatch(d, n, record_size=dev.SYSCALL_RECORD_TIMED,
                                     flags=dev.BATCH_SYNC | (dev.DISPATCH_THREADS if pair and a.progs != "syscount"
                                                             else 0))
                _lib.lib().bpftime_amd_sync()
                best = min(best, time.perf_counter() - t0)
            print(json.dumps({"case": ("%s pair" if pair else "%s exit only") % a.progs, "records": n,
                              "threads": t, "plan": "threads" if plan else "programs", "ms": round(best * 1e3, 3),
                              "Mrec_per_s": round(n / best / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
