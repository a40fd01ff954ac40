"""Headline benchmark: device-resident Mpps of example/xdp-counter over 64-B
packets (BASELINE.json metric, configs[1] at N=1; configs[3]'s per-GPU shard
at N>1).  One step = one ebpf_exec_batch of the loaded xdp-counter bytecode
over the whole resident batch (2^24 packets per GPU).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PKT = 64
ALGO_BYTES_PER_PKT = 28  # 12 B MAC read + 12 B MAC write + 4 B verdict
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2n", type=int, default=None, help="units per GPU = 2^log2n (xdp-counter: 24)")
    ap.add_argument("--workload", default="xdp-counter", choices=["xdp-counter", "flow-hash", "syscall-agg", "lpm-route", "ringbuf-sample", "tail-call", "syscount",
                             "syscount-latency"],
                    help="xdp-counter is the headline (BASELINE metric); the others are configs[2]/[4] "
                         "(bench_workloads.py)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline budget per leg (1 core, all cores; rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--unchecked", action="store_true", help="skip the global-window check")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe-inclusive) leg")
    ap.add_argument("--e2e-chunk-log2", type=int, default=20, help="packets per H2D chunk = 2^k")
    ap.add_argument("--e2e-streams", type=int, default=3, help="streams the host-memory leg rotates over")
    args = ap.parse_args()
    args.log2n_set = args.log2n is not None
    if args.log2n is None:
        args.log2n = 24
    return args


def main():
    args = parse()
    if args.workload != "xdp-counter":
        from bench_workloads import run
        run(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    rz = None
    if world > 1:
        # control plane only (barrier, timing max, map-shard gather) through
        # files, with no torch import: torch would load its own HIP runtime,
        # and every rank count must run the kernel on the library's
        # (bpftime_amd/rendezvous.py); the data path has no collective
        # 
        from bpftime_amd.rendezvous import Rendezvous
        rz = Rendezvous(rank, world)

    import numpy as np

    from bpftime_amd import gen, isa, programs
    from bpftime_amd import vm as dev

    # one process per GPU; ranks beyond the visible GPUs share them round-robin
    # (only to rehearse N>1 on a smaller box: the driver's nodes have one GPU per rank)
    ngpu = dev.lib().bpftime_amd_device_count()
    if ngpu <= 0 or dev.lib().bpftime_amd_set_device(local_rank % ngpu) != 0:
        raise SystemExit(f"rank {rank}: cannot select GPU {local_rank}")

    n = 1 << args.log2n
    first = rank * n  # contiguous shard of the global packet stream (configs[3])
    dev.reset_runtime()
    ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array")
    bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, flags=isa.BPF_F_MMAPABLE, name=".bss")
    code = programs.xdp_counter(ctl.fd, bss.fd)
    vm = dev.VM()
    vm.load(code)
    info = vm.info()

    pkts = dev.DeviceBuffer(n * PKT)
    if dev.lib().bpftime_amd_gen_xdp(pkts.ptr, n, PKT, PKT, gen.SEED_CFG2, first, None) != 0:
        raise SystemExit("generator failed")
    verd = dev.DeviceBuffer(4 * n)
    init_bss = bss.snapshot()
    flags = dev.BATCH_UNCHECKED if args.unchecked else 0

    def step():
        vm.exec_batch(dev.CTX_XDP, pkts, n, PKT, fixed_len=PKT, verdicts=verd, flags=flags, first_unit=first)

    for _ in range(args.warmup):
        step()
    dev.lib().bpftime_amd_sync()
    if rz:
        rz.barrier()
    dev.lib().bpftime_amd_sync()
    # two events on the launch stream bracket the K back-to-back launches (an
    # event between launches would add its own end-of-kernel cache
    # write-back to every step)
    ev0, ev1 = dev.Event(), dev.Event()
    t0 = time.perf_counter()
    ev0.record()
    for i in range(args.steps):
        step()
    ev1.record()
    dev.lib().bpftime_amd_sync()
    t1 = time.perf_counter()
    if rz:
        rz.barrier()
    wall = t1 - t0
    kern_avg_s = ev0.elapsed_ms(ev1) / args.steps / 1e3

    # ---- parity of the timed run (size-independent properties) ----
    total_runs = args.warmup + args.steps
    v = verd.download(np.uint32)
    ok_verdicts = bool((v == isa.XDP_TX).all())
    cnt = np.frombuffer(bss.lookup(b"\0\0\0\0"), dtype=np.uint64)
    ok_counter = int(cnt[0]) == total_runs * n and not cnt[1:].any()
    sample = min(n, 1 << 16)
    ref = gen.xdp_packets(sample, PKT, gen.SEED_CFG2, first)
    got = pkts.download(count=sample * PKT).reshape(sample, PKT)
    exp = ref.copy()
    if total_runs % 2:
        exp[:, :6], exp[:, 6:12] = ref[:, 6:12], ref[:, :6]
    ok_bytes = bool((got == exp).all())

    shard = bss.snapshot()
    e2e = None
    if not args.no_e2e:
        e2e = e2e_leg(dev, vm, bss, n, first, args.e2e_chunk_log2, rz, nstreams=args.e2e_streams)
    hip = dev.hip_runtime()
    gathered = gather_ranks(rz, world, (wall, shard.tobytes(), ok_verdicts and ok_counter and ok_bytes, e2e,
                                        hip["version"]))
    times = [g[0] for g in gathered]
    shards = [np.frombuffer(g[1], dtype=np.uint8) for g in gathered]
    oks = [g[2] for g in gathered]
    e2es = [g[3] for g in gathered]
    hip_versions = sorted({g[4] for g in gathered})
    if rank != 0:
        rz.close()
        return

    merged = merge_counter_shards(init_bss, shards)
    merged_cnt = int(merged.view(np.uint64)[0])
    parity = all(oks) and merged_cnt == world * total_runs * n

    tmax = max(times)
    value = world * n * args.steps / tmax / 1e6
    achieved_gbs = ALGO_BYTES_PER_PKT * n / kern_avg_s / 1e9
    # HBM bytes per launch from the committed PMC pass of this command
    # (tools/prof_workload.sh xdp-counter + tools/pmc_table.py: FETCH_SIZE x2 +
    # WRITE_SIZE), when it was taken at this launch size
    traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_xdp-counter.json")) as f:
            pmc = json.load(f)
        if pmc.get("units") == n:
            traffic = pmc.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        traffic = None

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)

    out = {
        "metric": "device-resident Mpps, 64B pkts, example/xdp-counter XDP prog",
        "value": round(value, 3),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(tmax / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded splitmix64 64-B Eth frames, seed 0x5EED0002)",
        "config": {
            "workload": "example/xdp-counter (hand-assembled, SURVEY.md App. A) over 2^%d device-resident "
                        "64-B packets per GPU, BPF_MAP_TYPE_ARRAY maps (BASELINE configs[1]; configs[3] shards "
                        "at N>1)" % args.log2n,
            "packets_per_gpu": n,
            "pkt_bytes": PKT,
            "parallelism": "dp%d (contiguous packet shards, host-merged map shards, no collective)" % world,
            "interp": {"stack_bytes_per_lane": info["stack_size"], "fused_rmw": info["fused_rmw"],
                       "checked": not args.unchecked},
        },
        "parity": {"verdicts_all_tx": ok_verdicts, "counter_exact": ok_counter, "mac_swap_sample": ok_bytes,
                   "merged_counter": merged_cnt, "ok": parity},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "kernel_avg_ms": round(kern_avg_s * 1e3, 4),
            "algo_bytes_per_pkt": ALGO_BYTES_PER_PKT,
        },
        "cpu_baseline": cpu,
        "e2e": merge_e2e(e2es, world, n),
        "hip_runtime": {"version": hip_versions[0] if len(hip_versions) == 1 else hip_versions, "lib": hip["lib"],
                        "control_plane": "files (bpftime_amd/rendezvous.py)" if rz else None},
    }
    print(json.dumps(out))
    if rz:
        rz.close()


def gather_ranks(rz, world, payload):
    """Every rank's (wall seconds, map shard bytes, parity, e2e, HIP runtime
    version) on every rank: the control plane of bpftime_amd/rendezvous.py,
    no data-path collective."""
    if not rz or world == 1:
        return [payload]
    return rz.all_gather(payload)


def merge_counter_shards(init, shards, width=8):
    """Host merge of the per-GPU map shards: final = init + sum(shard - init),
    counter by counter (xdp-counter's cntrs_array is u64)."""
    from bpftime_amd import shard as sh
    return sh.merge_array_delta(init, shards, width)


def gpu_local_cpus(device):
    """The CPUs of the NUMA node the GPU `device` hangs off (sysfs
    local_cpulist of its PCI function) that this process may use, and that
    node; (None, None) when the box does not say.  The host-memory leg runs
    on them, so its pinned buffers and copy threads sit on the GPU's socket:
    a two-socket box puts half its GPUs behind the other socket, where the
    leg measured 391-394 Mpps against 669-674."""
    import ctypes as C
    try:
        # the HIP runtime this process already mapped (the library's), by path
        with open("/proc/self/maps") as f:
            paths = [ln.split()[-1] for ln in f if "libamdhip64.so" in ln]
        hip = C.CDLL(paths[0] if paths else "libamdhip64.so")
        buf = C.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return None, None
        base = os.path.join("/sys/bus/pci/devices", buf.value.decode().lower())
        with open(os.path.join(base, "local_cpulist")) as f:
            spec = f.read().strip()
        with open(os.path.join(base, "numa_node")) as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        return None, None
    cpus = set()
    for part in spec.split(","):
        lo, _, hi = part.partition("-")
        if lo:
            cpus.update(range(int(lo), int(hi or lo) + 1))
    cpus &= os.sched_getaffinity(0)
    return (cpus or None), node


def e2e_leg(dev, vm, bss, n, first, chunk_log2, rz, passes=3, nstreams=2):
    """The host-memory leg on the GPU's own NUMA node (gpu_local_cpus): the
    process's CPU affinity narrowed to that node's CPUs while it allocates
    and runs, restored after."""
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ngpu = dev.lib().bpftime_amd_device_count()
    cpus, node = gpu_local_cpus(local_rank % max(1, ngpu))
    saved = os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)
    try:
        out = _e2e_leg(dev, vm, bss, n, first, chunk_log2, rz, passes, nstreams)
    finally:
        os.sched_setaffinity(0, saved)
    if isinstance(out, dict):
        out["gpu_numa_node"] = node
        out["cpus_used"] = len(cpus) if cpus else len(saved)
    return out


def _e2e_leg(dev, vm, bss, n, first, chunk_log2, rz, passes=3, nstreams=2):
    """Path that starts and ends in host memory: pinned host frames -> chunked
    hipMemcpyAsync H2D -> interpreter -> verdicts (and, in the second mode,
    the rewritten frames) D2H, double-buffered on two streams.  Reported
    beside `value`, never as it."""
    import ctypes as C

    import numpy as np

    from bpftime_amd import gen, isa
    L = dev.lib()
    chunk = min(n, 1 << chunk_log2)
    nch = n // chunk
    host = L.bpftime_amd_host_alloc(n * PKT)
    hverd = L.bpftime_amd_host_alloc(4 * n)
    if not host or not hverd:
        return {"error": "pinned host allocation failed"}
    dbuf = [dev.DeviceBuffer(chunk * PKT) for _ in range(nstreams)]
    dver = [dev.DeviceBuffer(4 * chunk) for _ in range(nstreams)]
    streams = [L.bpftime_amd_stream_create() for _ in range(nstreams)]
    ev = []
    try:
        for c in range(nch):  # host frames = the same seeded stream as the resident leg
            L.bpftime_amd_gen_xdp(dbuf[0].ptr, chunk, PKT, PKT, gen.SEED_CFG2, first + c * chunk, None)
            L.bpftime_amd_memcpy_dtoh(host + c * chunk * PKT, dbuf[0].ptr, chunk * PKT)
        L.bpftime_amd_sync()

        class _Host:  # pinned host memory handed to the kernel as it is (zero-copy)
            def __init__(self, ptr):
                self.ptr = ptr

        # the pipeline: H2D, the interpreter and D2H on a stream each, chained
        # by events, nbuf device buffers in flight, so chunk k+1's H2D runs
        # under chunk k's D2H (the two PCIe directions overlap; VERDICT r04:
        # one stream per chunk carrying both directions overlapped them
        # barely, 504 Mpps with frames back against 787 verdicts only)
        nbuf = max(3, nstreams)
        pbuf = [dev.DeviceBuffer(chunk * PKT) for _ in range(nbuf)]
        pver = [dev.DeviceBuffer(4 * chunk) for _ in range(nbuf)]
        ps = [L.bpftime_amd_stream_create() for _ in range(3)]
        ev.extend([L.bpftime_amd_event_create() for _ in range(3)] for _ in range(nbuf))
        streams.extend(ps)

        def pipelined(frames_back):
            h2d, comp, d2h = ps
            for c in range(nch):
                b = c % nbuf
                off = c * chunk
                eh, ec, ed = ev[b]
                if c >= nbuf:
                    L.bpftime_amd_stream_wait_event(h2d, ed)     # buffer b drained to the host
                L.bpftime_amd_memcpy_htod_async(pbuf[b].ptr, host + off * PKT, chunk * PKT, h2d)
                L.bpftime_amd_event_record(eh, h2d)
                L.bpftime_amd_stream_wait_event(comp, eh)
                vm.exec_batch(dev.CTX_XDP, pbuf[b], chunk, PKT, fixed_len=PKT, verdicts=pver[b], flags=0,
                              first_unit=first + off, stream=comp)
                L.bpftime_amd_event_record(ec, comp)
                L.bpftime_amd_stream_wait_event(d2h, ec)
                L.bpftime_amd_memcpy_dtoh_async(hverd + off * 4, pver[b].ptr, chunk * 4, d2h)
                if frames_back:
                    L.bpftime_amd_memcpy_dtoh_async(host + off * PKT, pbuf[b].ptr, chunk * PKT, d2h)
                L.bpftime_amd_event_record(ed, d2h)
            for s in ps:
                L.bpftime_amd_stream_sync(s)

        def one_pass(frames_back, zero_copy=False, pipeline=False):
            if pipeline:
                pipelined(frames_back)
                return
            if zero_copy:
                # the kernel reads the frames from pinned host memory over PCIe
                # and rewrites them there, verdicts straight to host memory: no
                # copies (an AF_XDP umem in host memory, processed in place)
                vm.exec_batch(dev.CTX_XDP, _Host(host), n, PKT, fixed_len=PKT, verdicts=_Host(hverd), flags=0,
                              first_unit=first, stream=streams[0])
                L.bpftime_amd_stream_sync(streams[0])
                return
            for c in range(nch):
                b, s = c % nstreams, streams[c % nstreams]
                off = c * chunk
                L.bpftime_amd_memcpy_htod_async(dbuf[b].ptr, host + off * PKT, chunk * PKT, s)
                vm.exec_batch(dev.CTX_XDP, dbuf[b], chunk, PKT, fixed_len=PKT, verdicts=dver[b], flags=0,
                              first_unit=first + off, stream=s)
                L.bpftime_amd_memcpy_dtoh_async(hverd + off * 4, dver[b].ptr, chunk * 4, s)
                if frames_back:
                    L.bpftime_amd_memcpy_dtoh_async(host + off * PKT, dbuf[b].ptr, chunk * PKT, s)
            for s in streams:
                L.bpftime_amd_stream_sync(s)

        out = {"chunk_packets": chunk, "streams": nstreams, "pipeline_buffers": nbuf, "passes": passes}
        c0 = int(np.frombuffer(bss.lookup(b"\0\0\0\0"), dtype=np.uint64)[0])
        modes = (("verdicts_out", False, False, True), ("frames_and_verdicts_out", True, False, True),
                 ("zero_copy", True, True, False), ("verdicts_out_rr", False, False, False),
                 ("frames_and_verdicts_out_rr", True, False, False))
        for mode, back, zc, pl in modes:
            one_pass(back, zc, pl)  # warm-up
            if rz:
                rz.barrier()
            t0 = time.perf_counter()
            for _ in range(passes):
                one_pass(back, zc, pl)
            out[mode + "_s"] = (time.perf_counter() - t0) / passes
        c1 = int(np.frombuffer(bss.lookup(b"\0\0\0\0"), dtype=np.uint64)[0])
        hv = np.ctypeslib.as_array(C.cast(hverd, C.POINTER(C.c_uint32)), shape=(n,))
        out["ok"] = bool((hv == isa.XDP_TX).all()) and c1 - c0 == len(modes) * (passes + 1) * n
        return out
    finally:
        for s in streams:
            L.bpftime_amd_stream_destroy(s)
        for row in ev:
            for e in row:
                L.bpftime_amd_event_destroy(e)
        L.bpftime_amd_host_free(host)
        L.bpftime_amd_host_free(hverd)


def merge_e2e(e2es, world, n):
    if any(e is None or "error" in e for e in e2es):
        return next((e for e in e2es if e is not None), None)
    out = {"unit": "Mpps", "chunk_packets": e2es[0]["chunk_packets"], "streams": e2es[0]["streams"],
           "ok": all(e["ok"] for e in e2es)}
    for mode in ("verdicts_out", "frames_and_verdicts_out", "zero_copy", "verdicts_out_rr",
                 "frames_and_verdicts_out_rr"):
        t = max(e[mode + "_s"] for e in e2es)
        out[mode] = round(world * n / t / 1e6, 3)
    out["gpu_numa_nodes"] = [e.get("gpu_numa_node") for e in e2es]
    out["cpus_used"] = [e.get("cpus_used") for e in e2es]
    out["note"] = ("on the CPUs of each GPU's NUMA node; "
                   "pinned host frames -> hipMemcpyAsync H2D -> interpreter -> D2H, a stream per stage chained by "
                   "events over rotating device buffers (H2D of chunk k+1 under the D2H of chunk k); *_rr: the "
                   "round-robin streams, each carrying a chunk's H2D, launch and D2H; zero_copy: one launch over "
                   "the pinned host frames in place, verdicts to host memory; PCIe-inclusive, not the headline value")
    return out


def cpu_baseline(budget_s, workload="xdp-counter"):
    """The oracle (restated reference CPU interpreter, -O2) over a bounded
    sample of the same workload: one pinned core and all the cores this
    process may use (bench_cpu.py, run as its own process: it never touches
    the GPU)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_cpu.py"), "--workload", workload,
                            "--seconds", str(budget_s)], capture_output=True, text=True, timeout=20 * budget_s + 120)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 -- a baseline failure must not lose the GPU line
        return {"error": "cpu baseline failed: %s" % e}


if __name__ == "__main__":
    main()
