"""Secondary benchmarks (BASELINE.json configs[2] and configs[4]) at full
size, device-resident, one GPU:

  python bench.py --workload flow-hash     # 2^24 frames in 2048-B slots, HASH map
  python bench.py --workload syscall-agg   # 2^25 trace_event_raw_sys_enter records
  python bench.py --workload syscount      # 2^25 32-B exit records (SoA), sys_exit through the dispatch
  python bench.py --workload syscount-latency  # syscount -L: enter + exit, thread-ordered dispatch

The headline line (xdp-counter) stays in bench.py.  Inputs are generated on
the device by csrc/gen.hip from the same seeded streams as bpftime_amd/gen.py;
parity at full size is checked through size-independent properties the host
recomputes from those streams: per-flow / per-id totals equal to the exact
histogram of the input times the number of runs, verdict classes, and r0.
"""
import json
import os
import struct
import time

import numpy as np

HBM_PEAK_GBS = 8000.0
ROOT = os.path.dirname(os.path.abspath(__file__))


def pmc_traffic(workload, units):
    """HBM bytes per launch from the committed PMC pass of this workload
    (profiles/pmc_<workload>.json, tools/prof_workload.sh + tools/pmc_table.py:
    FETCH_SIZE x2 + WRITE_SIZE), when it was taken at this launch size."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)) as f:
            pmc = json.load(f)
        return pmc.get("hbm_bytes_per_launch") if pmc.get("units") == units else None
    except (OSError, ValueError):
        return None


def _dbg_lcache(dev):
    """BPFTIME_AMD_DBG=512: the hash lookup cache's hit / miss lanes over
    the whole run (timing-perturbing counters, never a bench number)."""
    if not int(os.environ.get("BPFTIME_AMD_DBG", "0"), 0) & 512:
        return {}
    import ctypes as C
    out = (C.c_uint64 * 4)()
    if dev.lib().bpftime_amd_dbg_counters(out, 4, 1) < 2:
        return {"dbg_lcache": None}
    return {"dbg_lcache": {"hit_lanes": out[0], "miss_lanes": out[1],
                           "hit_rate": round(out[0] / max(1, out[0] + out[1]), 4),
                           "index_empty_or_reserved_lanes": out[2], "index_too_long_lanes": out[3]}}


def _timed(dev, step, steps, warmup):
    """(wall seconds, average kernel seconds) over `steps` back-to-back
    launches bracketed by two events on the launch stream."""
    for _ in range(warmup):
        step()
    dev.lib().bpftime_amd_sync()
    ev0, ev1 = dev.Event(), dev.Event()
    t0 = time.perf_counter()
    ev0.record()
    for i in range(steps):
        step()
    ev1.record()
    dev.lib().bpftime_amd_sync()
    wall = time.perf_counter() - t0
    return wall, ev0.elapsed_ms(ev1) / steps / 1e3


def flow_hash(args, dev, gen, isa, programs):
    n = 1 << (args.log2n if args.log2n_set else 24)
    stride = 2048
    nflows = 65536
    dev.reset_runtime()
    flows = dev.Map(isa.BPF_MAP_TYPE_HASH, 16, 16, nflows, name="flows")
    code = programs.flow_hash(flows.fd)
    vm = dev.VM()
    vm.load(code)
    cdf = gen.zipf_cdf(nflows, 1.1)
    dcdf = dev.DeviceBuffer.from_array(cdf)
    pk = dev.DeviceBuffer(n * stride)
    dl = dev.DeviceBuffer(4 * n)
    if dev.lib().bpftime_amd_gen_flow(pk.ptr, dl.ptr, n, stride, gen.SEED_CFG3, 0, dcdf.ptr, nflows, None):
        raise SystemExit("flow generator failed")
    dv = dev.DeviceBuffer(4 * n)

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, stride, lens=dl, verdicts=dv, flags=0)

    # the cold launch: the first batch over the empty map inserts every flow
    # it meets (BASELINE configs[2] traffic keeps adding flows; the timed
    # steps after it are the steady state with the table full)
    dev.lib().bpftime_amd_sync()
    t0 = time.perf_counter()
    vm.exec_batch(dev.CTX_XDP, pk, n, stride, lens=dl, verdicts=dv, flags=dev.BATCH_TIMED)
    cold_s = vm.last_batch_ms() / 1e3  # its kernels (host set-up of a first launch excluded)
    cold_wall = time.perf_counter() - t0
    cold_flows = flows.count()
    cold_dbg = _dbg_lcache(dev)  # (BPFTIME_AMD_DBG 512: the cold launch's own counts)
    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    runs = args.steps + args.warmup + 1
    # ---- expected totals from the generator's streams ----
    idx = np.arange(n, dtype=np.uint64)
    r = gen.sm64(gen.SEED_CFG3 ^ 0x1111, idx)
    sel = (r % np.uint64(12)).astype(np.int64)
    lens = np.where(sel < 7, 64, np.where(sel < 11, 570, 1500)).astype(np.uint64)
    is_ip = ((r >> np.uint64(8)) % np.uint64(100)) < np.uint64(95)
    del r, sel
    flow = gen.zipf_ids(gen.SEED_CFG3, 0, n, nflows, 1.1)
    fid = np.arange(nflows, dtype=np.uint64)
    fk = gen.sm64(gen.SEED_CFG3 ^ 0x2222, fid)
    fk2 = gen.sm64(gen.SEED_CFG3 ^ 0x3333, fid)
    proto = np.where((fk2 >> np.uint64(40)) & np.uint64(1), 6, 17)
    cnt = np.bincount(flow[is_ip], minlength=nflows).astype(np.uint64)
    byt = np.bincount(flow[is_ip], weights=lens[is_ip].astype(np.float64), minlength=nflows)
    byt = np.round(byt).astype(np.uint64)
    got = flows.hash_items()
    ok_map = len(got) == int((cnt > 0).sum())
    if ok_map:
        for f in np.nonzero(cnt)[0]:
            key = struct.pack("<IIII", int(fk[f] & np.uint64(0xFFFFFFFF)), int(fk[f] >> np.uint64(32)),
                              int(fk2[f] & np.uint64(0xFFFFFFFF)), int(proto[f]))
            v = got.get(key)
            if v is None or struct.unpack("<QQ", v) != (int(cnt[f]) * runs, int(byt[f]) * runs):
                ok_map = False
                break
    verd = dv.download(np.uint32)
    tcp = is_ip & (proto[flow] == 6)
    ok_verd = bool(((verd == isa.XDP_TX) == tcp).all() and ((verd == isa.XDP_PASS) == ~tcp).all())
    ip_frac = float(is_ip.mean())
    algo = 24.0 * ip_frac + 10.0 * (1 - ip_frac)
    cpu = None
    if not args.no_cpu_baseline:
        from bench import cpu_baseline
        cpu = cpu_baseline(args.cpu_seconds, "flow-hash")
    value = n * args.steps / wall / 1e6
    achieved = algo * n / kern_s / 1e9
    return {
        "metric": "device-resident Mpps, 5-tuple flow-hash XDP prog, mixed 64-1500B pkts",
        "value": round(value, 3), "unit": "Mpps", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 frames: 64/570/1500 B 7:4:1, 95% IPv4 TCP:UDP 1:1, "
                "65536 Zipf(1.1) flows, seed 0x5EED0003)",
        "config": {"workload": "flow-hash (BASELINE configs[2]) over 2^%d device-resident frames in "
                               "2048-B slots, HASH map max 65536" % int(np.log2(n)),
                   "packets": n, "interp": {"fast_specialized": vm.fast_specialized(dev.CTX_XDP)}},
        "parity": {"per_flow_totals_exact": ok_map, "verdict_classes": ok_verd, "flows": len(got),
                   "ok": ok_map and ok_verd},
        "cold": {"note": "the first launch, over the empty map: every flow it meets is inserted; ms = its "
                         "kernels (events around them), wall_ms = with the first launch's host set-up",
                 "ms": round(cold_s * 1e3, 4), "Mpps": round(n / cold_s / 1e6, 3), "flows_inserted": cold_flows,
                 "wall_ms": round(cold_wall * 1e3, 3), **cold_dbg},
        **_dbg_lcache(dev),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic("flow-hash", n),
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_pkt": round(algo, 2)},
        "cpu_baseline": cpu,
    }


def syscall_agg(args, dev, gen, isa, programs):
    n = 1 << (args.log2n if args.log2n_set else 25)
    dev.reset_runtime()
    counts = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, name="counts")
    code = programs.syscall_agg(counts.fd)
    vm = dev.VM()
    vm.load(code)
    cdf = gen.zipf_cdf(335, 1.2)
    dcdf = dev.DeviceBuffer.from_array(cdf)
    recs = dev.DeviceBuffer(n * 64)
    if dev.lib().bpftime_amd_gen_syscall(recs.ptr, n, gen.SEED_CFG5, 0, dcdf.ptr, 335, None):
        raise SystemExit("syscall generator failed")
    dr = dev.DeviceBuffer(8 * n)

    def step():
        vm.exec_batch(dev.CTX_SYSCALL, recs, n, 64, rets=dr, flags=0)

    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    runs = args.steps + args.warmup
    idx = np.arange(n, dtype=np.uint64)
    ids = gen.zipf_ids(gen.SEED_CFG5, 0, n, 335, 1.2)
    r = gen.sm64(gen.SEED_CFG5 ^ 0x5555, idx)
    special = (r % np.uint64(100)) == np.uint64(0)
    ids = np.where(special, np.where((r >> np.uint64(9)) & np.uint64(1), 60, 231), ids)
    del r, special
    live = (ids != 60) & (ids != 231)
    hist = np.bincount(ids[live], minlength=335).astype(np.uint64)
    a2 = gen.sm64(gen.SEED_CFG5 ^ 0x6002, idx) & np.uint64(0xFFFFFFFFFF)
    ns = {k: int(a2[ids == k].sum(dtype=np.uint64)) for k in (0, 1)}
    got = counts.hash_items()
    ok_map = len(got) == int((hist > 0).sum())
    for k in np.nonzero(hist)[0]:
        v = got.get(struct.pack("<I", int(k)))
        if v is None:
            ok_map = False
            break
        c, t = struct.unpack("<QQ", v[:16])
        exp_t = (ns.get(int(k), 0) * runs) & 0xFFFFFFFFFFFFFFFF
        if c != int(hist[k]) * runs or t != exp_t:
            ok_map = False
            break
    ok_ret = bool((dr.download(np.uint64) == 0).all())
    p = float(((ids == 0) | (ids == 1)).mean())
    algo = 12.0 + 8.0 * p
    cpu = None
    if not args.no_cpu_baseline:
        from bench import cpu_baseline
        cpu = cpu_baseline(args.cpu_seconds, "syscall-agg")
    value = n * args.steps / wall / 1e6
    achieved = algo * n / kern_s / 1e9
    return {
        "metric": "device-resident Mrec/s, syscall-agg prog over trace_event_raw_sys_enter records",
        "value": round(value, 3), "unit": "Mrec/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 records: id Zipf(1.2) over 0..334 + 1% exit/exit_group, "
                "seed 0x5EED0005)",
        "config": {"workload": "syscall-agg (BASELINE configs[4]) over 2^%d device-resident 64-B records, "
                               "HASH map max 8192" % int(np.log2(n)),
                   "records": n, "interp": {"fused_rmw": vm.info()["fused_rmw"],
                                            "fast_specialized": vm.fast_specialized(dev.CTX_SYSCALL)}},
        "parity": {"per_id_totals_exact": ok_map, "r0_all_zero": ok_ret, "keys": len(got),
                   "ok": ok_map and ok_ret},
        **_dbg_lcache(dev),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic("syscall-agg", n),
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_rec": round(algo, 2)},
        "cpu_baseline": cpu,
    }


def syscount(args, dev, gen, isa, programs):
    """syscount's sys_exit program (example/tracing/syscount/syscount.bpf.c:
    49-87) attached to raw_syscalls:sys_exit, replayed through the dispatch
    over 2^25 device-resident calls in struct-of-arrays form
    (bpftime_amd_syscall_dispatch_soa): the exit array only, 32 B per call
    {trace_event_raw_sys_exit, caller pid_tgid} -- an exit-only dispatch
    streams what its program reads (BPFTIME_AMD_SYSCOUNT_AOS=1: the 96-B
    records through bpftime_amd_syscall_dispatch_records instead, same
    calls)."""
    n = 1 << (args.log2n if args.log2n_set else 25)
    dev.reset_runtime()
    data = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, name="data")
    ro = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1, name="syscount.rodata")
    ro.update(b"\0" * 4, programs.syscount_rodata())
    code = programs.syscount_exit(data.fd, ro.fd)
    pfd = dev.prog_create(code, "sys_exit", 5)
    dev.syscall_attach(pfd, -1, enter=False)
    cdf = gen.zipf_cdf(335, 1.2)
    dcdf = dev.DeviceBuffer.from_array(cdf)
    aos = os.environ.get("BPFTIME_AMD_SYSCOUNT_AOS") == "1"
    recs = dev.DeviceBuffer(n * (96 if aos else 32))
    rc = (dev.lib().bpftime_amd_gen_syscall_full(recs.ptr, n, gen.SEED_CFG5, 0, dcdf.ptr, 335, None) if aos else
          dev.lib().bpftime_amd_gen_syscall_soa(None, recs.ptr, n, gen.SEED_CFG5, 0, dcdf.ptr, 335, None))
    if rc:
        raise SystemExit("syscall generator failed")

    def step():
        if aos:
            dev.syscall_dispatch(recs, n, flags=0)
        else:
            dev.syscall_dispatch_soa(recs, n, flags=0)

    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    runs = args.steps + args.warmup
    # host recomputation of the histogram from the same seeded stream
    idx = np.arange(n, dtype=np.uint64)
    ids = gen.zipf_ids(gen.SEED_CFG5, 0, n, 335, 1.2).astype(np.int64)
    r = gen.sm64(gen.SEED_CFG5 ^ 0x5555, idx)
    ids = np.where((r % np.uint64(100)) == np.uint64(0), np.where((r >> np.uint64(9)) & np.uint64(1), 60, 231), ids)
    ids = np.where((r % np.uint64(200)) == np.uint64(1), -1, ids)
    del r
    live = ~np.isin(ids, [60, 231, -1])
    hist = np.bincount(ids[live], minlength=335).astype(np.uint64)
    got = data.hash_items()
    ok_map = len(got) == int((hist > 0).sum()) and all(
        struct.unpack("<Q", got.get(struct.pack("<I", int(k)), b"\0" * 32)[:8])[0] == int(hist[k]) * runs
        for k in np.nonzero(hist)[0])
    algo = 24.0  # SURVEY.md §8d per record: id + ret of the exit ctx, the caller's pid_tgid
    cpu = None
    if not args.no_cpu_baseline:
        from bench import cpu_baseline
        cpu = cpu_baseline(args.cpu_seconds, "syscount")
    value = n * args.steps / wall / 1e6
    achieved = algo * n / kern_s / 1e9
    return {
        "metric": "device-resident Mrec/s, syscount sys_exit prog through the syscall dispatch",
        "value": round(value, 3), "unit": "Mrec/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 replay records: id Zipf(1.2) over 0..334 + 1% exit/exit_group + "
                "0.5% id -1, 20% negative rets, 64 callers; seed 0x5EED0005)",
        "config": {"workload": "syscount sys_exit (BASELINE configs[4]'s attach point) over 2^%d device-resident "
                               "calls, %s, HASH map max 8192"
                               % (int(np.log2(n)), "96-B records" if aos else
                                  "struct-of-arrays exit records (32 B: trace_event_raw_sys_exit + caller)"),
                   "records": n, "layout": "aos96" if aos else "soa"},
        "parity": {"per_id_totals_exact": ok_map, "keys": len(got), "ok": ok_map},
        **_dbg_lcache(dev),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic("syscount", n),
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_rec": algo},
        "cpu_baseline": cpu,
    }


def _lpm_routes(rng, nroutes):
    """Every /8 (so each address has a route) plus random /12../28 prefixes;
    values 1..3 = DROP / PASS / TX."""
    routes = [(8, i << 24, 1 + (i % 3)) for i in range(256)]
    while len(routes) < nroutes:
        plen = int(rng.integers(12, 29))
        net = int(rng.integers(0, 1 << 32)) & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF)
        routes.append((plen, net, int(rng.integers(1, 4))))
    return routes


def lpm_route(args, dev, gen, isa, programs):
    """LPM_TRIE routing: 2^24 random 64-B IPv4 frames,
    16384 routes, one lookup per frame on the device replica."""
    n = 1 << (args.log2n if args.log2n_set else 24)
    rng = np.random.default_rng(0x5EED0006)
    routes = _lpm_routes(rng, 16384)
    dev.reset_runtime()
    rt = dev.Map(isa.BPF_MAP_TYPE_LPM_TRIE, 8, 4, len(routes), name="routes")
    for plen, net, v in routes:
        rt.update(struct.pack("<I", plen) + struct.pack(">I", net), struct.pack("<I", v))
    code = programs.lpm_route(rt.fd)
    vm = dev.VM()
    vm.load(code)
    pk = dev.DeviceBuffer(n * 64)
    if dev.lib().bpftime_amd_gen_xdp(pk.ptr, n, 64, 64, gen.SEED_CFG2 ^ 0x6, 0, None):
        raise SystemExit("generator failed")
    dv = dev.DeviceBuffer(4 * n)

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0)

    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    from oracle import pyoracle as po   # checker: the oracle over a sample of the same frames
    sn = min(n, 1 << 18)
    sample = pk.download(count=sn * 64).reshape(sn, 64)
    po.reset()
    om = po.OracleMap(isa.BPF_MAP_TYPE_LPM_TRIE, 8, 4, len(routes), fd=rt.fd)
    for plen, net, v in routes:
        om.update(struct.pack("<I", plen) + struct.pack(">I", net), struct.pack("<I", v))
    ovm = po.OracleVM()
    ovm.load(code)
    want = ovm.run_xdp(sample.copy(), fixed_len=64)
    verd = dv.download(np.uint32)
    ok = bool((verd[:sn] == want).all()) and bool(np.isin(verd, [1, 2, 3]).all())
    cpu = None
    if not args.no_cpu_baseline:   # one pinned core and 16 (bench_cpu.py), over shards of the same frames
        from bench import cpu_baseline
        cpu = cpu_baseline(args.cpu_seconds, "lpm-route")
    algo = 2 + 4 + 4 + 4.0   # ethertype + daddr + verdict + the route entry the lookup reads
    achieved = algo * n / kern_s / 1e9
    return {
        "metric": "device-resident Mpps, LPM-trie routing XDP prog (16384 IPv4 routes), 64B pkts",
        "value": round(n * args.steps / wall / 1e6, 3), "unit": "Mpps", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 64-B IPv4 frames; routes: every /8 + random /12../28)",
        "config": {"workload": "lpm-route over 2^%d device-resident 64-B frames" % int(np.log2(n)),
                   "packets": n, "routes": len(routes)},
        "parity": {"sample_verdicts_exact": ok, "sample": sn, "ok": ok,
                   "verdicts": {str(k): int((verd == k).sum()) for k in (1, 2, 3)}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic("lpm-route", n),
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_pkt": algo},
        "cpu_baseline": cpu,
    }


def ringbuf_sample(args, dev, gen, isa, programs):
    """RINGBUF sampling: 2^24 64-B frames, every 64th
    (by its first byte) sends its 12 MAC bytes through bpf_ringbuf_output;
    the 256-MiB ring holds every run's records (the consumer drains it once,
    after the timed runs)."""
    n = 1 << (args.log2n if args.log2n_set else 24)
    os.environ.setdefault("BPFTIME_AMD_ARENA_MB", "1024")   # the ring's 2 x 256 MiB of records
    dev.reset_runtime()
    runs = args.steps + args.warmup
    size = 1 << 28
    rb = dev.Map(isa.BPF_MAP_TYPE_RINGBUF, 0, 0, size, name="samples")
    code = programs.ringbuf_sampler(rb.fd, every_log2=6)
    vm = dev.VM()
    vm.load(code)
    pk = dev.DeviceBuffer(n * 64)
    if dev.lib().bpftime_amd_gen_xdp(pk.ptr, n, 64, 64, gen.SEED_CFG2, 0, None):
        raise SystemExit("generator failed")
    dv = dev.DeviceBuffer(4 * n)

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0)

    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    first = pk.download(count=n * 64).reshape(n, 64)[:, 0]
    picked = int((first % 64 == 0).sum())
    recs = rb.ringbuf_fetch(cap=size * 2)
    fits = min(runs * picked, size // 24)
    verd = dv.download(np.uint32)
    ok = len(recs) == fits and all(r[0] % 64 == 0 for r in recs[:4096]) and \
        (runs * picked > fits or bool((verd == isa.XDP_PASS).all()))
    algo = 1 + 4 + 24 / 64   # first byte + verdict + a 24-B record for one frame in 64
    achieved = algo * n / kern_s / 1e9
    cpu = None
    if not args.no_cpu_baseline:   # the oracle over a sample of the same frames
        from oracle import pyoracle as po
        sn = min(n, 1 << 18)
        sample = pk.download(count=sn * 64).reshape(sn, 64)
        po.reset()
        om = po.OracleMap(isa.BPF_MAP_TYPE_RINGBUF, 0, 0, 1 << 24, fd=rb.fd)
        ovm = po.OracleVM()
        ovm.load(code)
        ovm.run_xdp(sample.copy(), fixed_len=64)
        ok = ok and len(om.ringbuf_fetch()) == int((sample[:, 0] % 64 == 0).sum())
        from bench import cpu_baseline   # one pinned core and 16 (bench_cpu.py)
        cpu = cpu_baseline(args.cpu_seconds, "ringbuf-sample")
    return {
        "metric": "device-resident Mpps, ring-buffer sampling XDP prog (1/64 frames), 64B pkts",
        "value": round(n * args.steps / wall / 1e6, 3), "unit": "Mpps", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 64-B frames, seed 0x5EED0002)",
        "config": {"workload": "ringbuf-sample over 2^%d device-resident 64-B frames, 256-MiB ring"
                               % int(np.log2(n)), "packets": n, "records_per_run": picked},
        "parity": {"records": len(recs), "expected_records": fits, "ok": ok},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic("ringbuf-sample", n),
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_pkt": algo},
        "cpu_baseline": cpu,
    }


def tail_call(args, dev, gen, isa, programs):
    """bpf_tail_call jump table: 2^24 64-B frames; the
    caller tail-calls slot data[0] & 3 of a PROG_ARRAY {0: a packet writer,
    1: a map counter, 2: empty (-1), 3: a counter that tail-calls slot 0}
    with per-CPU counters,
    so lanes of one wave take different targets and chains of two."""
    n = 1 << (args.log2n if args.log2n_set else 24)
    dev.reset_runtime()
    pa = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, name="jmp_table")
    # per-CPU counters, the XDP idiom for hot counters (virtual CPU = unit / 64)
    cnt = dev.Map(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 4, name="counts")
    targets = {0: programs.tail_target_write(0xA1), 1: programs.tail_target_count(cnt.fd),
               3: programs.tail_target_recurse(pa.fd, cnt.fd, 0)}
    pfd = {}
    for k, code in targets.items():
        pfd[k] = dev.prog_create(code, "t%d" % k, 6)
        pa.update(struct.pack("<i", k), struct.pack("<i", pfd[k]))
    code = programs.tail_xdp_caller(pa.fd, cnt.fd)
    vm = dev.VM()
    vm.load(code)
    pk = dev.DeviceBuffer(n * 64)
    if dev.lib().bpftime_amd_gen_xdp(pk.ptr, n, 64, 64, gen.SEED_CFG2 ^ 0x7, 0, None):
        raise SystemExit("generator failed")
    dv = dev.DeviceBuffer(4 * n)

    def step():
        vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0, ifindex=5)

    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    runs = args.steps + args.warmup
    frames = pk.download().reshape(n, 64)
    idx = frames[:, 0] & 3
    hist = np.bincount(idx, minlength=4).astype(np.uint64)
    want_v = np.array([64 + 0xA1, 2, 0xFFFFFFFF, 64 + 0xA1 + 1], dtype=np.uint64)[idx] + 1005
    verd = dv.download(np.uint32)
    got = [int(np.frombuffer(cnt.lookup(struct.pack("<i", i)), dtype=np.uint64).sum()) for i in range(4)]
    want_c = [runs * int(hist[0]), runs * 2 * int(hist[1]), runs * int(hist[2] + hist[3]), runs * int(hist[3])]
    ok = bool((verd == (want_v & 0xFFFFFFFF).astype(np.uint32)).all()) and got == want_c and \
        bool((frames[(idx == 0) | (idx == 3), 1] == 0xA1).all())
    cpu = None
    if not args.no_cpu_baseline:   # the oracle over a sample of the same frames
        from oracle import pyoracle as po
        sn = min(n, 1 << 18)
        po.reset()
        opa = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=pa.fd)
        po.OracleMap(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 4, fd=cnt.fd)
        for k, c in targets.items():
            po.prog_create(pfd[k], c)
            opa.update(struct.pack("<i", k), struct.pack("<i", pfd[k]))
        ovm = po.OracleVM()
        ovm.load(code)
        ov = ovm.run_xdp(frames[:sn].copy(), fixed_len=64, ifindex=5)
        ok = ok and bool((ov == verd[:sn]).all())
        from bench import cpu_baseline   # one pinned core and 16 (bench_cpu.py)
        cpu = cpu_baseline(args.cpu_seconds, "tail-call")
    algo = 1 + 4 + 0.5   # first byte + verdict + the writer's byte for half the frames (counters on-chip)
    achieved = algo * n / kern_s / 1e9
    return {
        "metric": "device-resident Mpps, bpf_tail_call jump-table XDP prog (4 slots), 64B pkts",
        "value": round(n * args.steps / wall / 1e6, 3), "unit": "Mpps", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 64-B frames)",
        "config": {"workload": "tail-call over 2^%d device-resident 64-B frames" % int(np.log2(n)),
                   "packets": n, "slots": 4},
        "parity": {"verdicts_exact": ok, "counters": got, "ok": ok},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc_traffic("tail-call", n),
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_pkt": algo},
        "cpu_baseline": cpu,
    }


def syscount_latency(args, dev, gen, isa, programs):
    """syscount -L: its sys_enter program (start[tid] = bpf_ktime_get_ns())
    and its sys_exit program with measure_latency (lat = now - start[tid])
    attached together (example/tracing/syscount/syscount.bpf.c:33-87).  The
    exit program reads what the same call's enter program wrote, so the
    dispatch runs thread-ordered (include/bpftime_amd.h "Order"): the records
    grouped by their recorded caller, one lane per thread, each call's enter
    and exit programs back to back; the clock is the recorded one.  Records:
    2^22 struct-of-arrays calls (64-B enter, 32-B exit + caller, 16-B clocks)
    from 4096 threads (BPFTIME_AMD_THREADS); the step is the whole dispatch
    (grouping sort included).  Parity at full size: per-id count and
    total_ns against the host recomputation (each call's exit - enter clock),
    and every thread's start entry."""
    n = 1 << (args.log2n if args.log2n_set else 22)
    threads = int(os.environ.get("BPFTIME_AMD_THREADS", "4096"))
    dev.reset_runtime()
    start = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 8, max(10240, 2 * threads), name="start")
    data = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 10240, name="data")
    ro = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, programs.SYSCOUNT_RODATA, 1, name="syscount.rodata")
    ro.update(b"\0" * 4, programs.syscount_rodata(measure_latency=True))
    dev.syscall_attach(dev.prog_create(programs.syscount_enter(start.fd, ro.fd), "sys_enter", 5), -1, True)
    dev.syscall_attach(dev.prog_create(programs.syscount_exit(data.fd, ro.fd, start.fd), "sys_exit", 5), -1, False)
    plan = dev.syscall_dispatch_plan()
    recs = gen.syscall_records_timed(n, threads=threads)
    enter, exit_, clock = gen.syscall_records_soa(recs)
    de, dx, dc = (dev.DeviceBuffer.from_array(a) for a in (enter, exit_, clock))

    def step():
        dev.syscall_dispatch_soa(dx, n, enter=de, clock=dc, flags=0)

    wall, kern_s = _timed(dev, step, args.steps, args.warmup)
    runs = args.steps + args.warmup
    w = recs.view(np.int64).reshape(n, 16)
    ids, rets = w[:, 1], w[:, 10]
    live = ~np.isin(ids, [60, 231, -1])
    lat = (w[:, 13] - w[:, 12]).astype(np.uint64)
    cnt = np.bincount(ids[live], minlength=335).astype(np.uint64)
    tot = np.zeros(335, dtype=np.uint64)
    np.add.at(tot, ids[live], lat[live])
    got = data.hash_items()
    ok_map = len(got) == int((cnt > 0).sum()) and all(
        struct.unpack("<QQ", got.get(struct.pack("<I", int(k)), b"\0" * 32)[:16]) ==
        (int(cnt[k]) * runs, int(tot[k]) * runs % (1 << 64)) for k in np.nonzero(cnt)[0])
    # start[tid] = the enter clock of each thread's last call (exit / exit_group run nothing)
    ent = ~np.isin(ids, [60, 231])
    tid = (w[:, 11] & 0xFFFFFFFF).astype(np.uint64)
    last = {}
    for t, c in zip(tid[ent].tolist(), w[ent, 12].tolist()):
        last[t] = c
    st = start.hash_items()
    ok_start = len(st) == len(last) and all(struct.unpack("<Q", st[struct.pack("<I", t)])[0] == c
                                            for t, c in last.items())
    del rets
    cpu = None
    if not args.no_cpu_baseline:
        from bench import cpu_baseline
        cpu = cpu_baseline(args.cpu_seconds, "syscount-latency")
    algo = 64.0 + 32.0 + 16.0  # per call: the enter ctx, the exit ctx + caller, the clocks
    achieved = algo * n / kern_s / 1e9
    return {
        "metric": "device-resident Mrec/s, syscount -L (sys_enter + sys_exit, measure_latency) through the "
                  "thread-ordered syscall dispatch",
        "value": round(n * args.steps / wall / 1e6, 3), "unit": "Mrec/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded splitmix64 replay calls from %d threads, recorded clocks; seed 0x5EED0005)"
                % threads,
        "config": {"workload": "syscount -L over 2^%d device-resident calls (struct-of-arrays, 112 B per call), "
                               "%d threads, thread-ordered dispatch" % (int(np.log2(n)), threads),
                   "records": n, "threads": threads, "plan": "threads" if plan == 1 else "programs"},
        "parity": {"per_id_count_and_latency_exact": ok_map, "start_per_thread_exact": ok_start,
                   "ok": bool(ok_map and ok_start and plan == 1)},
        "roofline": {"bound": "latency (one lane per thread: a thread's calls run in order)",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel_avg_ms": round(kern_s * 1e3, 4), "algo_bytes_per_rec": algo},
        "cpu_baseline": cpu,
    }


def run(args):
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--workload %s runs on one GPU (BASELINE configs[2]/[4])" % args.workload)
    from bpftime_amd import gen, isa, programs
    from bpftime_amd import vm as dev
    fn = {"flow-hash": flow_hash, "syscall-agg": syscall_agg, "lpm-route": lpm_route,
          "ringbuf-sample": ringbuf_sample, "tail-call": tail_call, "syscount": syscount,
          "syscount-latency": syscount_latency}[args.workload]
    print(json.dumps(fn(args, dev, gen, isa, programs)))
