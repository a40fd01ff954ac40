"""N>1 path on CPU: world_size-2 gloo ranks each process their contiguous
shard (the oracle stands in for the per-GPU interpreter here; the GPU side of
the same sharding is exercised by bench.py under torchrun), gather their map
shards, and the host merge reproduces the single-batch result exactly."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from bpftime_amd import gen, isa, programs, shard
    from oracle import pyoracle as po

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        po.reset()
        ctl = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2)
        bss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)
        flows = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 16, 16, 65536)
        init_bss = bss.raw()
        first, count = shard.shard_range(n_total, world, rank)
        vm = po.OracleVM()
        vm.load(programs.xdp_counter(ctl.fd, bss.fd))
        pk = gen.xdp_packets(count, 64, gen.SEED_CFG2, first)
        v = vm.run_xdp(pk, fixed_len=64)
        fvm = po.OracleVM()
        fvm.load(programs.flow_hash(flows.fd))
        slots, lens = gen.flow_packets(count, nflows=500, first=first, stride=256)
        lens = np.minimum(lens, 256).astype(np.uint32)
        fvm.run_xdp(slots, lens=lens)
        got = [None] * world
        dist.all_gather_object(got, (bss.raw().tobytes(), flows.items(), int((v == 3).sum()), init_bss.tobytes()))
        if rank == 0:
            merged = shard.merge_array_delta(np.frombuffer(got[0][3], np.uint8),
                                             [np.frombuffer(g[0], np.uint8) for g in got])
            fmerged = shard.merge_hash_additive({}, [g[1] for g in got], 65536)
            q.put((merged.tobytes(), fmerged, sum(g[2] for g in got)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_shard_merge_matches_single_batch(fresh_oracle):
    import multiprocessing as mp

    from bpftime_amd import gen, isa, programs
    po = fresh_oracle
    n_total = 3001  # ragged split
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged, fmerged, tx = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-batch reference
    ctl = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2)
    bss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)
    flows = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 16, 16, 65536)
    vm = po.OracleVM()
    vm.load(programs.xdp_counter(ctl.fd, bss.fd))
    v = vm.run_xdp(gen.xdp_packets(n_total), fixed_len=64)
    fvm = po.OracleVM()
    fvm.load(programs.flow_hash(flows.fd))
    slots, lens = gen.flow_packets(n_total, nflows=500, stride=256)
    fvm.run_xdp(slots, lens=np.minimum(lens, 256).astype(np.uint32))
    assert merged == bss.raw().tobytes()
    assert np.frombuffer(merged, np.uint64)[0] == n_total
    assert tx == int((v == 3).sum()) == n_total
    assert fmerged == flows.items()


def test_shard_range_covers_exactly():
    from bpftime_amd.shard import shard_range
    for n in (0, 1, 7, 1 << 20, 3001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == n
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1


def _bench_worker(rank, world, path, q):
    """bench.py's own N>1 control plane: gather_ranks over the file
    rendezvous (no torch: bpftime_amd/rendezvous.py), then the rank-0 merge
    (merge_counter_shards) of per-rank .bss shards."""
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    import bench
    from bpftime_amd.rendezvous import Rendezvous
    rz = Rendezvous(rank, world, path=path, timeout=120)
    init = np.zeros(4096, np.uint8)
    init.view(np.uint64)[:3] = (7, 1 << 40, 5)
    shard = init.copy()
    shard.view(np.uint64)[0] += 1000 * (rank + 1)      # this rank's packets
    shard.view(np.uint64)[1] += rank                    # a second counter
    rz.barrier()
    got = bench.gather_ranks(rz, world, (0.5 + rank, shard.tobytes(), True, None, 70200000 + rank % 1))
    if rank == 0:
        merged = bench.merge_counter_shards(init, [np.frombuffer(g[1], np.uint8) for g in got])
        q.put((merged.view(np.uint64)[:3].tolist(), [g[0] for g in got], sorted({g[4] for g in got}),
               "torch" in sys.modules))
    rz.close()


def test_bench_control_plane_two_ranks(tmp_path):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "rdzv")
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    counters, times, versions, torch_loaded = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert counters == [7 + 1000 + 2000, (1 << 40) + 1, 5]
    assert times == [0.5, 1.5]   # bench.py reports world * n * steps / max(times)
    assert versions == [70200000]
    assert not torch_loaded      # the control plane never imports torch
    assert not os.path.exists(path)  # rank 0 removed the rendezvous directory


def _rdzv_worker(rank, world, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_PORT="29533", TORCHELASTIC_RUN_ID="test-run")
    import time
    from bpftime_amd.rendezvous import Rendezvous, launch_dir
    rz = Rendezvous(rank, world, timeout=120)
    order = []
    rz.barrier()                        # (processes start with a skew of their own)
    for step in range(5):
        if rank == step % world:
            time.sleep(0.05)            # a late rank: nobody may pass the barrier before it arrives
        t = time.monotonic()
        rz.barrier()
        order.append(time.monotonic() - t)
    got = rz.all_gather({"rank": rank, "blob": bytes([rank]) * (rank + 1), "t": (rank, [1, 2])})
    q.put((rank, launch_dir(), order, got))
    rz.close()


def test_rendezvous_barrier_and_gather():
    """Four ranks started by one parent (as torchrun's agent starts a
    launch's workers) meet in the same directory; each barrier holds every
    rank until the late one arrives; the gather returns every rank's
    payload (bytes included) in rank order on every rank."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 4
    procs = [ctx.Process(target=_rdzv_worker, args=(r, world, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dirs = {r[1] for r in res}
    assert len(dirs) == 1 and f"_{os.getpid()}_" in dirs.pop()
    for rank, _, waits, got in res:
        for step, w in enumerate(waits):
            if rank != step % world:
                assert w >= 0.03, (rank, step, w)
        assert got == [{"rank": r, "blob": bytes([r]) * (r + 1), "t": [r, [1, 2]]} for r in range(world)]


def test_merge_at_counter_width():
    """u32 counters whose combined delta crosses 2^32 wrap at 32 bits and
    leave the neighbouring counter alone (a u64-word merge would carry)."""
    from bpftime_amd import shard
    init = np.array([0xFFFFFFF0, 5], np.uint32).view(np.uint8)
    s1 = np.array([0xFFFFFFF8, 5], np.uint32).view(np.uint8)   # +8
    s2 = np.array([0xFFFFFFFC, 6], np.uint32).view(np.uint8)   # +0xC, neighbour +1
    got = shard.merge_array_delta(init, [s1, s2], width=4).view(np.uint32)
    assert got.tolist() == [(0xFFFFFFF0 + 8 + 0xC) & 0xFFFFFFFF, 6]   # the total crosses 2^32
    wrong = shard.merge_array_delta(init, [s1, s2], width=8).view(np.uint32)
    assert wrong.tolist() != got.tolist()
    h = shard.merge_hash_additive({b"k": init.tobytes()}, [{b"k": s1.tobytes()}, {b"k": s2.tobytes()}], 8, width=4)
    assert np.frombuffer(h[b"k"], np.uint32).tolist() == got.tolist()
    assert shard.counter_width(12) == 4 and shard.counter_width(16) == 8
    with pytest.raises(ValueError):
        shard.counter_width(6)


def test_rendezvous_refuses_planted_or_unnamed_dirs(tmp_path, monkeypatch):
    """the directory must be this user's, mode 0700, and not a
    finished launch's; ranks outside torchrun must name their directory."""
    from bpftime_amd import rendezvous as rv
    planted = tmp_path / "planted"
    planted.mkdir(mode=0o777)
    os.chmod(planted, 0o777)
    with pytest.raises(PermissionError):
        rv.Rendezvous(0, 2, path=str(planted))
    old = tmp_path / "old"
    old.mkdir(mode=0o700)
    (old / "exit.1").write_bytes(b"")
    with pytest.raises(RuntimeError):
        rv.Rendezvous(0, 2, path=str(old))
    monkeypatch.delenv("BPFTIME_AMD_RDZV_DIR", raising=False)
    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    with pytest.raises(RuntimeError):
        rv.launch_dir()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "r/../x")
    d = rv.launch_dir()
    assert "/" not in os.path.basename(d) and f"_{os.getuid()}_" in d
