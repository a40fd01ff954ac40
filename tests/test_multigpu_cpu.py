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
