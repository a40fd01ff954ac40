"""BASELINE configs[3] on the device: one stream split into 8 contiguous
shards, each run as a GPU of an 8-GPU node runs it (a fresh runtime with
private map copies at the same fds, `first_unit` = the shard's offset in the
global stream), the map shards merged on the host (bpftime_amd/shard.py, the
rule bench.py applies at N>1), and the result compared bit-exactly with one
unsharded device batch over the whole stream and with the oracle.

This is the sharded path of SURVEY.md §8e with the 8 GPUs replaced by 8
successive runtimes on one GPU: what differs on a real node is only which
card each shard runs on.  Per-CPU slots are global across shards (virtual
CPU of unit u = ((first_unit + u) / 64) % ncpu), so per-CPU values merge
by addition too."""
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs, shard

pytestmark = pytest.mark.gpu

G = 8   # GPUs of the node (configs[3])


def _shards(n):
    return [shard.shard_range(n, G, g) for g in range(G)]


_FLOWS = {}


def _flow_stream(n):
    """config 3's frames at n (4 GiB of slots at 2^21: made once per module)"""
    if n not in _FLOWS:
        _FLOWS.clear()
        _FLOWS[n] = gen.flow_packets(n, nflows=65536, stride=2048)
    return _FLOWS[n]


# ---------------------------------------------------------------------------
# xdp-counter, 2^24 frames (configs[3]'s program and frame shape)
# ---------------------------------------------------------------------------
def test_xdp_counter_sharded_2p24(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    n = 1 << 24
    L = dev.lib()

    def maps():
        ctl = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, fd=3)
        bss = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, fd=4)
        return ctl, bss

    # 8 shards, each a fresh runtime (a GPU of its own)
    shard_bss, shard_verd, shard_pk = [], [], []
    init = None
    for first, cnt in _shards(n):
        dev.reset_runtime()
        dev.set_ncpu(64)
        ctl, bss = maps()
        if init is None:
            init = bss.snapshot()
        vm = dev.VM()
        vm.load(programs.xdp_counter(ctl.fd, bss.fd))
        pk = dev.DeviceBuffer(cnt * 64)
        assert L.bpftime_amd_gen_xdp(pk.ptr, cnt, 64, 64, gen.SEED_CFG2, first, None) == 0
        dv = dev.DeviceBuffer(4 * cnt)
        assert vm.exec_batch(dev.CTX_XDP, pk, cnt, 64, fixed_len=64, verdicts=dv, first_unit=first) == 0
        shard_bss.append(bss.snapshot())
        shard_verd.append(dv.download(np.uint32))
        shard_pk.append(pk.download().reshape(cnt, 64))
        del pk, dv, vm
    merged = shard.merge_array_delta(init, shard_bss, width=8)

    # one unsharded batch over the whole stream
    dev.reset_runtime()
    dev.set_ncpu(64)
    ctl, bss = maps()
    vm = dev.VM()
    vm.load(programs.xdp_counter(ctl.fd, bss.fd))
    pk = dev.DeviceBuffer(n * 64)
    assert L.bpftime_amd_gen_xdp(pk.ptr, n, 64, 64, gen.SEED_CFG2, 0, None) == 0
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv) == 0
    full_bss = bss.snapshot()
    full_verd = dv.download(np.uint32)
    assert merged.tobytes() == full_bss.tobytes()
    np.testing.assert_array_equal(np.concatenate(shard_verd), full_verd)

    # the oracle over the same stream (one map state across all of it)
    octl = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, fd=3)
    obss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, fd=4)
    ovm = po.OracleVM()
    ovm.load(programs.xdp_counter(octl.fd, obss.fd))
    for (first, cnt), sv, sp in zip(_shards(n), shard_verd, shard_pk):
        opk = gen.xdp_packets(cnt, 64, gen.SEED_CFG2, first)
        ov = ovm.run_xdp(opk, fixed_len=64)
        np.testing.assert_array_equal(sv, ov)
        assert (sp == opk).all()
        full_slice = pk.download(count=cnt * 64, offset=first * 64).reshape(cnt, 64)
        assert (full_slice == opk).all()
        del opk
    assert merged.tobytes() == obss.raw().tobytes()
    assert int(merged.view(np.uint64)[0]) == n


# ---------------------------------------------------------------------------
# flow-hash (configs[2]'s program) at 2^21 frames in 2048-B slots: a HASH map
# and a PERCPU_HASH map (per-CPU slots of the global virtual CPUs)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mtype", [isa.BPF_MAP_TYPE_HASH, isa.BPF_MAP_TYPE_PERCPU_HASH])
def test_flow_hash_sharded_2p21(fresh_oracle, fresh_runtime, mtype):
    po, dev = fresh_oracle, fresh_runtime
    n = 1 << 21
    ncpu = 64
    slots, lens = _flow_stream(n)

    def run(first, cnt):
        dev.reset_runtime()
        dev.set_ncpu(ncpu)
        flows = dev.Map(mtype, 16, 16, 65536, fd=5)
        vm = dev.VM()
        vm.load(programs.flow_hash(flows.fd))
        d = dev.DeviceBuffer.from_array(slots[first:first + cnt])
        dl = dev.DeviceBuffer.from_array(lens[first:first + cnt])
        dv = dev.DeviceBuffer(4 * cnt)
        assert vm.exec_batch(dev.CTX_XDP, d, cnt, 2048, lens=dl, verdicts=dv, first_unit=first) == 0
        return dv.download(np.uint32), flows.hash_items()

    shard_verd, shard_items = [], []
    for first, cnt in _shards(n):
        v, items = run(first, cnt)
        shard_verd.append(v)
        shard_items.append(items)
    merged = shard.merge_hash_additive({}, shard_items, 65536, width=8)
    full_verd, full_items = run(0, n)
    np.testing.assert_array_equal(np.concatenate(shard_verd), full_verd)
    assert merged == full_items

    po.set_ncpu(ncpu)
    om = po.OracleMap(mtype, 16, 16, 65536, fd=5)
    ovm = po.OracleVM()
    ovm.load(programs.flow_hash(om.fd))
    ov = ovm.run_xdp(slots.copy(), lens=lens, ncpu=ncpu)
    np.testing.assert_array_equal(full_verd, ov)
    assert merged == om.items()
    # size-independent: packet totals = the IPv4 frames of the stream
    vs = 16 * (ncpu if mtype == isa.BPF_MAP_TYPE_PERCPU_HASH else 1)
    tot = sum(sum(struct.unpack("<%dQ" % (vs // 8), v)[0::2]) for v in merged.values())
    assert tot == int(((slots[:, 12] == 0x08) & (slots[:, 13] == 0)).sum())
    assert len(merged) > 50000


# ---------------------------------------------------------------------------
# syscall-agg (configs[4]'s program) at 2^22 records
# ---------------------------------------------------------------------------
def test_syscall_agg_sharded_2p22(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    n = 1 << 22
    recs = gen.syscall_records(n)

    def run(first, cnt):
        dev.reset_runtime()
        dev.set_ncpu(64)
        counts = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, fd=6)
        vm = dev.VM()
        vm.load(programs.syscall_agg(counts.fd))
        d = dev.DeviceBuffer.from_array(recs[first:first + cnt])
        dr = dev.DeviceBuffer(8 * cnt)
        assert vm.exec_batch(dev.CTX_SYSCALL, d, cnt, 64, rets=dr, first_unit=first) == 0
        return dr.download(np.uint64), counts.hash_items()

    shard_ret, shard_items = [], []
    for first, cnt in _shards(n):
        r, items = run(first, cnt)
        shard_ret.append(r)
        shard_items.append(items)
    merged = shard.merge_hash_additive({}, shard_items, 8192, width=8)
    full_ret, full_items = run(0, n)
    np.testing.assert_array_equal(np.concatenate(shard_ret), full_ret)
    assert merged == full_items

    om = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, fd=6)
    ovm = po.OracleVM()
    ovm.load(programs.syscall_agg(om.fd))
    orets, _ = ovm.run_syscall(recs)
    np.testing.assert_array_equal(full_ret, orets)
    assert merged == om.items()
    ids = recs.view(np.uint64).reshape(n, 8)[:, 1]
    live = int(((ids != 60) & (ids != 231)).sum())
    assert sum(struct.unpack("<Q", v[:8])[0] for v in merged.values()) == live
