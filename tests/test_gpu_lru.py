"""BPF_MAP_TYPE_LRU_HASH on the device (common.hpp LRU_HASH, dev_helpers.hpp
lru_*, maps.cpp lru_host_*) against the oracle's restatement of
lru_var_hash_map.cpp:
  * the reference's own LRU unit tests over the host-side (syscall) ops;
  * a random op script: identical results / errno / values on both;
  * a program's lookups, inserts, deletes and evictions in an ORDERED batch:
    identical per-unit returns and final contents;
  * a parallel batch that does not fill the map: identical contents, and an
    identical recency order afterwards (host inserts then evict the same keys);
  * a parallel batch that overflows the map: count == max_entries, no key twice,
    every element's tag one its key was given."""
import ctypes as C
import struct

import numpy as np
import pytest

import _lru_cases as L
from bpftime_amd import isa, programs

pytestmark = pytest.mark.gpu
LRU = isa.BPF_MAP_TYPE_LRU_HASH


def _dev_errno():
    return C.get_errno()


@pytest.mark.parametrize("case", L.ALL, ids=lambda f: f.__name__)
def test_reference_lru_unit_tests_on_device(case, fresh_runtime):
    dev = fresh_runtime
    made = []

    def mk(cap, ks, vs):
        m = dev.Map(LRU, ks, vs, cap)
        made.append(m)
        return m
    case(mk, _dev_errno)


def test_random_script_matches_oracle(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    script = L.lru_script(seed=5, n_ops=1500, n_keys=40, cap=16)
    om = po.OracleMap(LRU, 4, 8, 16)
    dm = dev.Map(LRU, 4, 8, 16)
    assert L.replay(dm, script, _dev_errno) == L.replay(om, script, po.OracleMap.errno)
    assert dm.count() == om.count()
    assert dm.hash_items() == om.items()


def _units(recs):
    u = np.zeros((len(recs), 16), np.uint8)
    for i, (k, op, t) in enumerate(recs):
        u[i] = np.frombuffer(struct.pack("<IIQ", k, op, t), np.uint8)
    return u


def _run_both(po, dev, recs, cap, flags, n_keys=None):
    om = po.OracleMap(LRU, 4, 16, cap)
    dm = dev.Map(LRU, 4, 16, cap)
    ovm = po.OracleVM()
    ovm.load(programs.lru_track(om.fd))
    dvm = dev.VM()
    dvm.load(programs.lru_track(dm.fd))
    u = _units(recs)
    oret = ovm.run_raw(u.copy(), 16)
    d = dev.DeviceBuffer.from_array(u)
    r = dev.DeviceBuffer(8 * len(recs))
    dvm.exec_batch(dev.CTX_RAW, d, len(recs), 16, fixed_len=16, rets=r, flags=flags)
    return om, dm, oret, r.download(np.uint64)


def _script(seed, n, n_keys, ops=(0, 0, 0, 0, 1, 2, 3)):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, n_keys, n)
    op = rng.choice(ops, n)
    return [(int(k), int(o), i + 1) for i, (k, o) in enumerate(zip(keys, op))]


@pytest.mark.parametrize("cap,n_keys", [(8, 30), (64, 200), (1, 5)])
def test_ordered_batch_evictions_match_oracle(fresh_oracle, fresh_runtime, cap, n_keys):
    po, dev = fresh_oracle, fresh_runtime
    recs = _script(11 + cap, 3000, n_keys)
    om, dm, oret, dret = _run_both(po, dev, recs, cap, dev.BATCH_SYNC | dev.BATCH_ORDERED)
    np.testing.assert_array_equal(dret.astype(np.int64), oret.astype(np.int64))
    assert dm.count() == om.count()
    assert dm.hash_items() == om.items()


def test_parallel_batch_without_overflow_is_exact(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    # lookups / inserts only (no deletes, no flags that race): 300 keys in a
    # 512-entry map over 2^16 units: contents are order-independent
    n, n_keys, cap = 1 << 16, 300, 512
    rng = np.random.default_rng(3)
    keys = rng.integers(0, n_keys, n)
    recs = [(int(k), 0, 7) for k in keys]
    om, dm, oret, dret = _run_both(po, dev, recs, cap, dev.BATCH_SYNC)
    o = {k: v for k, v in om.items().items()}
    dv = dm.hash_items()
    assert set(dv) == set(o)
    for k in o:
        assert dv[k] == o[k], k                     # hits counted exactly (direct adds)
    assert dm.count() == om.count() == len(set(keys.tolist()))
    # every unit either inserted (100) or hit (tag 7)
    assert set(np.unique(dret).tolist()) <= {7, 100}
    assert int((dret == 100).sum()) >= len(o)


def test_parallel_batch_leaves_the_serial_recency_order(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    n, n_keys, cap = 1 << 14, 48, 64
    rng = np.random.default_rng(8)
    keys = rng.integers(0, n_keys, n)
    recs = [(int(k), 0, 5) for k in keys]
    om, dm, _, _ = _run_both(po, dev, recs, cap, dev.BATCH_SYNC)
    # host inserts of new keys now evict in recency order: the stamps the
    # parallel batch left must equal the serial run's order
    for j in range(40):
        k = struct.pack("<I", 1000 + j)
        v = struct.pack("<QQ", 0, j)
        assert dm.update(k, v) == 0 and om.update(k, v) == 0
    assert set(dm.hash_items()) == set(om.items())


def test_parallel_batch_with_overflow_properties(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    n, n_keys, cap = 1 << 16, 5000, 256
    rng = np.random.default_rng(4)
    keys = rng.integers(0, n_keys, n)
    recs = [(int(k), 0, 10_000 + int(k)) for k in keys]
    _, dm, _, dret = _run_both(po, dev, recs, cap, dev.BATCH_SYNC)
    items = dm.hash_items()
    assert dm.count() == cap == len(items)           # full, never above max_entries
    for k, v in items.items():
        key = struct.unpack("<I", k)[0]
        hits, tag = struct.unpack("<QQ", v)
        assert tag == 10_000 + key and hits <= n
    assert set(np.unique(dret).tolist()) <= {99, 100} | {10_000 + k for k in range(n_keys)}


def test_parallel_deletes_and_reinserts_keep_the_table_consistent(fresh_runtime):
    dev = fresh_runtime
    n, n_keys, cap = 1 << 15, 2000, 512
    recs = _script(9, n, n_keys, ops=(0, 0, 2, 1))
    m = dev.Map(LRU, 4, 16, cap)
    vm = dev.VM()
    vm.load(programs.lru_track(m.fd))
    d = dev.DeviceBuffer.from_array(_units(recs))
    for _ in range(20):                                # tombstones pile up, then get compacted
        vm.exec_batch(dev.CTX_RAW, d, n, 16, fixed_len=16)
        items = m.hash_items()
        assert len(items) == m.count() <= cap
    for k in items:
        assert m.lookup(k) is not None


def test_lru_values_take_counter_adds_directly(fresh_runtime):
    dev = fresh_runtime
    m = dev.Map(LRU, 4, 16, 64)
    vm = dev.VM()
    vm.load(programs.lru_track(m.fd))
    assert vm.counter_info(dev.CTX_RAW) == (0, 2)     # the hits adds are never deferred
