"""Oracle LRU hash map (oracle/maps.c, restating lru_var_hash_map.cpp) pinned
by the reference's own LRU unit tests (tests/_lru_cases.py)."""
import pytest

import _lru_cases as L
from bpftime_amd import isa


@pytest.fixture
def make(fresh_oracle):
    po = fresh_oracle

    def mk(cap, ks, vs):
        return po.OracleMap(isa.BPF_MAP_TYPE_LRU_HASH, ks, vs, cap)
    return mk


@pytest.mark.parametrize("case", L.ALL, ids=lambda f: f.__name__)
def test_reference_lru_unit_tests(case, make, fresh_oracle):
    case(make, fresh_oracle.OracleMap.errno)


def test_lru_recency_order_is_the_eviction_order(make, fresh_oracle):
    # every touch (lookup hit, update of an existing key) moves to the head;
    # inserts past capacity evict the tail, one per insert
    m = make(4, 4, 8)
    for k in range(4):
        assert m.update(L.u32(k), L.u64(k)) == 0
    m.lookup(L.u32(0))                       # order (tail..head): 1 2 3 0
    m.update(L.u32(1), L.u64(11), L.BPF_EXIST)   # 2 3 0 1
    m.update(L.u32(7), L.u64(7))             # evicts 2: 3 0 1 7
    m.update(L.u32(8), L.u64(8))             # evicts 3: 0 1 7 8
    assert m.update(L.u32(9), L.u64(9), L.BPF_EXIST) == -1     # EXIST never inserts
    assert m.update(L.u32(0), L.u64(5), L.BPF_NOEXIST) == -1   # a failed NOEXIST does not touch
    m.update(L.u32(10), L.u64(10))           # evicts 0: 1 7 8 10
    assert m.count() == 4
    for k in (0, 2, 3, 9):
        assert m.lookup(L.u32(k)) is None
    assert m.lookup(L.u32(1)) == L.u64(11)
    for k in (7, 8, 10):
        assert m.lookup(L.u32(k)) == L.u64(k)


def test_lru_rejects_empty_geometry(fresh_oracle):
    with pytest.raises(RuntimeError):
        fresh_oracle.OracleMap(isa.BPF_MAP_TYPE_LRU_HASH, 4, 8, 0)
