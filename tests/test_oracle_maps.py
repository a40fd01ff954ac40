"""Map semantics KATs, ported from the reference's Catch2 unit tests and run
against the oracle (CPU):
  runtime/unit-test/maps/test_bpftime_hash_map.cpp:25-159
  runtime/unit-test/maps/kernel_unit_tests.cpp:371-426 (array), :431-488 (percpu array)
  runtime/unit-test/maps/test_per_cpu_array.cpp:20-80
  runtime/unit-test/maps/test_per_cpu_hash.cpp:22-99
The same assertions run against the device maps in tests/test_gpu_maps.py.
"""
import errno
import random
import struct

from bpftime_amd import isa

I32 = lambda v: struct.pack("<i", v)  # noqa: E731
I64 = lambda v: struct.pack("<q", v)  # noqa: E731


def test_hash_map_basic(fresh_oracle):
    po = fresh_oracle
    # bpftime_hash_map(num_buckets=10, key 4, value 8) via the HASH map type
    m = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 8, 10)
    assert po.lib().orc_map_buckets(m.fd) == 11  # next_prime(10)
    # Insert and Lookup
    assert m.update(I32(1234), I64(5678)) == 0
    assert m.update(I32(4321), I64(8765)) == 0
    assert m.lookup(I32(1234)) == I64(5678)
    assert m.lookup(I32(4321)) == I64(8765)
    assert m.lookup(I32(9999)) is None
    # Update existing
    assert m.update(I32(1234), I64(1)) == 0
    assert m.lookup(I32(1234)) == I64(1)
    assert m.count() == 2
    # Delete
    assert m.delete(I32(1234)) == 0
    assert m.lookup(I32(1234)) is None and m.lookup(I32(4321)) == I64(8765)
    assert m.count() == 1
    assert m.delete(I32(4321)) == 0 and m.count() == 0
    # fix_hash_map::elem_delete returns 0 even if absent (fix_hash_map.cpp:41-45)
    assert m.delete(I32(4321)) == 0


def test_hash_map_full(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 8, 10)
    for i in range(10):
        assert m.update(I32(i), I64(i * 100)) == 0
    # 11th key rejected (bpftime_hash_map.hpp:153-156) but the wrapper returns 0
    assert m.update(I32(10), I64(1000)) == 0
    assert m.lookup(I32(10)) is None
    for i in range(10):
        assert m.lookup(I32(i)) == I64(i * 100)


def test_hash_map_reinsert(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 8, 10)
    m.update(I32(1234), I64(5678))
    m.update(I32(4321), I64(8765))
    m.delete(I32(1234))
    assert m.lookup(I32(1234)) is None
    m.update(I32(5678), I64(4321))
    assert m.lookup(I32(5678)) == I64(4321)
    assert m.lookup(I32(4321)) == I64(8765)


def test_hash_next_key_bucket_order(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 4, 100)
    rnd = random.Random(7)
    keys = rnd.sample(range(1 << 31), 50)
    for k in keys:
        m.update(I32(k), I32(k ^ 1))
    nb = po.lib().orc_map_buckets(m.fd)
    walked = list(m.items().keys())
    assert sorted(walked) == sorted(I32(k) for k in keys)
    # get_next_key walks buckets in index order (fix_hash_map.cpp:47-84):
    # the walk equals the filled slots of the raw [u32 used][key][value] table
    raw = m.raw().reshape(nb, 12)
    filled = [bytes(r[4:8]) for r in raw if r[:4].view("<u4")[0] == 1]
    assert walked == filled


def test_arraymap(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 2)
    assert m.update(I32(1), I64(1234), isa.BPF_ANY) == 0
    assert m.update(I32(1), I64(0), isa.BPF_NOEXIST) < 0 and m.errno() == errno.EEXIST
    assert m.lookup(I32(1)) == I64(1234)
    assert m.lookup(I32(0)) == I64(0)  # zero-initialised
    assert m.update(I32(2), I64(0), isa.BPF_EXIST) < 0 and m.errno() == errno.E2BIG
    assert m.lookup(I32(2)) is None and m.errno() == errno.ENOENT
    assert m.next_key(None) == I32(0)
    assert m.next_key(I32(2)) == I32(0)
    assert m.next_key(I32(0)) == I32(1)
    assert m.next_key(I32(1)) is None and m.errno() == errno.ENOENT
    assert m.delete(I32(1)) < 0 and m.errno() == errno.EINVAL
    assert m.update(I32(0), I64(0), 7) < 0 and m.errno() == errno.EINVAL  # check_update_flags


def test_arraymap_percpu(fresh_oracle):
    po = fresh_oracle
    ncpu = 4
    po.set_ncpu(ncpu)
    m = po.OracleMap(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 2)
    vals = b"".join(I64(i + 100) for i in range(ncpu))
    assert m.update(I32(1), vals, isa.BPF_ANY) == 0
    assert m.update(I32(1), vals, isa.BPF_NOEXIST) < 0 and m.errno() == errno.EEXIST
    assert m.lookup(I32(1))[:8] == I64(100)
    v0 = m.lookup(I32(0))
    assert v0 == b"\0" * 8 * ncpu
    assert m.update(I32(2), vals, isa.BPF_EXIST) < 0 and m.errno() == errno.E2BIG
    assert m.lookup(I32(2)) is None
    assert m.next_key(None) == I32(0) and m.next_key(I32(0)) == I32(1) and m.next_key(I32(1)) is None
    assert m.delete(I32(1)) < 0 and m.errno() == errno.EINVAL


def test_per_cpu_array_helpers_vs_userspace(fresh_oracle):
    po = fresh_oracle
    ncpu = 4
    po.set_ncpu(ncpu)
    m = po.OracleMap(isa.BPF_MAP_TYPE_PERCPU_ARRAY, 4, 8, 10)
    for j in range(ncpu):
        po.set_cpu(j)
        for i in range(10):
            assert m.update(I32(i), struct.pack("<Q", (i << 32) | j), 0, user=False) == 0
    for i in range(10):
        p = struct.unpack(f"<{ncpu}Q", m.lookup(I32(i)))
        assert list(p) == [(i << 32) | j for j in range(ncpu)]


def test_per_cpu_hash_helpers_vs_userspace(fresh_oracle):
    po = fresh_oracle
    ncpu = 4
    po.set_ncpu(ncpu)
    m = po.OracleMap(isa.BPF_MAP_TYPE_PERCPU_HASH, 4, 8, 1 << 20)
    rnd = random.Random(3)
    keys = rnd.sample(range(1 << 32), 100)
    for j in range(ncpu):
        po.set_cpu(j)
        for k in keys:
            assert m.update(struct.pack("<I", k), struct.pack("<Q", (k << 32) | j), 0, user=False) == 0
    for k in keys:
        p = struct.unpack(f"<{ncpu}Q", m.lookup(struct.pack("<I", k)))
        assert list(p) == [(k << 32) | j for j in range(ncpu)]
    # userspace flags (per_cpu_hash_map.cpp:157-183)
    k0 = struct.pack("<I", keys[0])
    assert m.update(k0, b"\0" * 8 * ncpu, isa.BPF_NOEXIST) < 0 and m.errno() == errno.EEXIST
    assert m.update(struct.pack("<I", 1), b"\0" * 8 * ncpu, isa.BPF_EXIST) < 0 and m.errno() == errno.ENOENT


def test_lddw_helpers(fresh_oracle):
    po = fresh_oracle
    m = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 16, 3)
    lib = po.lib()
    assert lib.orc_map_ptr_by_fd(m.fd) == m.fd           # bpftime_shm.cpp:637-652
    assert lib.orc_map_ptr_by_fd(999) == (1 << 64) - 1   # INVALID_MAP_PTR
    assert lib.orc_map_val(m.fd) != 0                    # value of key 0
    assert lib.orc_map_val(999) == 0
