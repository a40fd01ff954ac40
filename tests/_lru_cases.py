"""The reference's LRU hash map unit tests, restated over any map object with
lookup / update / delete / next_key (the oracle's OracleMap, the device
runtime's Map).  Sources:
  runtime/unit-test/maps/test_lru_var_hash_map.cpp (basic ops, capacity-5 eviction)
  runtime/unit-test/maps/test_lru_hash_map.cpp (basic, eviction, flags, capacity, iteration)
`make(max_entries, key_size, value_size)` returns a fresh map; `errno()` the
last error of the implementation under test."""
import struct

BPF_ANY, BPF_NOEXIST, BPF_EXIST = 0, 1, 2
ENOENT, EEXIST, EINVAL = 2, 17, 22


def i32(x):
    return struct.pack("<i", x)


def u32(x):
    return struct.pack("<I", x)


def u64(x):
    return struct.pack("<Q", x)


def var_hash_basic(make, errno):
    """test_lru_var_hash_map.cpp 'Test basic lru map operations'."""
    m = make(1000, 4, 4)
    for i in range(500):
        assert m.update(i32(i), i32(500 + i), BPF_NOEXIST) == 0
    for i in range(499, -1, -1):
        assert m.lookup(i32(i)) == i32(i + 500)
    for i in range(500):
        assert m.update(i32(i), i32(5000 + i), BPF_EXIST) == 0
    for i in range(499, -1, -1):
        assert m.lookup(i32(i)) == i32(i + 5000)
    for i in range(0, 500, 2):
        assert m.delete(i32(i)) == 0
    for i in range(499, -1, -1):
        v = m.lookup(i32(i))
        assert (v is None) if i % 2 == 0 else (v == i32(i + 5000))
    m = make(5, 4, 4)
    for i in range(5):
        assert m.update(i32(i), i32(i), BPF_NOEXIST) == 0
    for i in range(5):
        if i != 3:
            assert m.lookup(i32(i)) == i32(i)
    assert m.update(i32(10), i32(10), BPF_NOEXIST) == 0
    assert m.lookup(i32(10)) == i32(10)
    assert m.lookup(i32(3)) is None       # the least recently used element went


def basic_ops(make, errno):
    """test_lru_hash_map.cpp 'LRU Hash Map Basic Operations' (its three sections)."""
    cap = 10
    m = make(cap, 4, 8)
    for i in range(cap):
        assert m.update(u32(i), u64(i * 100), BPF_NOEXIST) == 0
    for i in range(cap):
        assert m.lookup(u32(i)) == u64(i * 100)
    m = make(cap, 4, 8)
    for i in range(cap):
        assert m.update(u32(i), u64(i), BPF_NOEXIST) == 0
    for i in range(1, cap):
        assert m.lookup(u32(i)) is not None
    assert m.update(u32(cap), u64(999), BPF_NOEXIST) == 0
    assert m.lookup(u32(cap)) == u64(999)
    assert m.lookup(u32(0)) is None and errno() == ENOENT
    m = make(cap, 4, 8)
    assert m.update(u32(42), u64(123), BPF_NOEXIST) == 0
    assert m.update(u32(42), u64(456), BPF_EXIST) == 0
    assert m.lookup(u32(42)) == u64(456)
    assert m.delete(u32(42)) == 0
    assert m.lookup(u32(42)) is None and errno() == ENOENT
    assert m.delete(u32(42)) == -1 and errno() == ENOENT


def update_flags(make, errno):
    """test_lru_hash_map.cpp 'LRU Hash Map Update Flags' (+ the exact-flag rule
    of lru_var_hash_map.cpp:8-11: anything but 0/1/2 is EINVAL)."""
    k, v1, v2 = u32(123), u64(456), u64(789)
    m = make(10, 4, 8)
    assert m.update(k, v1, BPF_NOEXIST) == 0
    assert m.lookup(k) == v1
    assert m.update(k, v2, BPF_NOEXIST) == -1 and errno() == EEXIST
    m = make(10, 4, 8)
    assert m.update(k, v1, BPF_NOEXIST) == 0
    assert m.update(k, v2, BPF_EXIST) == 0
    assert m.lookup(k) == v2
    assert m.delete(k) == 0
    assert m.update(k, v1, BPF_EXIST) == -1 and errno() == ENOENT
    m = make(10, 4, 8)
    assert m.update(k, v1, BPF_ANY) == 0
    assert m.update(k, v2, BPF_ANY) == 0
    assert m.lookup(k) == v2
    assert m.update(k, v1, 4) == -1 and errno() == EINVAL
    assert m.update(k, v1, (1 << 32) | BPF_ANY) == -1 and errno() == EINVAL


def capacity(make, errno):
    """test_lru_hash_map.cpp 'LRU Hash Map Capacity Limits'."""
    cap = 5
    m = make(cap, 4, 8)
    for i in range(cap):
        assert m.update(u32(i), u64(i * 10), BPF_NOEXIST) == 0
    for i in range(cap):
        assert m.lookup(u32(i)) == u64(i * 10)
    assert m.update(u32(cap), u64(999), BPF_NOEXIST) == 0
    assert m.lookup(u32(cap)) == u64(999)
    assert m.count() == cap
    assert m.lookup(u32(0)) is None       # key 0 was the list tail


def iteration(make, errno):
    """test_lru_hash_map.cpp 'LRU Hash Map Iteration'."""
    m = make(8, 4, 8)
    assert m.next_key(None) is None and errno() == ENOENT
    keys = [10, 20, 30, 40]
    for k in keys:
        assert m.update(u32(k), u64(2 * k), BPF_NOEXIST) == 0
    visited, cur = set(), m.next_key(None)
    while cur is not None:
        visited.add(struct.unpack("<I", cur)[0])
        cur = m.next_key(cur)
    assert errno() == ENOENT
    assert visited == set(keys)
    nk = m.next_key(u32(9999))                # a missing key restarts at the first
    assert nk is not None and struct.unpack("<I", nk)[0] in visited


ALL = [var_hash_basic, basic_ops, update_flags, capacity, iteration]


def lru_script(seed, n_ops, n_keys, cap):
    """A random mixed op sequence: (op, key, value, flags) tuples."""
    import random
    rnd = random.Random(seed)
    out = []
    for _ in range(n_ops):
        op = rnd.choice("lluud")
        k = rnd.randrange(n_keys)
        out.append((op, k, rnd.randrange(1 << 32), rnd.choice([0, 0, 1, 2])))
    return out


def replay(m, script, errno):
    """Run a script against a map; the (result, errno) trace."""
    tr = []
    for op, k, v, f in script:
        if op == "l":
            r = m.lookup(u32(k))
            tr.append((op, k, r, 0 if r is not None else errno()))
        elif op == "u":
            r = m.update(u32(k), u64(v), f)
            tr.append((op, k, r, errno() if r else 0))
        else:
            r = m.delete(u32(k))
            tr.append((op, k, r, errno() if r else 0))
    return tr
