"""LPM trie: the oracle against the assertions of the
reference's runtime/unit-test/maps/test_lpm_trie_map.cpp:1093-1350
(constructor validation, IPv4 operations, longest-prefix match, deletion,
update flags, full map).  lpm_kats() runs unchanged against the device
registry in tests/test_gpu_lpm.py."""
import errno
import socket
import struct

import pytest

from bpftime_amd import isa

LPM = isa.BPF_MAP_TYPE_LPM_TRIE


def k4(plen, dotted):
    """struct bpf_lpm_trie_key {u32 prefixlen; u8 data[4]} with network-order data."""
    return struct.pack("<I", plen) + socket.inet_aton(dotted)


def u32(v):
    return struct.pack("<I", v)


def lpm_kats(make, err=lambda: None):
    # IPv4 operations (test_lpm_trie_map.cpp:1143-1187)
    m = make(LPM, 8, 4, 10)
    assert m.update(k4(16, "192.168.0.0"), u32(1)) == 0 and m.count() == 1
    assert m.lookup(k4(32, "192.168.0.1")) == u32(1)
    assert m.update(k4(24, "192.168.1.0"), u32(2)) == 0 and m.count() == 2
    assert m.lookup(k4(32, "192.168.1.1")) == u32(2)
    assert m.lookup(k4(32, "192.168.2.1")) == u32(1)
    # invalid prefix length (:1215-1237)
    assert m.update(k4(40, "192.168.0.0"), u32(1)) == -1 and err() in (None, errno.EINVAL)
    assert m.lookup(k4(40, "192.168.0.0")) is None
    # deletion (:1189-1213)
    m = make(LPM, 8, 4, 10)
    assert m.update(k4(24, "192.168.0.0"), u32(100)) == 0
    assert m.lookup(k4(24, "192.168.0.0")) == u32(100)
    assert m.delete(k4(24, "192.168.0.0")) == 0 and m.count() == 0
    assert m.lookup(k4(24, "192.168.0.0")) is None and err() in (None, errno.ENOENT)
    assert m.delete(k4(24, "192.168.0.0")) == -1
    # longest prefix match (:1263-1350)
    m = make(LPM, 8, 4, 20)
    for plen, net, v in ((8, "10.0.0.0", 1), (16, "10.1.0.0", 2), (24, "10.1.1.0", 3), (25, "10.1.1.128", 4)):
        assert m.update(k4(plen, net), u32(v)) == 0
    assert m.count() == 4
    for addr, v in (("10.1.1.200", 4), ("10.1.1.50", 3), ("10.1.2.1", 2), ("10.2.0.1", 1)):
        assert m.lookup(k4(32, addr)) == u32(v), addr
    assert m.lookup(k4(32, "192.168.1.1")) is None
    # update flags and a full map (BPF_NOEXIST / BPF_EXIST, ENOSPC)
    m = make(LPM, 8, 4, 2)
    assert m.update(k4(8, "10.0.0.0"), u32(1), isa.BPF_EXIST) == -1
    assert m.update(k4(8, "10.0.0.0"), u32(1), isa.BPF_NOEXIST) == 0
    assert m.update(k4(8, "10.0.0.0"), u32(2), isa.BPF_NOEXIST) == -1
    assert m.update(k4(8, "10.0.0.0"), u32(3), isa.BPF_EXIST) == 0 and m.lookup(k4(32, "10.9.9.9")) == u32(3)
    assert m.update(k4(16, "10.1.0.0"), u32(4)) == 0
    assert m.update(k4(24, "10.1.2.0"), u32(5)) == -1 and err() in (None, errno.ENOSPC)
    assert m.update(k4(16, "10.1.0.0"), u32(6)) == 0          # existing key: no room needed
    assert m.update(k4(8, "10.0.0.0"), u32(1), 4) == -1        # bad flags
    # deleted node stays as an intermediate: re-insert reuses it
    assert m.delete(k4(8, "10.0.0.0")) == 0 and m.count() == 1
    assert m.lookup(k4(32, "10.9.9.9")) is None and m.lookup(k4(32, "10.1.9.9")) == u32(6)
    assert m.update(k4(8, "10.0.0.0"), u32(7), isa.BPF_EXIST) == -1
    assert m.update(k4(8, "10.0.0.0"), u32(7)) == 0 and m.lookup(k4(32, "10.9.9.9")) == u32(7)
    # get_next_key: the first key only (lpm_trie_map.cpp:543-590)
    first = m.next_key(None)
    assert first is not None and m.next_key(first) is None


def test_oracle_lpm_kats(fresh_oracle):
    po = fresh_oracle
    lpm_kats(lambda t, k, v, mx: po.OracleMap(t, k, v, mx), po.OracleMap.errno)


@pytest.mark.parametrize("ksize,vsize,mx", [(3, 4, 10), (4, 4, 10), (261, 4, 10), (8, 0, 10), (8, 4, 0)])
def test_oracle_lpm_constructor_validation(fresh_oracle, ksize, vsize, mx):
    with pytest.raises(RuntimeError):
        fresh_oracle.OracleMap(LPM, ksize, vsize, mx)
