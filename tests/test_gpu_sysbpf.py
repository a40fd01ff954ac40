"""A libbpf loader's bpf(2) sequence through bpftime_amd_handle_sysbpf
(runtime/syscall-server/syscall_context.cpp:429-668): BPF_MAP_CREATE for
xdp-counter's two maps, BPF_MAP_UPDATE_ELEM of ctl_array, BPF_PROG_LOAD,
BPF_LINK_CREATE(BPF_XDP); the runner finds the link, runs a batch on the
device, and the loader reads the counter back with BPF_MAP_LOOKUP_ELEM --
verdicts, packets and the counter against the oracle."""
import ctypes as C
import errno
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs

from _helpers import xdp_counter_maps

pytestmark = pytest.mark.gpu


def _buf(b):
    a = bytearray(b)
    return a, C.addressof((C.c_char * max(len(a), 1)).from_buffer(a))


def test_libbpf_sequence_through_sysbpf(fresh_oracle, fresh_runtime):
    po, dev = fresh_oracle, fresh_runtime
    ctl, e = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array"))
    assert ctl >= 0, e
    bss, e = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1,
                                                                 name="xdp_coun.bss"))
    assert bss >= 0 and bss != ctl
    k, kp = _buf(struct.pack("<I", 0))
    v, vp = _buf(struct.pack("<I", 0))
    assert dev.sys_bpf(dev.BPF_MAP_UPDATE_ELEM, dev.attr_map_elem(ctl, kp, vp, isa.BPF_ANY))[0] == 0
    code = programs.xdp_counter(ctl, bss)
    ins, ip = _buf(code)
    pfd, e = dev.sys_bpf(dev.BPF_PROG_LOAD, dev.attr_prog_load(6, ip, len(code) // 8, name="xdp_pass"))
    assert pfd >= 0, e
    lfd, e = dev.sys_bpf(dev.BPF_LINK_CREATE, dev.attr_link_create(pfd, 3, 37))
    assert lfd >= 0, e
    assert dev.sys_bpf(dev.BPF_LINK_CREATE, dev.attr_link_create(999, 3, 37))[0] == -1
    links = dev.xdp_links()
    assert (lfd, pfd, 3) in links
    vm = dev.prog_instantiate(pfd)
    n = 5000
    pk = gen.xdp_packets(n, seed=44)
    (octl, obss), _ = xdp_counter_maps(po, None)
    ovm = po.OracleVM()
    ovm.load(programs.xdp_counter(octl.fd, obss.fd))
    opk = pk.copy()
    ov = ovm.run_xdp(opk, fixed_len=64)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    out, op = _buf(bytes(4096))
    assert dev.sys_bpf(dev.BPF_MAP_LOOKUP_ELEM, dev.attr_map_elem(bss, kp, op))[0] == 0
    assert bytes(out) == obss.lookup(struct.pack("<I", 0))
    assert struct.unpack_from("<Q", out)[0] == n
    # syscall-side errors: array key out of range, delete on an array, last key
    k2, k2p = _buf(struct.pack("<I", 2))
    assert dev.sys_bpf(dev.BPF_MAP_LOOKUP_ELEM, dev.attr_map_elem(ctl, k2p, vp)) == (-1, errno.ENOENT)
    assert dev.sys_bpf(dev.BPF_MAP_DELETE_ELEM, dev.attr_map_elem(ctl, kp))[0] == -1
    nk, nkp = _buf(bytes(4))
    assert dev.sys_bpf(dev.BPF_MAP_GET_NEXT_KEY, dev.attr_map_elem(ctl, 0, nkp))[0] == 0 and bytes(nk) == bytes(4)
    k1, k1p = _buf(struct.pack("<I", 1))
    assert dev.sys_bpf(dev.BPF_MAP_GET_NEXT_KEY, dev.attr_map_elem(ctl, k1p, nkp))[0] == -1


BPF_PROG_ATTACH, BPF_OBJ_GET_INFO_BY_FD, BPF_MAP_LOOKUP_AND_DELETE_ELEM = 8, 15, 21


def test_bss_mmap_view_write_read(fresh_oracle, fresh_runtime):
    """libbpf's .bss handling (syscall_context.cpp:515-528, 915-920): create
    the MMAPABLE array, write its initial bytes with BPF_MAP_UPDATE_ELEM, mmap
    it (bpftime_get_array_map_raw_data), then read and write globals through
    the mapping while batches run on the device."""
    po, dev = fresh_oracle, fresh_runtime
    L = dev.lib()
    ctl, _ = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, name="ctl_array"))
    bss, e = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1,
                                                                 flags=isa.BPF_F_MMAPABLE, name="xdp_coun.bss"))
    assert bss >= 0, e
    init = bytearray(4096)
    struct.pack_into("<QQ", init, 8, 7, 9)          # cntrs_array[1] = 7, [2] = 9 (initialised .bss)
    k, kp = _buf(struct.pack("<I", 0))
    iv, ivp = _buf(init)
    assert dev.sys_bpf(dev.BPF_MAP_UPDATE_ELEM, dev.attr_map_elem(bss, kp, ivp, isa.BPF_ANY))[0] == 0
    p = L.bpftime_get_array_map_raw_data(bss)
    assert p and p % 4096 == 0
    view = (C.c_uint64 * 512).from_address(p)
    assert (view[0], view[1], view[2]) == (0, 7, 9)
    assert L.bpftime_get_array_map_raw_data(bss) == p        # one stable view per map
    assert not L.bpftime_get_array_map_raw_data(ctl + 1000)
    view[2] = 42                                          # the loader writes a global
    code = programs.xdp_counter(ctl, bss)
    ins, ip = _buf(code)
    pfd, _ = dev.sys_bpf(dev.BPF_PROG_LOAD, dev.attr_prog_load(6, ip, len(code) // 8, name="xdp_pass"))
    assert dev.sys_bpf(dev.BPF_LINK_CREATE, dev.attr_link_create(pfd, 3, 37))[0] >= 0
    vm = dev.prog_instantiate(pfd)
    # a reader of cntrs_array[2]: the host write reaches the device before the launch
    rd = dev.VM()
    rd.load(isa.Asm().ld_map_value(1, bss, 16).ldx(8, 0, 1, 0).exit().assemble())
    n = 3000
    pk = dev.DeviceBuffer.from_array(gen.xdp_packets(n, seed=9))
    dv = dev.DeviceBuffer(4 * n)
    assert rd.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv) == 0
    assert (dv.download(np.uint32) == 42).all()
    assert vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv) == 0   # synchronous: view refreshed
    assert (view[0], view[1], view[2]) == (n, 7, 42)
    # an asynchronous batch reaches the view on msync
    assert vm.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0) == 0
    assert L.bpftime_amd_map_msync(bss) == 0 and view[0] == 2 * n
    out, op = _buf(bytes(4096))
    assert dev.sys_bpf(dev.BPF_MAP_LOOKUP_ELEM, dev.attr_map_elem(bss, kp, op))[0] == 0
    assert struct.unpack_from("<QQQ", out) == (2 * n, 7, 42)
    # host writes on both sides of a counter an asynchronous batch is
    # advancing: only the written bytes reach the device, so the counter's
    # increments the view has not seen survive (the push used to upload the
    # whole span between the first and last changed byte, stale counter
    # included)
    inc = dev.VM()
    inc.load(isa.Asm().ld_map_value(1, bss, 8).mov64(2, 1).atomic(8, isa.ATOMIC_ADD, 1, 0, "r2")
             .mov64(0, 2).exit().assemble())
    c0 = view[1]
    assert inc.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0) == 0
    view[0], view[2] = 111, 222
    assert inc.exec_batch(dev.CTX_XDP, pk, n, 64, fixed_len=64, verdicts=dv, flags=0) == 0
    assert L.bpftime_amd_map_msync(bss) == 0
    assert (view[0], view[1], view[2]) == (111, c0 + 2 * n, 222)
    dev.close_fd(bss)
    assert L.bpftime_amd_map_msync(bss) == -1


def test_obj_get_info_and_lookup_and_delete(fresh_runtime):
    dev = fresh_runtime
    m, _ = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_HASH, 8, 16, 100, name="flows"))
    info = bytearray(88)
    buf = (C.c_char * len(info)).from_buffer(info)
    a = bytearray(128)
    struct.pack_into("<IIQ", a, 0, m, len(info), C.addressof(buf))
    assert dev.sys_bpf(BPF_OBJ_GET_INFO_BY_FD, a)[0] == 0
    typ, mid, ks, vs, mx, fl = struct.unpack_from("<IIIIII", info, 0)
    assert (typ, mid, ks, vs, mx, fl) == (isa.BPF_MAP_TYPE_HASH, m, 8, 16, 100, 0)
    assert info[24:29] == b"flows"
    code = programs.kat_mul()
    ins = (C.c_char * len(code)).from_buffer(bytearray(code))
    pfd, _ = dev.sys_bpf(dev.BPF_PROG_LOAD, dev.attr_prog_load(1, C.addressof(ins), len(code) // 8, name="p"))
    pinfo = bytearray(64)
    pb = (C.c_char * len(pinfo)).from_buffer(pinfo)
    struct.pack_into("<IIQ", a, 0, pfd, len(pinfo), C.addressof(pb))
    assert dev.sys_bpf(BPF_OBJ_GET_INFO_BY_FD, a)[0] == 0 and struct.unpack_from("<II", pinfo)[1] == pfd
    # map_pop_elem exists for queue / stack maps only (map_handler.cpp:1411-1434)
    v, vp = _buf(bytes(16))
    assert dev.sys_bpf(BPF_MAP_LOOKUP_AND_DELETE_ELEM, dev.attr_map_elem(m, 0, vp))[0] == -errno.ENOTSUP
    assert dev.sys_bpf(BPF_MAP_LOOKUP_AND_DELETE_ELEM, dev.attr_map_elem(pfd, 0, vp))[0] == -1


def test_prog_attach_to_syscall_perf_event(fresh_oracle, fresh_runtime):
    """BPF_PROG_ATTACH(prog, perf fd) (syscall_context.cpp:723-735 ->
    bpftime_attach_perf_to_bpf): the program runs on that syscall's enter
    records in the dispatch; closing the link detaches it."""
    po, dev = fresh_oracle, fresh_runtime
    L = dev.lib()
    cm, _ = dev.sys_bpf(dev.BPF_MAP_CREATE, dev.attr_map_create(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, name="counts"))
    code = programs.syscall_agg(cm)
    ins = (C.c_char * len(code)).from_buffer(bytearray(code))
    pfd, _ = dev.sys_bpf(dev.BPF_PROG_LOAD, dev.attr_prog_load(5, C.addressof(ins), len(code) // 8, name="sys"))
    perf = L.bpftime_amd_perf_event_syscall(-1, 1)          # syscalls:sys_enter_write
    assert perf >= 0 and L.bpftime_is_perf_event_fd(perf)
    a = bytearray(128)
    struct.pack_into("<IIII", a, 0, pfd, pfd, 0, 0)           # target is not a perf event
    assert dev.sys_bpf(BPF_PROG_ATTACH, a) == (-1, errno.ENOENT)
    struct.pack_into("<IIII", a, 0, perf, pfd, 0, 0)
    link, e = dev.sys_bpf(BPF_PROG_ATTACH, a)
    assert link >= 0, e
    n = 30000
    recs = gen.syscall_records(n)
    d = dev.DeviceBuffer.from_array(recs)
    assert L.bpftime_amd_syscall_dispatch(d.ptr, n, dev.BATCH_SYNC, None) == 0
    om = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, fd=cm)
    ovm = po.OracleVM()
    ovm.load(code)
    ids = recs.view(np.uint64)[:, 1]
    ovm.run_syscall(recs[ids == 1].copy())
    got = dev.Map.from_fd(cm)
    got.key_size, got.value_size = 4, 32
    k = struct.pack("<I", 1)
    assert got.lookup(k) == om.lookup(k) and struct.unpack_from("<Q", got.lookup(k))[0] == (ids == 1).sum()
    assert got.lookup(struct.pack("<I", 0)) is None
    dev.close_fd(link)                                        # detached
    assert L.bpftime_amd_syscall_dispatch(d.ptr, n, dev.BATCH_SYNC, None) == 0
    assert got.lookup(k) == om.lookup(k)
