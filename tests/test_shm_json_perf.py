"""Perf event records in the reference's handler JSON
(runtime/src/bpftime_shm_json.cpp:66-95 export, :103-194 import) and
syscall tracepoint ids (attach/syscall_trace_attach_impl/src/
syscall_trace_attach_private_data.cpp:8-63, syscall_table.cpp:17-98).

The reference's own exported state `tools/aot/example/malloc.json` is the
fixture `tests/golden/ref_malloc_shm.json` (copied unchanged): maps 3 (HASH)
and 4 (`.rodata.str1.1` ARRAY), the clang-built 55-instruction `do_count`
uprobe program, a uprobe perf event and the link between them.  Tracepoint
ids come from a tracefs events directory (a test-made one here, with the
layout of /sys/kernel/tracing/events: syscalls/<name>/id and
raw_syscalls/sys_{enter,exit}/id)."""
import ctypes as C
import errno
import json
import os
import struct

import numpy as np
import pytest

from bpftime_amd import _lib, gen, isa, programs

from _helpers import make_maps

HERE = os.path.dirname(os.path.abspath(__file__))
MALLOC = os.path.join(HERE, "golden", "ref_malloc_shm.json")

# tracepoint ids of the test tracefs
TP = {"sys_enter_fork": 101, "sys_exit_fork": 102, "sys_enter_read": 103, "sys_exit_read": 104,
      "sys_enter_write": 105, "sys_enter_umount": 106, "sys_enter_bogus": 107}
TP_ENTER, TP_EXIT = 900, 901


def make_tracefs(root):
    for name, tid in TP.items():
        d = root / "syscalls" / name
        d.mkdir(parents=True)
        (d / "id").write_text(f"{tid}\n")
    for name, tid in (("sys_enter", TP_ENTER), ("sys_exit", TP_EXIT)):
        d = root / "raw_syscalls" / name
        d.mkdir(parents=True)
        (d / "id").write_text(f"{tid}\n")
    return root


@pytest.fixture()
def clean(tmp_path):
    l = _lib.lib()
    l.bpftime_amd_reset()
    l.bpftime_amd_set_tracefs_events(str(make_tracefs(tmp_path / "events")).encode())
    yield l
    l.bpftime_amd_reset()
    l.bpftime_amd_set_tracefs_events(None)


def resolve(l, tid):
    nr, enter = C.c_int64(-7), C.c_int(-7)
    rc = l.bpftime_amd_tracepoint_resolve(tid, C.byref(nr), C.byref(enter))
    return rc, nr.value, enter.value


def perf_get(l, fd):
    e = _lib.PerfEvent()
    assert l.bpftime_amd_perf_event_get(fd, C.byref(e)) == 0
    return e


def export(l, tmp_path):
    out = tmp_path / "export.json"
    assert l.bpftime_export_global_shm_to_json(str(out).encode()) == 0, l.bpftime_amd_last_error()
    return json.loads(out.read_text())


def test_tracepoint_ids_resolve_like_the_reference(clean):
    """test_private_data_parsing.cpp: global enter / exit -> sys_nr -1, a
    sys_enter_fork id -> fork's number, enter; plus exit ids, the umount2 ->
    umount rename, and the -EEXIST failures of initialize_from_string."""
    l = clean
    fork = l.bpftime_amd_syscall_nr(b"fork")
    assert fork == 57 and l.bpftime_amd_syscall_nr(b"read") == 0
    assert l.bpftime_amd_syscall_nr(b"umount") == 166 and l.bpftime_amd_syscall_nr(b"umount2") == -1
    assert resolve(l, TP_ENTER) == (0, -1, 1)
    assert resolve(l, TP_EXIT) == (0, -1, 0)
    assert resolve(l, TP["sys_enter_fork"]) == (0, fork, 1)
    assert resolve(l, TP["sys_exit_read"]) == (0, 0, 0)
    assert resolve(l, TP["sys_enter_umount"]) == (0, 166, 1)
    assert resolve(l, TP["sys_enter_bogus"])[0] == -errno.EEXIST       # no such syscall
    assert resolve(l, 12345)[0] == -errno.EEXIST                        # no such tracepoint
    assert l.bpftime_amd_tracepoint_id(57, 1) == TP["sys_enter_fork"]
    assert l.bpftime_amd_tracepoint_id(-1, 0) == TP_EXIT
    assert l.bpftime_amd_tracepoint_id(2, 1) == -1                      # open: not in this tracefs


def test_missing_tracefs_resolves_nothing(clean, tmp_path):
    l = clean
    l.bpftime_amd_set_tracefs_events(str(tmp_path / "absent").encode())
    assert resolve(l, TP_ENTER)[0] == -errno.EEXIST
    assert l.bpftime_amd_tracepoint_id(-1, 1) == -1


def _no_maps(state):
    return {k: v for k, v in state.items() if v["type"] != "bpf_map_handler"}


def test_reference_export_records_import_and_export_unchanged(clean, tmp_path):
    """The fixture's prog, uprobe perf event and link (fds 5-7) re-created
    with their attributes, exported back identical; the link is a record
    (nothing on this path probes a process)."""
    l = clean
    ref = json.load(open(MALLOC))
    sub = _no_maps(ref)
    p = tmp_path / "in.json"
    p.write_text(json.dumps(sub))
    assert l.bpftime_import_global_shm_from_json(str(p).encode()) == 0, l.bpftime_amd_last_error()
    assert l.bpftime_is_prog_fd(5) and l.bpftime_is_perf_event_fd(6) and l.bpftime_amd_link_attached(7) == 0
    e = perf_get(l, 6)
    assert (e.type, e.pid, e.offset, e.ref_ctr_off, e.enabled) == (6, -1, 676000, 0, 1)
    assert e.module_name == b"/lib/x86_64-linux-gnu/libc.so.6"
    assert export(l, tmp_path) == sub


@pytest.mark.skipif(_lib.lib().bpftime_amd_device_count() > 0, reason="checks the no-device error")
def test_reference_export_maps_need_a_device(clean, tmp_path):
    """Maps live in HBM: without a device the whole-file import fails loudly
    at the first map, naming it."""
    l = clean
    assert l.bpftime_import_global_shm_from_json(MALLOC.encode()) < 0
    assert l.bpftime_amd_last_error().startswith(b"map 3:")


def test_malloc_program_on_the_oracle(tmp_path):
    """The clang-emitted do_count (55 insns) on the oracle: per call it
    prints "malloc called from pid %d\\n" and counts the call in map 3 under
    the pid (lookup, NOEXIST insert of 0, lookup, EXIST update of *v + 1)."""
    from oracle import pyoracle as po
    ref = json.load(open(MALLOC))
    po.reset()
    for fd in ("3", "4"):
        a = ref[fd]["attr"]
        po.OracleMap(a["map_type"], a["key_size"], a["value_size"], a["max_entries"], a["flags"], fd=int(fd))
    code = bytes.fromhex(ref["5"]["attr"]["insns"])
    assert len(code) == 8 * ref["5"]["attr"]["cnt"] == 8 * 55
    vm = po.OracleVM()
    rc, msg = vm.try_load(code)
    # bpf_get_current_pid_tgid (14) is a default helper; bpf_trace_printk is not
    assert rc < 0 and msg == "call to nonexistent function 6 at PC 20"   # compat_ubpf.cpp:83-94
    vm = po.OracleVM()
    vm.register_trace_helpers()
    vm.load(code)
    po.trace_log_reset()
    for pid, calls in ((4242, 5), (77, 2), (4242, 1)):
        po.set_pid_tgid(pid << 32 | 9)
        for _ in range(calls):
            assert vm.exec(bytearray(8)) == (0, 0)
    m = po.OracleMap.__new__(po.OracleMap)
    m.fd, m.key_size, m.value_size = 3, 4, 8
    assert m.items() == {struct.pack("<I", 4242): struct.pack("<Q", 6), struct.pack("<I", 77): struct.pack("<Q", 2)}
    assert po.trace_log() == b"".join(b"malloc called from pid %d\n" % p for p in [4242] * 5 + [77] * 2 + [4242])
    po.reset()


def test_perf_event_kinds_roundtrip(clean, tmp_path):
    """Every perf event kind the reference imports (:130-180) re-created
    with its fields and exported as the reference exports it (:66-95);
    links to the non-tracepoint kinds stay records (a sys_exit tracepoint
    link attaches to the dispatch: tests/test_gpu_syscall_exit.py); an
    unsupported type fails the file."""
    l = clean
    code = programs.kat_mul()
    prog = {"type": "bpf_prog_handler", "name": "p", "attr": {"type": 5, "insns": code.hex(), "cnt": len(code) // 8}}
    state = {
        "3": prog,
        "4": {"type": "bpf_perf_event_handler", "enabled": True,
              "attr": {"type": 2, "pid": 5, "tracepoint_id": TP["sys_exit_read"]}},
        "5": {"type": "bpf_perf_event_handler", "enabled": False,
              "attr": {"type": 7, "pid": 9, "offset": 4096, "ref_ctr_off": 16, "_module_name": "/bin/x"}},
        "6": {"type": "bpf_perf_event_handler", "enabled": False,
              "attr": {"type": 1008, "pid": -1, "offset": 64, "_module_name": "/bin/y"}},
        "7": {"type": "bpf_perf_event_handler", "enabled": True,
              "attr": {"type": 1, "pid": -1, "cpu": 3, "sample_type": 1024, "config": 10}},
        "8": {"type": "bpf_link_handler", "attr": {"prog_fd": 3, "target_fd": 7}},
        "9": {"type": "bpf_link_handler", "attr": {"prog_fd": 3, "target_fd": 5}},
    }
    p = tmp_path / "in.json"
    p.write_text(json.dumps(state))
    assert l.bpftime_import_global_shm_from_json(str(p).encode()) == 0, l.bpftime_amd_last_error()
    e = perf_get(l, 4)
    assert (e.type, e.pid, e.tracepoint_id, e.enabled) == (2, 5, TP["sys_exit_read"], 1)
    e = perf_get(l, 5)
    assert (e.type, e.pid, e.offset, e.ref_ctr_off, e.module_name) == (7, 9, 4096, 16, b"/bin/x")
    e = perf_get(l, 7)
    assert (e.type, e.cpu, e.sample_type, e.config, e.enabled) == (1, 3, 1024, 10, 1)
    assert l.bpftime_amd_link_attached(8) == 0 and l.bpftime_amd_link_attached(9) == 0
    got = export(l, tmp_path)
    assert got["4"] == {"type": "bpf_perf_event_handler", "enabled": True,
                        "attr": {"type": 2, "pid": 5, "tracepoint_id": TP["sys_exit_read"],
                                 "data_type": "tracepoint_perf_event_data"}}
    assert got["5"] == {"type": "bpf_perf_event_handler", "enabled": False,
                        "attr": {"type": 7, "pid": 9, "offset": 4096, "ref_ctr_off": 16, "_module_name": "/bin/x",
                                 "data_type": "uprobe_perf_event_data"}}
    assert got["6"]["attr"]["type"] == 1008 and got["6"]["attr"]["_module_name"] == "/bin/y"
    assert got["7"] == {"type": "bpf_perf_event_handler", "enabled": True,
                        "attr": {"type": 1, "pid": -1, "cpu": 3, "sample_type": 1024, "config": 10,
                                 "data_type": "software_perf_event_shared_ptr"}}
    assert got["8"] == state["8"] and got["9"] == state["9"]
    # enable / disable flip the flag the export carries
    assert l.bpftime_perf_event_disable(4) == 0 and l.bpftime_perf_event_enable(5) == 0
    assert l.bpftime_perf_event_enable(3) < 0                          # not a perf event
    got = export(l, tmp_path)
    assert got["4"]["enabled"] is False and got["5"]["enabled"] is True
    # an unsupported perf event type fails like the reference's (:174-177)
    l.bpftime_amd_reset()
    bad = {"3": {"type": "bpf_perf_event_handler", "enabled": False, "attr": {"type": 3, "pid": -1}}}
    p.write_text(json.dumps(bad))
    assert l.bpftime_import_global_shm_from_json(str(p).encode()) < 0
    assert b"Unsupported perf event type 3" in l.bpftime_amd_last_error()


def test_attach_fds_become_links(clean, tmp_path):
    """A prog's attach_fds (:123-125): a link per fd at a fresh fd, made once
    every record of the file exists (the perf event comes later in the
    file here); the single-handler import links at once."""
    l = clean
    code = programs.kat_mul()
    state = {
        "3": {"type": "bpf_prog_handler", "name": "p",
              "attr": {"type": 5, "insns": code.hex(), "cnt": len(code) // 8, "attach_fds": [4, 5]}},
        "4": {"type": "bpf_perf_event_handler", "enabled": False,
              "attr": {"type": 6, "pid": -1, "offset": 8, "ref_ctr_off": 0, "_module_name": "m"}},
        "5": {"type": "bpf_perf_event_handler", "enabled": False,
              "attr": {"type": 2, "pid": -1, "tracepoint_id": 99999}},   # (no such id here: a record)
    }
    p = tmp_path / "in.json"
    p.write_text(json.dumps(state))
    assert l.bpftime_import_global_shm_from_json(str(p).encode()) == 0, l.bpftime_amd_last_error()
    got = export(l, tmp_path)
    links = sorted((v["attr"]["prog_fd"], v["attr"]["target_fd"]) for v in got.values()
                   if v["type"] == "bpf_link_handler")
    assert links == [(3, 4), (3, 5)]
    assert "attach_fds" not in got["3"]["attr"]       # the reference's export writes none
    h = {"type": "bpf_prog_handler", "name": "q",
         "attr": {"type": 5, "insns": code.hex(), "cnt": len(code) // 8, "attach_fds": [4]}}
    assert l.bpftime_import_shm_handler_from_json(20, json.dumps(h).encode()) == 0
    got = export(l, tmp_path)
    assert sum(1 for v in got.values() if v["type"] == "bpf_link_handler" and v["attr"]["prog_fd"] == 20) == 1


def test_perf_link_checks(clean):
    """bpftime_shm_internal.cpp:566-600 / :282-315: a BPF_PERF_EVENT link
    needs a perf event target (EBADF, also libbpf's target_fd -1 probe);
    BPF_PROG_ATTACH needs a perf fd and a prog fd (ENOENT); an unresolvable
    tracepoint id leaves the link a record that runs nothing, as the
    reference's add_bpf_prog_attach_target / add_bpf_link, which check the
    handler kinds only and resolve the id when the agent attaches."""
    l = clean
    code = programs.kat_mul()
    pfd = l.bpftime_progs_create(-1, code, len(code) // 8, b"p", 5)
    a = _lib.BpfLinkCreateArgs(prog_fd=pfd, target_fd=0xFFFFFFFF, attach_type=41)
    assert l.bpftime_link_create(-1, C.byref(a)) < 0 and C.get_errno() in (0, errno.EBADF)
    tfd = l.bpftime_tracepoint_create(-1, -1, 5555)
    assert tfd > 0 and l.bpftime_is_perf_event_fd(tfd)
    lfd = l.bpftime_attach_perf_to_bpf(tfd, pfd)                       # id 5555 does not resolve here
    assert lfd > 0 and l.bpftime_amd_link_attached(lfd) == 0
    assert l.bpftime_attach_perf_to_bpf(pfd, pfd) < 0 and C.get_errno() == errno.ENOENT  # not a perf fd
    a = _lib.BpfLinkCreateArgs(prog_fd=pfd, target_fd=tfd, attach_type=41)
    lfd2 = l.bpftime_link_create(-1, C.byref(a))
    assert lfd2 > 0 and l.bpftime_amd_link_attached(lfd2) == 0
    a = _lib.BpfLinkCreateArgs(prog_fd=tfd, target_fd=tfd, attach_type=41)
    assert l.bpftime_link_create(-1, C.byref(a)) < 0 and C.get_errno() == errno.EBADF  # not a program
    assert l.bpftime_amd_link_perf(-1, pfd, tfd) > 0                   # the JSON import's record


def _syscall_agg_state(map_fd, prog_fd, code, perf_fd, link_fd, tp_id, extra=None):
    st = {
        str(map_fd): {"type": "bpf_map_handler", "name": "counts",
                      "attr": {"map_type": 1, "key_size": 4, "value_size": 32, "max_entries": 8192, "flags": 0,
                               "ifindex": 0, "btf_vmlinux_value_type_id": 0, "btf_id": 0, "btf_key_type_id": 0,
                               "btf_value_type_id": 0, "map_extra": 0, "kernel_bpf_map_id": 0}},
        str(prog_fd): {"type": "bpf_prog_handler", "name": "syscount",
                       "attr": {"type": 5, "insns": code.hex(), "cnt": len(code) // 8}},
        str(perf_fd): {"type": "bpf_perf_event_handler", "enabled": True,
                       "attr": {"type": 2, "pid": -1, "tracepoint_id": tp_id}},
        str(link_fd): {"type": "bpf_link_handler", "attr": {"prog_fd": prog_fd, "target_fd": perf_fd}},
    }
    st.update(extra or {})
    return st


@pytest.mark.gpu
def test_reference_export_imports_on_device(clean, tmp_path):
    """The whole fixture on the device: fds 3-7 with their attributes, the
    export identical to the reference's file; do_count itself is refused by
    the device loader, naming the helper (compat_ubpf.cpp:83-94)."""
    from bpftime_amd import vm as dev
    l = clean
    ref = json.load(open(MALLOC))
    assert l.bpftime_import_global_shm_from_json(MALLOC.encode()) == 0, l.bpftime_amd_last_error()
    assert l.bpftime_is_map_fd(3) and l.bpftime_is_map_fd(4) and l.bpftime_is_prog_fd(5)
    assert l.bpftime_is_perf_event_fd(6) and l.bpftime_amd_link_attached(7) == 0
    assert export(l, tmp_path) == ref
    with pytest.raises(dev.EbpfError, match="function 6 at PC 20"):
        dev.prog_instantiate(5)


@pytest.mark.gpu
def test_tracepoint_state_runs_the_dispatch(fresh_oracle, fresh_runtime, clean, tmp_path):
    """A syscall-agg state attached to raw_syscalls:sys_enter (global) and a
    read counter attached to sys_enter_read, imported from JSON by
    tracepoint id, and the read counter also attached to sys_exit_read,
    replayed through bpftime_amd_syscall_dispatch_records over 96-B records
    bit-exact against the oracle's dispatch; the export round-trips and
    re-imports into the same attachments."""
    po, dev, l = fresh_oracle, fresh_runtime, clean
    l.bpftime_amd_set_tracefs_events(str(tmp_path / "events").encode())
    code = programs.syscall_agg(3)
    from test_gpu_syscall_dispatch import counter_prog
    rd = counter_prog(9, 0)
    extra = {
        "9": {"type": "bpf_map_handler", "name": "reads",
              "attr": {"map_type": 2, "key_size": 4, "value_size": 8, "max_entries": 1, "flags": 0,
                       "ifindex": 0, "btf_vmlinux_value_type_id": 0, "btf_id": 0, "btf_key_type_id": 0,
                       "btf_value_type_id": 0, "map_extra": 0, "kernel_bpf_map_id": 0}},
        "10": {"type": "bpf_prog_handler", "name": "reads", "attr": {"type": 5, "insns": rd.hex(),
                                                                   "cnt": len(rd) // 8}},
        "11": {"type": "bpf_perf_event_handler", "enabled": True,
               "attr": {"type": 2, "pid": -1, "tracepoint_id": TP["sys_enter_read"]}},
        "12": {"type": "bpf_link_handler", "attr": {"prog_fd": 10, "target_fd": 11}},
        "13": {"type": "bpf_perf_event_handler", "enabled": True,
               "attr": {"type": 2, "pid": -1, "tracepoint_id": TP["sys_exit_read"]}},
        "14": {"type": "bpf_link_handler", "attr": {"prog_fd": 10, "target_fd": 13}},
    }
    state = _syscall_agg_state(3, 5, code, 6, 7, TP_ENTER, extra)
    p = tmp_path / "state.json"
    p.write_text(json.dumps(state))
    n = 60000
    recs = gen.syscall_records_full(n)
    ids_col = recs.view(np.int64).reshape(n, 12)[:, 1]

    def run_and_check():
        assert [l.bpftime_amd_link_attached(f) for f in (7, 12, 14)] == [1, 1, 1]
        po.reset()
        om = po.OracleMap(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192, fd=3)
        orm = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 1, fd=9)
        d = dev.DeviceBuffer.from_array(recs)
        # a sys_exit program is attached: 64-B records hold no exit ctx
        assert l.bpftime_amd_syscall_dispatch(d.ptr, n, dev.BATCH_SYNC, None) == -1
        assert dev.syscall_dispatch(d, n) == 0
        od = po.OracleSyscallDispatch()
        od.attach(code, -1, enter=True)
        od.attach(rd, 0, enter=True)
        od.attach(rd, 0, enter=False)
        od.dispatch(recs)
        assert dev.Map.from_fd(3).hash_items() == om.items()
        assert dev.Map.from_fd(9).lookup(b"\0\0\0\0") == orm.lookup(b"\0\0\0\0")
        # the read counter runs at sys_enter_read and at sys_exit_read
        assert struct.unpack("<Q", orm.lookup(b"\0\0\0\0"))[0] == 2 * int((ids_col == 0).sum()) > 0
        assert len(om.items()) > 100

    assert l.bpftime_import_global_shm_from_json(str(p).encode()) == 0, l.bpftime_amd_last_error()
    run_and_check()
    got = export(l, tmp_path)
    for fd in ("6", "7", "11", "12", "13", "14"):
        assert {k: v for k, v in got[fd].items()} == {**state[fd], **({"attr": {**state[fd]["attr"],
                                                                               "data_type":
                                                                               "tracepoint_perf_event_data"}}
                                                                      if state[fd]["type"] ==
                                                                      "bpf_perf_event_handler" else {})}
    # re-import the export into a fresh runtime: the same attachments
    l.bpftime_amd_reset()
    p2 = tmp_path / "again.json"
    p2.write_text(json.dumps(got))
    assert l.bpftime_import_global_shm_from_json(str(p2).encode()) == 0, l.bpftime_amd_last_error()
    run_and_check()
    # closing the link detaches the program
    _lib.lib().bpftime_close(7)
    d = dev.DeviceBuffer.from_array(recs)
    before = dev.Map.from_fd(3).hash_items()
    assert dev.syscall_dispatch(d, n) == 0
    assert dev.Map.from_fd(3).hash_items() == before
