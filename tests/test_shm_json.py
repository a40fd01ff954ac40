"""The reference's handler JSON (runtime/src/bpftime_shm_json.cpp:103-327):
import / export of prog and link records without a GPU, and a whole
reference-format state (maps + xdp-counter + XDP link) imported and run on
the device against the oracle."""
import ctypes
import json
import struct

import numpy as np
import pytest

from bpftime_amd import _lib, gen, isa, programs

C_int, C_u32 = ctypes.c_int, ctypes.c_uint32


def reference_state(ctl_fd=3, bss_fd=4, prog_fd=5, link_fd=6, ifindex=2):
    """What `bpftimetool export` writes for the xdp-counter example (field
    names and encodings of bpftime_shm_json.cpp: hex insns, map attrs)."""
    code = programs.xdp_counter(ctl_fd, bss_fd)
    attr = lambda t, k, v, m, f: {"map_type": t, "key_size": k, "value_size": v, "max_entries": m,  # noqa
                                  "flags": f, "ifindex": 0, "btf_vmlinux_value_type_id": 0, "btf_id": 0,
                                  "btf_key_type_id": 0, "btf_value_type_id": 0, "map_extra": 0,
                                  "kernel_bpf_map_id": 0}
    return code, {
        str(ctl_fd): {"type": "bpf_map_handler", "name": "ctl_array", "attr": attr(2, 4, 4, 2, 0)},
        str(bss_fd): {"type": "bpf_map_handler", "name": "xdp_coun.bss", "attr": attr(2, 4, 4096, 1, 0x400)},
        str(prog_fd): {"type": "bpf_prog_handler", "name": "xdp_pass",
                       "attr": {"type": 6, "insns": code.hex(), "cnt": len(code) // 8, "attach_fds": []}},
        str(link_fd): {"type": "bpf_link_handler", "attr": {"prog_fd": prog_fd, "target_fd": ifindex}},
    }


@pytest.fixture()
def clean():
    l = _lib.lib()
    l.bpftime_amd_reset()
    yield l
    l.bpftime_amd_reset()


def test_prog_and_link_roundtrip(clean, tmp_path):
    l = clean
    code, state = reference_state()
    sub = {k: v for k, v in state.items() if v["type"] != "bpf_map_handler"}
    p = tmp_path / "in.json"
    p.write_text(json.dumps(sub, indent=4))
    assert l.bpftime_import_global_shm_from_json(str(p).encode()) == 0
    assert l.bpftime_is_prog_fd(5)
    links = (C_int * 4)()
    progs = (C_int * 4)()
    ifx = (C_u32 * 4)()
    assert l.bpftime_amd_xdp_links(links, progs, ifx, 4) == 1      # XDP prog -> BPF_XDP link
    assert (links[0], progs[0], ifx[0]) == (6, 5, 2)
    out = tmp_path / "out.json"
    assert l.bpftime_export_global_shm_to_json(str(out).encode()) == 0
    got = json.loads(out.read_text())
    assert got["5"]["type"] == "bpf_prog_handler" and got["5"]["name"] == "xdp_pass"
    assert bytes.fromhex(got["5"]["attr"]["insns"]) == code and got["5"]["attr"]["cnt"] == len(code) // 8
    assert got["6"] == {"type": "bpf_link_handler", "attr": {"prog_fd": 5, "target_fd": 2}}


def test_single_handler_and_errors(clean):
    l = clean
    code = programs.kat_mul()
    h = {"type": "bpf_prog_handler", "name": "mul", "attr": {"type": 5, "insns": code.hex(), "cnt": len(code) // 8}}
    assert l.bpftime_import_shm_handler_from_json(9, json.dumps(h).encode()) == 0
    assert l.bpftime_is_prog_fd(9)
    bad = dict(h, attr=dict(h["attr"], cnt=len(code) // 8 + 1))          # hex length != cnt * 8
    assert l.bpftime_import_shm_handler_from_json(10, json.dumps(bad).encode()) < 0
    assert l.bpftime_import_shm_handler_from_json(11, b"{\"type\": ") < 0
    perf = {"type": "bpf_perf_event_handler", "attr": {"type": 6, "pid": 1}, "enabled": True}
    assert l.bpftime_import_shm_handler_from_json(12, json.dumps(perf).encode()) < 0
    link = {"type": "bpf_link_handler", "attr": {"prog_fd": 77, "target_fd": 1}}
    assert l.bpftime_import_shm_handler_from_json(13, json.dumps(link).encode()) < 0


@pytest.mark.gpu
def test_reference_state_runs_on_device(fresh_oracle, fresh_runtime, tmp_path):
    po, dev = fresh_oracle, fresh_runtime
    l = _lib.lib()
    code, state = reference_state()
    p = tmp_path / "state.json"
    p.write_text(json.dumps(state, indent=4))
    assert l.bpftime_import_global_shm_from_json(str(p).encode()) == 0, l.bpftime_amd_last_error()
    links = (C_int * 4)()
    progs = (C_int * 4)()
    ifx = (C_u32 * 4)()
    assert l.bpftime_amd_xdp_links(links, progs, ifx, 4) == 1
    vm = dev.prog_instantiate(progs[0])
    octl = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, fd=3)
    obss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, fd=4)
    n = 1 << 15
    pk = gen.xdp_packets(n)
    d = dev.DeviceBuffer.from_array(pk)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv) == 0
    ovm = po.OracleVM()
    ovm.load(code)
    opk = pk.copy()
    ov = ovm.run_xdp(opk, fixed_len=64)
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(d.download().reshape(n, 64), opk)
    assert dev.Map.from_fd(4).lookup(b"\0\0\0\0") == obss.lookup(b"\0\0\0\0")
    assert struct.unpack_from("<Q", obss.lookup(b"\0\0\0\0"))[0] == n
