"""The bpftime VM plugin (bpftime_amd/plugin/compat_mi355x.hpp) driven the way
bpftime_prog drives a bpftime_vm_impl (runtime/src/bpftime_prog.cpp:106-127,
231-260), with libbpftime_amd reached only through dlopen (tests/cpp/
vm_plugin_test.cpp): the runtime's maps are mirrored into the device registry
on load (contents included), the device's lddw helpers replace the host ones,
and the counter comes back through sync_maps_to_host()."""
import json
import os
import subprocess

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bpftime_amd", "lib", "vm_plugin_test")
LIB = os.path.join(ROOT, "bpftime_amd", "lib", "libbpftime_amd.so")
ENV = dict(os.environ, BPFTIME_AMD_LIB=LIB)


def test_plugin_binds_every_symbol_through_dlopen():
    out = subprocess.run([BIN, "--symbols"], env=ENV, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "OK symbols"


@pytest.mark.gpu
def test_plugin_runs_xdp_counter_with_mirrored_maps(tmp_path, fresh_oracle):
    po = fresh_oracle
    ctl_fd, bss_fd, n = 5, 6, 3000
    code = programs.xdp_counter(ctl_fd, bss_fd)
    pk = gen.xdp_packets(n, seed=41)
    (tmp_path / "prog").write_bytes(code)
    (tmp_path / "pkts").write_bytes(pk.tobytes())
    out = subprocess.run([BIN, "--run", str(tmp_path / "prog"), str(tmp_path / "pkts"), str(n), str(ctl_fd),
                          str(bss_fd), str(tmp_path / "o")], env=ENV, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout.strip())
    # the oracle, with the runtime's starting .bss
    po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2, fd=ctl_fd)
    obss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1, fd=bss_fd)
    start = np.zeros(512, np.uint64)
    start[0] = 1000
    obss.update(b"\0\0\0\0", start.tobytes())
    ovm = po.OracleVM()
    ovm.load(code)
    opk = pk.copy()
    ov = ovm.run_xdp(opk, fixed_len=64, ifindex=5)
    np.testing.assert_array_equal(np.fromfile(tmp_path / "o.verdicts", np.uint32), ov)
    np.testing.assert_array_equal(np.fromfile(tmp_path / "o.frames", np.uint8).reshape(n, 64), opk)
    assert res["mirrored"] == 2
    assert res["counter"] == int(np.frombuffer(obss.lookup(b"\0\0\0\0"), np.uint64)[0]) == 1000 + n
