"""Chained units (gen_fast.py chain_routine, interp.hip chain_ok): with a grid
of 1-3 blocks every lane runs tens to hundreds of units, and the asm tier
starts each wave's next unit itself.  The parity tests of the other files
re-run under BPFTIME_AMD_MAX_GRID against the same oracle, covering XDP /
raw / syscall entry forms, lengths from an array, divergence, failed units
in the middle of a chain, per-CPU counters, hash maps and tail-call images;
BPFTIME_AMD_DBG=64 (chaining off) must give identical results."""
import numpy as np
import pytest

import test_gpu_counters as C
import test_gpu_maps as M
import test_gpu_parity as P
import test_gpu_tailcall as T
from bpftime_amd.isa import Asm

pytestmark = pytest.mark.gpu
GRIDS = ["1", "3"]


@pytest.fixture(params=GRIDS)
def small_grid(request, monkeypatch):
    monkeypatch.setenv("BPFTIME_AMD_MAX_GRID", request.param)
    return int(request.param)


def test_xdp_counter(fresh_oracle, fresh_runtime, small_grid):
    P.test_xdp_counter_parity(fresh_oracle, fresh_runtime, 100003)


@pytest.mark.parametrize("asm_groups", [True, False])
def test_random_raw_programs(fresh_oracle, fresh_runtime, monkeypatch, small_grid, asm_groups):
    P.test_random_programs(fresh_oracle, fresh_runtime, monkeypatch, asm_groups)


def test_random_xdp_programs(fresh_oracle, fresh_runtime, monkeypatch, small_grid):
    P.test_random_xdp_programs(fresh_oracle, fresh_runtime, monkeypatch, True)


def test_divergent_loops(fresh_oracle, fresh_runtime, small_grid):
    P.test_divergent_loops_sum(fresh_oracle, fresh_runtime)


def test_staged_raw_slots(fresh_oracle, fresh_runtime, small_grid):
    P.test_staged_raw_slot_accesses(fresh_oracle, fresh_runtime)


def test_flow_hash_with_lengths(fresh_oracle, fresh_runtime, small_grid):
    M.test_flow_hash_parity(fresh_oracle, fresh_runtime, 50000, 4000)


def test_syscall_records(fresh_oracle, fresh_runtime, small_grid):
    M.test_syscall_agg_parity(fresh_oracle, fresh_runtime)


def test_percpu_counters(fresh_oracle, fresh_runtime, small_grid):
    M.test_percpu_array_counter(fresh_oracle, fresh_runtime)


def test_sampler(fresh_oracle, fresh_runtime, small_grid):
    C.test_sampler_every_64(fresh_oracle, fresh_runtime, 6401)


def test_tailcall_image(fresh_oracle, fresh_runtime, small_grid):
    T.test_xdp_tailcall_parity(fresh_oracle, fresh_runtime, 70000)


def test_failed_units_inside_a_chain(fresh_runtime, small_grid):
    """Units that fail (wild load) between units that exit in the asm tier:
    each failed unit reports 0 and counts once, the rest are exact."""
    dev = fresh_runtime
    a = Asm().ldx(8, 2, 1, 0).jmp("jne", 2, 7, "ok").lddw(3, 0x1000).ldx(8, 0, 3, 0).exit()
    a.label("ok").mov64(0, "r2").add64(0, 1).exit()
    vm = dev.VM()
    vm.load(a.assemble())
    n = 40000
    rng = np.random.default_rng(small_grid)
    vals = rng.integers(0, 50, n).astype(np.uint64)
    vals[rng.random(n) < 0.01] = 7                     # ~1% of units fail
    d = dev.DeviceBuffer.from_array(vals.view(np.uint8).reshape(n, 8))
    dr = dev.DeviceBuffer(8 * n)
    failed = vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr)
    r = dr.download(np.uint64)
    bad = vals == 7
    assert failed == int(bad.sum())
    assert (r[bad] == 0).all() and (r[~bad] == vals[~bad] + 1).all()


def test_chaining_off_is_identical(fresh_oracle, fresh_runtime, monkeypatch, small_grid):
    monkeypatch.setenv("BPFTIME_AMD_DBG", "64")
    P.test_xdp_counter_parity(fresh_oracle, fresh_runtime, 100003)


def test_step_limit_per_chained_unit(fresh_runtime, small_grid):
    """The step count restarts with every chained unit: a loop of 100 taken
    jumps per unit passes a limit of 150 in every unit."""
    dev = fresh_runtime
    a = Asm().mov64(0, 0).label("top").add64(0, 1).jmp("jlt", 0, 100, "top").exit()
    vm = dev.VM()
    vm.load(a.assemble())
    vm.set_step_limit(150)
    n = 20000
    d = dev.DeviceBuffer(8 * n)
    dr = dev.DeviceBuffer(8 * n)
    failed = vm.exec_batch(dev.CTX_RAW, d, n, 8, fixed_len=8, rets=dr)
    assert failed == 0
    assert (dr.download(np.uint64) == 100).all()
