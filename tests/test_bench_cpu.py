"""The CPU baseline leg (bench_cpu.py): one pinned core and N pinned worker
processes over contiguous shards with private maps, map totals checked."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _leg(workload):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_cpu.py"), "--workload", workload,
                        "--seconds", "0.3", "--cores", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("workload", ["xdp-counter", "syscall-agg"])
def test_cpu_baseline_legs(workload):
    out = _leg(workload)
    assert out["ok"] and out["cores"] == min(2, len(os.sched_getaffinity(0)))
    assert out["value"] > 0 and out["single_core"]["value"] > 0 and out["single_core"]["cores"] == 1
    assert out["kind"] == "port"
    # the workers' timed loops run side by side (a common start, one loop
    # each, nothing untimed inside: VERDICT r05 item 6).  Concurrency is a
    # timing: a host busy with other work (a build) can stagger two
    # 0.3-s workers once, so a low reading is measured again before it fails
    n = out["cores_16"]["cores"]
    if out["cores_16"]["concurrency"] < 0.85 * n:
        out = _leg(workload)
    assert out["cores_16"]["concurrency"] >= 0.85 * n, out["cores_16"]


def test_cpu_baseline_ringbuf_leg_wraps():
    """The ring-buffer leg refills one ring run after run; with a 128 KiB ring
    every worker wraps it many times (≈ 98 KB of records per 2^18-frame
    run).  Its check (records fetched per run == frames with byte0 % 64 ==
    0) failed on the GPU box's faster cores before the oracle's
    bpf_ringbuf_output submitted by fd (profiles/r02_bench_lines.jsonl:6)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_cpu.py"), "--workload", "ringbuf-sample",
                        "--seconds", "0.4", "--cores", "2", "--ring-log2", "17"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"], out


def test_union_of_timed_intervals():
    sys.path.insert(0, ROOT)
    import bench_cpu
    assert bench_cpu.union_seconds([]) == 0.0
    assert bench_cpu.union_seconds([(0, 1), (0.5, 2), (3, 4)]) == pytest.approx(3.0)
    assert bench_cpu.union_seconds([(2, 3), (0, 1)]) == pytest.approx(2.0)


def test_serialized_leg_is_not_counted_as_parallel():
    """under the GPU box's CPU quota the workers of a leg did
    not run side by side, and units / the longest single loop made serial
    loops look parallel (2,108 Mpps on 15.6 busy cores).  Two workers whose
    loops never overlap (the second starts after the first ended) must give
    about one worker's rate, with concurrency about 1."""
    sys.path.insert(0, ROOT)
    import bench_cpu
    cores = sorted(os.sched_getaffinity(0))
    c = cores[:2] if len(cores) > 1 else cores * 2
    v1, _, _, ok1, _, conc1 = bench_cpu.leg("xdp-counter", c[:1], 0.5)
    v2, union2, _, ok2, _, conc2 = bench_cpu.leg("xdp-counter", c, 0.5, stagger=3.0)
    assert ok1 and ok2
    assert conc2 < 1.15 and union2 > 0.9
    assert v2 < 1.3 * v1


def test_syscount_leg():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_cpu.py"), "--workload", "syscount",
                        "--seconds", "0.3", "--cores", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["unit"] == "Mrec/s" and out["value"] > 0
    # the chosen leg never claims more per usable CPU than 1.1 x one core
    assert out["value"] / out["cores"] <= 1.1 * out["single_core"]["value"] or out["cores"] == 1
