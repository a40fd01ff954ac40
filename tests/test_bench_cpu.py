"""The CPU baseline leg (bench_cpu.py): one pinned core and N pinned worker
processes over contiguous shards with private maps, map totals checked."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("workload", ["xdp-counter", "syscall-agg"])
def test_cpu_baseline_legs(workload):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_cpu.py"), "--workload", workload,
                        "--seconds", "0.3", "--cores", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["cores"] == min(2, len(os.sched_getaffinity(0)))
    assert out["value"] > 0 and out["single_core"]["value"] > 0 and out["single_core"]["cores"] == 1
    assert out["kind"] == "port"


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
