"""Generates the committed golden fixtures for BASELINE.json configs[0]
(xdp-counter over a 1k-packet pcap through the CPU path).

Inputs are seeded (bpftime_amd/gen.py config1_frames, seed 1); expected
outputs come from the oracle (oracle/, the restated reference CPU path) and
are cross-checked here against the analytic expectations of
example/xdp-counter/xdp-counter.bpf.c:50-70 before
being written.  Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from bpftime_amd import gen, isa, programs  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def run_oracle(frames, ctl_flag):
    po.reset()
    ctl = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2)
    bss = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)
    if ctl_flag:
        ctl.update(struct.pack("<I", 0), struct.pack("<I", ctl_flag))
    vm = po.OracleVM()
    vm.load(programs.xdp_counter(ctl.fd, bss.fd))
    slots, lens = gen.frames_to_slots(frames, stride=128)
    v = vm.run_xdp(slots, lens=lens)
    out = [bytes(slots[i, :lens[i]]) for i in range(len(frames))]
    cnt = np.frombuffer(bss.lookup(b"\0\0\0\0"), dtype=np.uint64)
    return v, out, cnt


def main():
    frames = gen.config1_frames()
    pcap = os.path.join(HERE, "xdp_counter_1k.pcap")
    gen.write_pcap(pcap, frames)
    assert gen.read_pcap(pcap) == frames
    result = {"input_pcap_sha256": hashlib.sha256(open(pcap, "rb").read()).hexdigest(), "runs": {}}
    for flag in (0, 1):
        v, out, cnt = run_oracle(frames, flag)
        # analytic cross-check (xdp-counter.bpf.c:50-70)
        for f, o, vv in zip(frames, out, v):
            if flag:
                assert vv == isa.XDP_PASS and o == f
            elif len(f) < 14:
                assert vv == isa.XDP_DROP and o == f
            else:
                assert vv == isa.XDP_TX and o == f[6:12] + f[0:6] + f[12:]
        assert cnt[0] == (0 if flag else 1000) and not cnt[1:].any()
        h = hashlib.sha256()
        for o in out:
            h.update(struct.pack("<I", len(o)) + o)
        result["runs"][f"ctl_flag_{flag}"] = {
            "verdicts": [int(x) for x in v],
            "output_frames_sha256": h.hexdigest(),
            "cntrs_array_0": int(cnt[0]),
        }
    with open(os.path.join(HERE, "xdp_counter_1k.expected.json"), "w") as f:
        json.dump(result, f, indent=1)
    print("wrote", pcap)


if __name__ == "__main__":
    main()
