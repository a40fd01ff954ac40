"""Golden fixtures for BASELINE.json configs[0] (xdp-counter over the 1k
pcap): the oracle on CPU, and the device through the C ABI (gpu)."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from bpftime_amd import gen, isa, programs

from _helpers import xdp_counter_maps

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PCAP = os.path.join(HERE, "xdp_counter_1k.pcap")
EXPECTED = json.load(open(os.path.join(HERE, "xdp_counter_1k.expected.json")))


def _digest(frames):
    h = hashlib.sha256()
    for o in frames:
        h.update(struct.pack("<I", len(o)) + o)
    return h.hexdigest()


def test_pcap_fixture_is_the_seeded_input():
    assert hashlib.sha256(open(PCAP, "rb").read()).hexdigest() == EXPECTED["input_pcap_sha256"]
    assert gen.read_pcap(PCAP) == gen.config1_frames()


@pytest.mark.parametrize("flag", [0, 1])
def test_oracle_matches_golden(fresh_oracle, flag):
    po = fresh_oracle
    frames = gen.read_pcap(PCAP)
    (octl, obss), _ = xdp_counter_maps(po, None, ctl_flag=flag)
    vm = po.OracleVM()
    vm.load(programs.xdp_counter(octl.fd, obss.fd))
    slots, lens = gen.frames_to_slots(frames, stride=128)
    v = vm.run_xdp(slots, lens=lens)
    exp = EXPECTED["runs"][f"ctl_flag_{flag}"]
    assert [int(x) for x in v] == exp["verdicts"]
    assert _digest([bytes(slots[i, :lens[i]]) for i in range(len(frames))]) == exp["output_frames_sha256"]
    assert np.frombuffer(obss.lookup(b"\0\0\0\0"), np.uint64)[0] == exp["cntrs_array_0"]


@pytest.mark.gpu
@pytest.mark.parametrize("flag", [0, 1])
def test_device_matches_golden(fresh_runtime, flag):
    dev = fresh_runtime
    frames = gen.read_pcap(PCAP)
    _, (dctl, dbss) = xdp_counter_maps(None, dev, ctl_flag=flag)
    vm = dev.VM()
    vm.load(programs.xdp_counter(dctl.fd, dbss.fd))
    slots, lens = gen.frames_to_slots(frames, stride=128)
    d = dev.DeviceBuffer.from_array(slots)
    dl = dev.DeviceBuffer.from_array(lens)
    dv = dev.DeviceBuffer(4 * len(frames))
    assert vm.exec_batch(dev.CTX_XDP, d, len(frames), 128, lens=dl, verdicts=dv) == 0
    v = dv.download(np.uint32)
    out = d.download().reshape(len(frames), 128)
    exp = EXPECTED["runs"][f"ctl_flag_{flag}"]
    assert [int(x) for x in v] == exp["verdicts"]
    assert _digest([bytes(out[i, :lens[i]]) for i in range(len(frames))]) == exp["output_frames_sha256"]
    assert np.frombuffer(dbss.lookup(b"\0\0\0\0"), np.uint64)[0] == exp["cntrs_array_0"]
    assert isa.XDP_TX in v or flag
