"""Debug: program-side LPM writes on the device vs the oracle (first mismatches)."""
import struct
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "tests"))
import numpy as np
from bpftime_amd import vm as dev, isa
from oracle import pyoracle as po
from test_gpu_lpm import learn_prog, learn_units, LPM

dev.lib().bpftime_amd_set_device(0)
for seq in ("tiny", "stream"):
    dev.reset_runtime(); po.reset()
    dm = dev.Map(LPM, 8, 4, 64, fd=3); om = po.OracleMap(LPM, 8, 4, 64, fd=3)
    code = learn_prog(3)
    v = dev.VM(); v.load(code); ov = po.OracleVM(); ov.load(code)
    if seq == "tiny":
        u = np.zeros((4, 16), np.uint8); w = u.view(np.uint32)
        w[:, 0] = [1, 0, 1, 0]; w[:, 1] = [8, 32, 16, 32]
        u[:, 8:12] = [[10, 0, 0, 0], [10, 1, 2, 3], [10, 1, 0, 0], [10, 1, 2, 3]]
        w[:, 3] = [5, 0, 6, 0]
    else:
        u = learn_units(np.random.default_rng(11), 3000)
    want = ov.run_raw(u.copy(), 16)
    d = dev.DeviceBuffer.from_array(u); dr = dev.DeviceBuffer(8 * len(u))
    rc = v.exec_batch(dev.CTX_RAW, d, len(u), 16, fixed_len=16, rets=dr, flags=dev.BATCH_SYNC | dev.BATCH_ORDERED)
    got = dr.download(np.uint64)
    print(seq, "rc", rc, "dev count", dm.count(), "oracle count", om.count())
    bad = np.nonzero(got != want)[0]
    print(seq, "mismatches", len(bad))
    for i in bad[:8]:
        print("  unit", i, u[i].view(np.uint32).tolist(), bytes(u[i, 8:12]).hex(), "dev", int(got[i]), "oracle", int(want[i]))
    if seq == "tiny":
        print("  got", got.tolist(), "want", want.tolist())
