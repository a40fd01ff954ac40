"""Debug: device unwind on a lookup miss (tests/test_unwind.py case ARRAY / lookup)."""
import os
import struct
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "tests"))
import numpy as np
from bpftime_amd import vm as dev, isa
from test_unwind import prog, _units

dev.lib().bpftime_amd_set_device(0)
for no_asm in (False, True):
    dev.reset_runtime()
    m = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)
    for k in range(4):
        m.update(struct.pack("<I", k), struct.pack("<Q", 10 * k))
    vm = dev.VM()
    vm.load(prog(m.fd))
    print("set_unwind", vm.set_unwind(12), flush=True)
    u = _units(128)
    d = dev.DeviceBuffer.from_array(u)
    dr = dev.DeviceBuffer(8 * 128)
    flags = dev.BATCH_SYNC | (dev.BATCH_ORDERED if no_asm else 0)
    vm.exec_batch(dev.CTX_RAW, d, 128, 8, fixed_len=8, rets=dr, flags=flags)
    print("ordered" if no_asm else "parallel", dr.download(np.uint64)[:16].tolist(),
          (u.view(np.uint32)[:16, 0] & 7).tolist(), flush=True)
