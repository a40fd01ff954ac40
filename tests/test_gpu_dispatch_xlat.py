"""Direct dispatch of the asm tier (gen_fast.py): linked FInsns name their
handlers by offset from the asm's handler base, which the host learns from
one query launch per asm variant (vm_api.cpp fast_xlat).  Those offsets are
assembly-time constants of the asm text, so every kernel instance that runs
one variant must report the same table; this checks it over every instance a
launch can select."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CTX_RAW, CTX_XDP, CTX_SYSCALL = 0, 1, 2


def _xlat(dev, kind, big_stack, greg, image, count):
    L = dev.lib()
    f = L.bpftime_amd_launch_fast_xlat
    f.restype = C.c_int
    f.argtypes = [C.c_uint32, C.c_bool, C.c_bool, C.c_bool, C.c_void_p, C.c_void_p]
    buf = dev.DeviceBuffer(4 * count)
    assert f(kind, big_stack, greg, image, buf.ptr, None) == 0
    L.bpftime_amd_sync()
    return buf.download(np.uint32, count=count)


def _count():
    import os
    src = os.path.join(os.path.dirname(__file__), "..", "bpftime_amd", "csrc", "fast_ops.hpp")
    for line in open(src):
        if "F_COUNT" in line and "=" in line:
            return int(line.split("=")[1].strip().rstrip(","))
    raise AssertionError("F_COUNT not found")


def test_handler_offsets_agree_across_instances(fresh_runtime):
    dev = fresh_runtime
    n = _count()
    ref = {g: _xlat(dev, CTX_RAW, False, g, False, n) for g in (False, True)}
    for g in (False, True):
        t = ref[g]
        assert t[0] == 0 and (np.diff(t.astype(np.int64)) > 0).all(), "handler offsets must rise in id order"
        assert (t % 64 == 0).all(), "every divergent stub starts a 64-B aligned handler slot"
    for kind in (CTX_RAW, CTX_XDP, CTX_SYSCALL):
        for g in (False, True):
            for image in (False, True):
                got = _xlat(dev, kind, False, g, image, n)
                assert (got == ref[g]).all(), (kind, g, image)
        got = _xlat(dev, kind, True, False, False, n)  # BIGSTACK instances run the LDS-copy variant
        assert (got == ref[False]).all(), (kind, "big stack")
