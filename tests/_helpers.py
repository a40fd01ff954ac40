"""Shared helpers for the parity tests: build the same maps on the oracle
(CPU checker) and on the device, run a program on both, compare."""
import struct

import numpy as np

from bpftime_amd import isa


def make_maps(specs, po=None, dev=None):
    """specs: list of (type, ksize, vsize, max). Creates them at identical fds
    on the oracle and the device registry so the same bytecode loads on both."""
    om, dm = [], []
    for t, k, v, mx in specs:
        d = dev.Map(t, k, v, mx) if dev is not None else None
        fd = d.fd if d is not None else -1
        o = po.OracleMap(t, k, v, mx, fd=fd) if po is not None else None
        om.append(o)
        dm.append(d)
    return om, dm


def xdp_counter_maps(po, dev, ctl_flag=0):
    (octl, obss), (dctl, dbss) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2),
                                            (isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)], po, dev)
    if ctl_flag:
        for m in (octl, dctl):
            if m is not None:
                m.update(struct.pack("<I", 0), struct.pack("<I", ctl_flag))
    return (octl, obss), (dctl, dbss)


def u64s(b):
    return np.frombuffer(b, dtype=np.uint64)
