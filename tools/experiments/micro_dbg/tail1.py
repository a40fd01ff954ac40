"""Tail-call parity per first-byte index at n=1 (debug)."""
import os, struct, sys
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bpftime_amd import vm as dev, isa, gen
from bpftime_amd import programs
import _tailcall as tc
from oracle import pyoracle as po
I32 = lambda v: struct.pack("<i", v)
PA = 20
for idx in range(4):
    po.reset(); dev.reset_runtime(); dev.set_ncpu(64)
    pa_o = po.OracleMap(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA)
    pa_d = dev.Map(isa.BPF_MAP_TYPE_PROG_ARRAY, 4, 4, 4, fd=PA)
    cnt_d = dev.Map(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4)
    cnt_o = po.OracleMap(isa.BPF_MAP_TYPE_ARRAY, 4, 8, 4, fd=cnt_d.fd)
    progs = {900: tc.target_write(0xA1), 901: tc.target_count(cnt_d.fd), 903: tc.target_recurse(PA, cnt_d.fd, 3)}
    for fd, code in progs.items():
        po.prog_create(fd, code); dev.prog_create(code, f"t{fd}", 6, fd=fd)
    for k, fd in ((0, 900), (1, 901), (3, 903)):
        pa_o.update(I32(k), I32(fd)); pa_d.update(I32(k), I32(fd))
    code = tc.xdp_caller(PA, cnt_d.fd)
    ovm = po.OracleVM(); ovm.load(code)
    dvm = dev.VM(); dvm.load(code)
    n = 64
    pk = gen.xdp_packets(n, seed=3); pk[:, 0] = idx
    opk = pk.copy(); ov = ovm.run_xdp(opk, fixed_len=64, ifindex=5)
    d = dev.DeviceBuffer.from_array(pk); dv = dev.DeviceBuffer(4 * n)
    rt = dev.DeviceBuffer(8 * n)
    bad = dvm.exec_batch(dev.CTX_XDP, d, n, 64, fixed_len=64, verdicts=dv, rets=rt, ifindex=5)
    r = rt.download(np.uint64)[0]
    print("  ret0 %x err %d pc %d lpc %d" % (r, r & 0xff, (r >> 8) & 0xfffffff, r >> 36))
    got = dv.download(np.uint32)
    print("idx", idx, "failed", bad, "dev", got[:2], "oracle", ov[:2],
          "pkt ok", bool((d.download().reshape(n, 64) == opk).all()),
          "cnt", [cnt_d.lookup(I32(i)) == cnt_o.lookup(I32(i)) for i in range(4)])
