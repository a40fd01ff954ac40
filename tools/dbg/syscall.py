"""Debug: instrumented syscall_agg on the device (lookup/update/re-lookup outcomes)."""
import sys, os, struct
sys.path.insert(0, os.getcwd())
import numpy as np
from bpftime_amd import gen, isa
from bpftime_amd import vm as dev
from bpftime_amd.isa import Asm


def prog(fd):
    a = Asm()
    a.ldx(8, 6, 1, 8).stx(4, 10, -4, "r6")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(1)
    a.mov64(9, 1)
    a.jmp("jne", 0, 0, "have")
    for o in (-40, -32, -24, -16):
        a.st(8, 10, o, 0)
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).mov64(3, "r10").add64(3, -40).mov64(4, isa.BPF_NOEXIST).call(2)
    a.mov64(8, "r0")
    a.ld_map_fd(1, fd).mov64(2, "r10").add64(2, -4).call(1)
    a.mov64(9, 2)
    a.jmp("jne", 0, 0, "have")
    a.mov64(0, "r8").alu64("and", 0, 0xff).add64(0, 1000).exit()
    a.label("have")
    a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, "r1")
    a.mov64(0, "r9").exit()
    return a.assemble()


def run(ordered, n):
    dev.reset_runtime()
    m = dev.Map(isa.BPF_MAP_TYPE_HASH, 4, 32, 8192)
    vm = dev.VM(); vm.load(prog(m.fd))
    recs = gen.syscall_records(n)
    d = dev.DeviceBuffer.from_array(recs); dr = dev.DeviceBuffer(8 * n)
    fl = dev.BATCH_SYNC | (dev.BATCH_ORDERED if ordered else 0)
    f = vm.exec_batch(dev.CTX_SYSCALL, d, n, 64, rets=dr, flags=fl)
    r = dr.download(np.uint64)
    ids = recs.view(np.uint64).reshape(n, 8)[:, 1]
    u, c = np.unique(r, return_counts=True)
    items = m.hash_items()
    cnt = {struct.unpack("<I", k)[0]: struct.unpack("<Q", v[:8])[0] for k, v in items.items()}
    live = ids[(ids != 60) & (ids != 231)]
    exp_ids, exp_c = np.unique(live, return_counts=True)
    exp = dict(zip(exp_ids.tolist(), exp_c.tolist()))
    missing = [k for k in exp if k not in cnt]
    diff = {k: (cnt.get(k), exp[k]) for k in exp if cnt.get(k) != exp[k]}
    print(f"ordered={ordered} n={n} failed={f} rets={dict(zip(u.tolist(), c.tolist()))} keys={len(cnt)}/{len(exp)} "
          f"count()={m.count()} missing={missing[:8]} ndiff={len(diff)} diff={list(diff.items())[:6]}", flush=True)
    if missing:
        bad = np.nonzero(r >= 1000)[0]
        print("  failing units:", bad[:10].tolist(), "ids:", ids[bad[:10]].tolist(), flush=True)


for n in (2000, 60000):
    for ordered in (True, False):
        run(ordered, n)
