"""AF_XDP-umem descriptor batches: frames scattered in
a umem of 2048-B chunks, addressed by struct xdp_desc {addr, len}, in ring
order; checked against the oracle run over the same frames gathered into
slots.  Covers aligned frames (staged fast path), misaligned ones (waves
without staging) and descriptors outside the umem (unit fails, verdict 0)."""
import numpy as np
import pytest

from bpftime_amd import gen, isa, programs

from _helpers import make_maps

pytestmark = pytest.mark.gpu

CHUNK = 2048


def _umem(n, rng, misaligned_every=0):
    nchunks = n + 64
    umem = np.zeros(nchunks * CHUNK, np.uint8)
    chunks = rng.permutation(nchunks)[:n]
    heads = np.full(n, 256, np.uint64)                    # XDP_PACKET_HEADROOM
    if misaligned_every:
        heads[::misaligned_every] += 6
    addrs = chunks.astype(np.uint64) * CHUNK + heads
    slots, lens = gen.flow_packets(n, nflows=500, stride=CHUNK)
    for i in range(n):
        a = int(addrs[i])
        umem[a:a + lens[i]] = slots[i, :lens[i]]
    descs = np.zeros((n, 2), np.uint64)
    descs[:, 0] = addrs
    descs[:, 1] = lens
    return umem, descs, slots, lens


@pytest.mark.parametrize("misaligned_every", [0, 7])
def test_flow_hash_descriptor_batch(fresh_oracle, fresh_runtime, misaligned_every):
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(11)
    n = 6000
    umem, descs, slots, lens = _umem(n, rng, misaligned_every)
    bad = [5, 4000]                                        # outside the umem
    descs[bad[0], 0] = umem.size - 10
    descs[bad[1], 0] = umem.size + 4096
    (om,), (dm,) = make_maps([(isa.BPF_MAP_TYPE_HASH, 16, 16, 4096)], po, dev)
    code = programs.flow_hash(dm.fd)
    ovm = po.OracleVM()
    ovm.load(code)
    keep = np.ones(n, bool)
    keep[bad] = False
    want = np.zeros(n, np.uint32)
    want[keep] = ovm.run_xdp(slots[keep].copy(), lens=lens[keep])
    vm = dev.VM()
    vm.load(code)
    du = dev.DeviceBuffer.from_array(umem)
    dd = dev.DeviceBuffer.from_array(descs)
    dv = dev.DeviceBuffer(4 * n)
    failed = vm.exec_batch(dev.CTX_XDP, du, n, CHUNK, verdicts=dv, descs=dd, umem_bytes=umem.size)
    assert failed == len(bad)
    np.testing.assert_array_equal(dv.download(np.uint32), want)
    assert dm.hash_items() == om.items()


def test_xdp_counter_descriptor_batch_rewrites_frames(fresh_oracle, fresh_runtime):
    """The MAC swap lands in the frames inside the umem, nowhere else."""
    po, dev = fresh_oracle, fresh_runtime
    rng = np.random.default_rng(3)
    n = 4096
    umem, descs, _, _ = _umem(n, rng)
    descs[:, 1] = 64
    (octl, obss), (dctl, dbss) = make_maps([(isa.BPF_MAP_TYPE_ARRAY, 4, 4, 2),
                                            (isa.BPF_MAP_TYPE_ARRAY, 4, 4096, 1)], po, dev)
    code = programs.xdp_counter(dctl.fd, dbss.fd)
    frames = np.stack([umem[int(a):int(a) + 64] for a in descs[:, 0]])
    ovm = po.OracleVM()
    ovm.load(code)
    ov = ovm.run_xdp(frames, fixed_len=64)
    want = umem.copy()
    for i, a in enumerate(descs[:, 0]):
        want[int(a):int(a) + 64] = frames[i]
    vm = dev.VM()
    vm.load(code)
    du = dev.DeviceBuffer.from_array(umem)
    dd = dev.DeviceBuffer.from_array(descs)
    dv = dev.DeviceBuffer(4 * n)
    assert vm.exec_batch(dev.CTX_XDP, du, n, CHUNK, verdicts=dv, descs=dd, umem_bytes=umem.size) == 0
    np.testing.assert_array_equal(dv.download(np.uint32), ov)
    np.testing.assert_array_equal(du.download(), want)
    assert dbss.lookup(b"\0\0\0\0") == obss.lookup(b"\0\0\0\0")
