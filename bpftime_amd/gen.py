"""Seeded synthetic inputs.  Counter-based splitmix64: word k of
a stream is ``sm64(seed, k)``, so a shard at any offset regenerates the same
bytes on host (numpy, here) and device (csrc/gen.hip)."""
from __future__ import annotations

import struct
from typing import Tuple

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

SEED_CFG1 = 1
SEED_CFG2 = 0x5EED0002
SEED_CFG3 = 0x5EED0003
SEED_CFG4 = 0x5EED0004
SEED_CFG5 = 0x5EED0005


def sm64(seed: int, k: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (k.astype(np.uint64) + np.uint64(1)) * GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def xdp_packets(n: int, stride: int = 64, seed: int = SEED_CFG2, first: int = 0) -> np.ndarray:
    """n slots of `stride` random bytes, ethertype 0x0800 (csrc/gen.hip k_gen_xdp)."""
    w = stride // 8
    k = np.arange(first * w, (first + n) * w, dtype=np.uint64)
    words = sm64(seed, k).reshape(n, w)
    words[:, 1] = (words[:, 1] & np.uint64(~0x0000FFFF00000000 & 0xFFFFFFFFFFFFFFFF)) | np.uint64(0x0008 << 32)
    return words.view(np.uint8).reshape(n, stride)


def _uniform(seed: int, k: np.ndarray) -> np.ndarray:
    return (sm64(seed, k) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def zipf_cdf(support: int, s: float) -> np.ndarray:
    """CDF table of the bounded Zipf(s) law (also uploaded for csrc/gen.hip)."""
    w = 1.0 / np.arange(1, support + 1, dtype=np.float64) ** s
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return cdf


def zipf_ids(seed: int, first: int, n: int, support: int, s: float) -> np.ndarray:
    """Bounded Zipf(s) ids in [0, support) by inverse CDF of a uniform stream."""
    cdf = zipf_cdf(support, s)
    u = _uniform(seed, np.arange(first, first + n, dtype=np.uint64))
    return np.minimum(np.searchsorted(cdf, u, side="right"), support - 1).astype(np.int64)


def flow_packets(n: int, seed: int = SEED_CFG3, nflows: int = 65536, stride: int = 2048,
                 first: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """config 3: frames of 64/570/1500 B (7:4:1) in `stride`-byte slots;
    95 % IPv4 (TCP:UDP 1:1, ihl 5), 5 % other ethertype; flows Zipf(1.1)."""
    idx = np.arange(first, first + n, dtype=np.uint64)
    r = sm64(seed ^ 0x1111, idx)
    size_sel = (r % np.uint64(12)).astype(np.int64)
    lens = np.where(size_sel < 7, 64, np.where(size_sel < 11, 570, 1500)).astype(np.uint32)
    is_ip = ((r >> np.uint64(8)) % np.uint64(100)) < np.uint64(95)
    flow = zipf_ids(seed, first, n, nflows, 1.1)
    fk = sm64(seed ^ 0x2222, flow.astype(np.uint64))
    saddr = (fk & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    daddr = (fk >> np.uint64(32)).astype(np.uint32)
    fk2 = sm64(seed ^ 0x3333, flow.astype(np.uint64))
    ports = (fk2 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    proto = np.where((fk2 >> np.uint64(40)) & np.uint64(1), 6, 17).astype(np.uint8)
    # fill slot bytes with noise, then write headers
    w = stride // 8
    body = sm64(seed ^ 0x4444, np.arange(first * w, (first + n) * w, dtype=np.uint64)).view(np.uint8)
    slots = body.reshape(n, stride).copy()
    slots[:, 12] = np.where(is_ip, 0x08, 0x86)
    slots[:, 13] = np.where(is_ip, 0x00, 0xDD)
    slots[:, 14] = 0x45
    slots[:, 23] = proto
    slots[:, 26:30] = saddr.view(np.uint8).reshape(n, 4)
    slots[:, 30:34] = daddr.view(np.uint8).reshape(n, 4)
    slots[:, 34:38] = ports.view(np.uint8).reshape(n, 4)
    return slots, lens


def syscall_records(n: int, seed: int = SEED_CFG5, first: int = 0) -> np.ndarray:
    """config 5: 64-B trace_event_raw_sys_enter records (ent zeroed), id
    Zipf(1.2) over 0..334 plus 1 % exit(60)/exit_group(231)."""
    idx = np.arange(first, first + n, dtype=np.uint64)
    ids = zipf_ids(seed, first, n, 335, 1.2)
    r = sm64(seed ^ 0x5555, idx)
    special = (r % np.uint64(100)) == np.uint64(0)
    ids = np.where(special, np.where((r >> np.uint64(9)) & np.uint64(1), 60, 231), ids)
    recs = np.zeros((n, 8), dtype=np.uint64)
    recs[:, 1] = ids.astype(np.uint64)
    for j in range(6):
        recs[:, 2 + j] = sm64(seed ^ (0x6000 + j), idx) & np.uint64(0xFFFFFFFFFF)
    return recs.view(np.uint8).reshape(n, 64)


def syscall_records_full(n: int, seed: int = SEED_CFG5, first: int = 0) -> np.ndarray:
    """96-B replay records (include/bpftime_amd.h BPFTIME_AMD_SYSCALL_RECORD_FULL):
    the config 5 enter record (id -1 instead for 0.5 %: the tracepoint's
    interrupt marker), then trace_event_raw_sys_exit {ent 0, id, ret} with
    ret a negative errno in [-133, -1] for 20 % of the records, else in
    [0, 65535], then the caller's pid_tgid (tgid 1000 + [0, 64) << 32 | tid
    tgid + [0, 4))."""
    idx = np.arange(first, first + n, dtype=np.uint64)
    enter = syscall_records(n, seed, first).view(np.uint64).reshape(n, 8).copy()
    r = sm64(seed ^ 0x5555, idx)
    ids = np.where((r % np.uint64(200)) == np.uint64(1), np.uint64(0xFFFFFFFFFFFFFFFF), enter[:, 1])
    enter[:, 1] = ids
    rr = sm64(seed ^ 0x7777, idx)
    neg = (np.uint64(0) - (np.uint64(1) + (rr >> np.uint64(8)) % np.uint64(133)))
    ret = np.where((rr % np.uint64(5)) == np.uint64(0), neg, (rr >> np.uint64(16)) & np.uint64(0xFFFF))
    recs = np.zeros((n, 12), dtype=np.uint64)
    recs[:, :8] = enter
    recs[:, 9] = ids
    recs[:, 10] = ret
    rp = sm64(seed ^ 0x8888, idx)
    tgid = np.uint64(1000) + rp % np.uint64(64)
    recs[:, 11] = (tgid << np.uint64(32)) | (tgid + (rp >> np.uint64(8)) % np.uint64(4))
    return recs.view(np.uint8).reshape(n, 96)


def syscall_records_timed(n: int, seed: int = SEED_CFG5, first: int = 0, threads: int = 64) -> np.ndarray:
    """128-B replay records (include/bpftime_amd.h BPFTIME_AMD_SYSCALL_RECORD_TIMED):
    the 96-B records of :func:`syscall_records_full` with the caller drawn
    from ``threads`` threads (thread t: tgid 1000 + t // 4, tid 2000 + t,
    tids unique as a kernel's are), then the clock at sys_enter (1 s + 1 us
    per record index + [0, 500) ns: monotonic within a thread) and after the
    call (enter + [50, 100050) ns), then 16 zero bytes."""
    idx = np.arange(first, first + n, dtype=np.uint64)
    full = syscall_records_full(n, seed, first).view(np.uint64).reshape(n, 12)
    recs = np.zeros((n, 16), dtype=np.uint64)
    recs[:, :12] = full
    t = sm64(seed ^ 0x9999, idx) % np.uint64(threads)
    recs[:, 11] = ((np.uint64(1000) + t // np.uint64(4)) << np.uint64(32)) | (np.uint64(2000) + t)
    rc = sm64(seed ^ 0xAAAA, idx)
    recs[:, 12] = np.uint64(1_000_000_000) + idx * np.uint64(1000) + rc % np.uint64(500)
    recs[:, 13] = recs[:, 12] + np.uint64(50) + (rc >> np.uint64(16)) % np.uint64(100000)
    return recs.view(np.uint8).reshape(n, 128)


def syscall_records_soa(recs: np.ndarray):
    """The struct-of-arrays form of 96- / 128-B replay records (include/
    bpftime_amd.h struct bpftime_amd_sys_records): (enter n x 64 B, exit n x
    32 B {exit ctx, pid_tgid}, clock n x 16 B or None)."""
    n, rs = recs.shape
    enter = np.ascontiguousarray(recs[:, :64])
    exit_ = np.ascontiguousarray(recs[:, 64:96])
    clock = np.ascontiguousarray(recs[:, 96:112]) if rs == 128 else None
    return enter, exit_, clock


# ---------------------------------------------------------------------------
# config 1: 1k-packet pcap (990 x 64 B Eth/IPv4/UDP + 10 runts, seed 1)
# ---------------------------------------------------------------------------
def _ipv4_csum(h: bytes) -> int:
    s = sum(struct.unpack("!10H", h))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def config1_frames(seed: int = SEED_CFG1) -> list:
    r = sm64(seed, np.arange(1000 * 8, dtype=np.uint64)).reshape(1000, 8)
    frames = []
    runt_at = set(range(45, 1000, 100))  # 10 runts spread over the capture
    runt_len = iter(range(4, 14))
    for i in range(1000):
        b = r[i].view(np.uint8).tobytes()
        if i in runt_at:
            frames.append(b[: next(runt_len)])
            continue
        dst, src = b[0:6], b[6:12]
        saddr, daddr = b[12:16], b[16:20]
        sport, dport = b[20:22], b[22:24]
        payload = b[24:46].ljust(22, b"\0")
        ip = bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, 0, 50, i & 0xFFFF, 0, 64, 17, 0, saddr, daddr))
        ip[10:12] = struct.pack("!H", _ipv4_csum(bytes(ip)))
        udp = sport + dport + struct.pack("!HH", 30, 0)
        frames.append(dst + src + b"\x08\x00" + bytes(ip) + udp + payload)
    assert sum(len(f) == 64 for f in frames) == 990
    return frames


def write_pcap(path: str, frames: list) -> None:
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))  # LINKTYPE_ETHERNET
        for i, fr in enumerate(frames):
            f.write(struct.pack("<IIII", 1700000000 + i // 1000, (i % 1000) * 1000, len(fr), len(fr)))
            f.write(fr)


def read_pcap(path: str) -> list:
    with open(path, "rb") as f:
        data = f.read()
    magic = struct.unpack_from("<I", data, 0)[0]
    if magic != 0xA1B2C3D4:
        raise ValueError("not a little-endian classic pcap")
    off, frames = 24, []
    while off < len(data):
        _, _, incl, _ = struct.unpack_from("<IIII", data, off)
        off += 16
        frames.append(data[off:off + incl])
        off += incl
    return frames


def frames_to_slots(frames: list, stride: int = 2048) -> Tuple[np.ndarray, np.ndarray]:
    slots = np.zeros((len(frames), stride), dtype=np.uint8)
    lens = np.zeros(len(frames), dtype=np.uint32)
    for i, fr in enumerate(frames):
        slots[i, :len(fr)] = np.frombuffer(fr, dtype=np.uint8)
        lens[i] = len(fr)
    return slots, lens
