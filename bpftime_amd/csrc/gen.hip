// bpftime_amd: seeded synthetic batch generators, written
// as counter-based splitmix64 so host (bpftime_amd/gen.py) and device agree
// word for word at any shard offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpftime_amd {

__host__ __device__ __forceinline__ uint64_t sm64(uint64_t seed, uint64_t k) {
  uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Unit i fills its whole slot with words sm64(seed, (first+i)*W + j),
// W = stride/8, then writes ethertype 0x0800 at bytes 12..13.
__global__ void k_gen_xdp(uint8_t *base, uint64_t n, uint64_t stride, uint64_t seed, uint64_t first) {
  const uint64_t W = stride / 8;
  const uint64_t total = n * W;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total;
       w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t unit = w / W, j = w % W;
    uint64_t v = sm64(seed, (first + unit) * W + j);
    if (j == 1) v = (v & ~0x0000ffff00000000ull) | (0x0008ull << 32);  // bytes 12,13 = 08 00
    *(uint64_t *)(base + unit * stride + j * 8) = v;
  }
}

// Bounded Zipf id by inverse CDF (gen.py zipf_ids): the first index whose
// cdf entry exceeds u (numpy searchsorted side="right"), clamped.
__device__ __forceinline__ uint32_t zipf_pick(const double *cdf, uint32_t support, uint64_t seed, uint64_t g) {
  const double u = (double)(sm64(seed, g) >> 11) * (1.0 / 9007199254740992.0);
  uint32_t lo = 0, hi = support;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cdf[mid] <= u) lo = mid + 1;
    else hi = mid;
  }
  return lo < support ? lo : support - 1;
}

// config 3 frames (gen.py flow_packets): slot noise, then Ethernet/IPv4
// header fields of the unit's Zipf flow; one thread per 8-B word, the
// thread holding word 1 of a slot also writes its length.
__global__ void k_gen_flow(uint8_t *base, uint32_t *lens, uint64_t n, uint64_t stride, uint64_t seed,
                           uint64_t first, const double *cdf, uint32_t nflows) {
  const uint64_t W = stride / 8;
  const uint64_t total = n * W;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total;
       w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t unit = w / W, j = w % W, g = first + unit;
    uint64_t v = sm64(seed ^ 0x4444, g * W + j);
    if (j >= 1 && j <= 4) {
      const uint64_t r = sm64(seed ^ 0x1111, g);
      const bool is_ip = ((r >> 8) % 100) < 95;
      const uint64_t flow = zipf_pick(cdf, nflows, seed, g);
      const uint64_t fk = sm64(seed ^ 0x2222, flow), fk2 = sm64(seed ^ 0x3333, flow);
      uint8_t *b = (uint8_t *)&v;
      const uint64_t o = j * 8;  // byte offset of this word in the slot
      auto put = [&](uint64_t at, uint8_t x) {
        if (at >= o && at < o + 8) b[at - o] = x;
      };
      put(12, is_ip ? 0x08 : 0x86);
      put(13, is_ip ? 0x00 : 0xDD);
      put(14, 0x45);
      put(23, ((fk2 >> 40) & 1) ? 6 : 17);
      for (int k = 0; k < 4; k++) {
        put(26 + k, (uint8_t)(fk >> (8 * k)));
        put(30 + k, (uint8_t)(fk >> (32 + 8 * k)));
        put(34 + k, (uint8_t)(fk2 >> (8 * k)));
      }
      if (j == 1 && lens) {
        const uint64_t sel = r % 12;
        lens[unit] = sel < 7 ? 64 : sel < 11 ? 570 : 1500;
      }
    }
    *(uint64_t *)(base + unit * stride + j * 8) = v;
  }
}

// config 5 records (gen.py syscall_records): 64-B trace_event_raw_sys_enter,
// id Zipf over [0, support) with 1 % exit(60) / exit_group(231).
__global__ void k_gen_syscall(uint8_t *base, uint64_t n, uint64_t seed, uint64_t first, const double *cdf,
                              uint32_t support) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n * 8;
       w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t unit = w / 8, j = w % 8, g = first + unit;
    uint64_t v = 0;
    if (j == 1) {
      const uint64_t r = sm64(seed ^ 0x5555, g);
      v = (r % 100) == 0 ? (((r >> 9) & 1) ? 60 : 231) : zipf_pick(cdf, support, seed, g);
    } else if (j >= 2) {
      v = sm64(seed ^ (0x6000 + (j - 2)), g) & 0xFFFFFFFFFFull;
    }
    *(uint64_t *)(base + unit * 64 + j * 8) = v;
  }
}

// 96-B replay records (gen.py syscall_records_full): the enter record of
// k_gen_syscall (id -1 instead for 0.5 % of the records, the tracepoint's
// interrupt marker syscount skips), then trace_event_raw_sys_exit {0, id,
// ret}: ret a negative errno in [-133, -1] for 20 % of the records, else in
// [0, 65535]; then the caller's pid_tgid: tgid 1000 + [0, 64), tid tgid + [0, 4)
// Words 0-7 (the enter ctx) go to enter + unit * estride (enter null: not
// written), words 8-11 (exit ctx, pid_tgid) to exit + unit * xstride: the
// 96-B records (enter = base, exit = base + 64, strides 96) or the
// struct-of-arrays form (strides 64 and 32).
__global__ void k_gen_syscall_full(uint8_t *enter, uint64_t estride, uint8_t *exit, uint64_t xstride, uint64_t n,
                                   uint64_t seed, uint64_t first, const double *cdf, uint32_t support) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n * 12;
       w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t unit = w / 12, j = w % 12, g = first + unit;
    uint64_t v = 0;
    if (j == 1 || j == 9) {
      const uint64_t r = sm64(seed ^ 0x5555, g);
      v = (r % 100) == 0 ? (((r >> 9) & 1) ? 60 : 231) : zipf_pick(cdf, support, seed, g);
      if ((r % 200) == 1) v = ~0ull;
    } else if (j >= 2 && j < 8) {
      v = sm64(seed ^ (0x6000 + (j - 2)), g) & 0xFFFFFFFFFFull;
    } else if (j == 10) {
      const uint64_t r = sm64(seed ^ 0x7777, g);
      v = (r % 5) == 0 ? (uint64_t)(-(int64_t)(1 + (r >> 8) % 133)) : (r >> 16) & 0xFFFF;
    } else if (j == 11) {
      const uint64_t r = sm64(seed ^ 0x8888, g), tgid = 1000 + r % 64;
      v = (tgid << 32) | (tgid + (r >> 8) % 4);
    }
    if (j >= 8)
      *(uint64_t *)(exit + unit * xstride + (j - 8) * 8) = v;
    else if (enter)
      *(uint64_t *)(enter + unit * estride + j * 8) = v;
  }
}

}  // namespace bpftime_amd

static uint32_t gen_blocks(uint64_t total) {
  uint64_t blocks = (total + 255) / 256;
  return (uint32_t)(blocks > 16384 ? 16384 : blocks);
}

extern "C" int bpftime_amd_gen_flow(void *dev, uint32_t *lens, uint64_t n, uint64_t stride, uint64_t seed,
                                    uint64_t first, const double *cdf, uint32_t nflows, void *stream) {
  if (stride % 8 || stride < 64 || !cdf || !nflows) return -1;
  if (!n) return 0;
  hipLaunchKernelGGL(bpftime_amd::k_gen_flow, dim3(gen_blocks(n * (stride / 8))), dim3(256), 0,
                     (hipStream_t)stream, (uint8_t *)dev, lens, n, stride, seed, first, cdf, nflows);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int bpftime_amd_gen_syscall(void *dev, uint64_t n, uint64_t seed, uint64_t first, const double *cdf,
                                       uint32_t support, void *stream) {
  if (!cdf || !support) return -1;
  if (!n) return 0;
  hipLaunchKernelGGL(bpftime_amd::k_gen_syscall, dim3(gen_blocks(n * 8)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t *)dev, n, seed, first, cdf, support);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int bpftime_amd_gen_syscall_full(void *dev, uint64_t n, uint64_t seed, uint64_t first, const double *cdf,
                                            uint32_t support, void *stream) {
  if (!cdf || !support) return -1;
  if (!n) return 0;
  hipLaunchKernelGGL(bpftime_amd::k_gen_syscall_full, dim3(gen_blocks(n * 12)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t *)dev, 96, (uint8_t *)dev + 64, 96, n, seed, first, cdf, support);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int bpftime_amd_gen_syscall_soa(void *enter, void *exit, uint64_t n, uint64_t seed, uint64_t first,
                                           const double *cdf, uint32_t support, void *stream) {
  if (!cdf || !support || !exit) return -1;
  if (!n) return 0;
  hipLaunchKernelGGL(bpftime_amd::k_gen_syscall_full, dim3(gen_blocks(n * 12)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t *)enter, 64, (uint8_t *)exit, 32, n, seed, first, cdf, support);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int bpftime_amd_gen_xdp(void *dev, uint64_t n, uint64_t stride, uint32_t len, uint64_t seed,
                                   uint64_t first, void *stream) {
  (void)len;
  if (stride % 8 || stride < 16) return -1;
  uint64_t total = n * (stride / 8);
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(bpftime_amd::k_gen_xdp, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t *)dev, n, stride, seed, first);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
