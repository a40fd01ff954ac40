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

}  // namespace bpftime_amd

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
