// PMC calibration kernels (tools only, not product): each kernel moves a
// byte count known by construction in one access shape the interpreter's
// bench lines use, over buffers far past the 256 MiB Infinity Cache, so
// tools/calib_table.py can turn rocprofv3's FETCH_SIZE / WRITE_SIZE of that
// shape into bytes (MI355X_MICROARCH.md HBM section: only 16-B/lane
// streaming reads and stores are calibrated there).  Kernel names carry the
// shape; every kernel is launched REPS times, timed with events (the
// achieved GB/s of the shape is its speed of light).
//
//   calib [log2 slots = 24]
//
// shapes (n = 2^log2 slots):
//   c_rd16of64     16 B read of each 64-B slot             (xdp-counter staged read)
//   c_rd64of64     all 64 B of each 64-B slot                (full-line reads, known bytes)
//   c_rw16of64     16 B read + 16 B written back per slot   (xdp-counter in-place rewrite)
//   c_rwfull64     64 B read + 64 B written per slot        (copy-shaped in-place update)
//   c_wr4          4 B per lane, coalesced                  (verdicts)
//   c_rd128of2048  128 B read of each 2048-B slot           (flow-hash header line), 2^22 slots
//   c_gather8_4M   8-B random gathers over a 4 MiB table    (hash probes, L2-resident)
//   c_gather8_64M  8-B random gathers over a 64 MiB table   (L3-resident)
//   c_gather8_1G   8-B random gathers over a 1 GiB table    (HBM)
//   c_wr32of64     32-B masked store per 64-B slot          (partial-line writes)
//   c_atom8_4M     8-B atomic adds, random over 4 MiB       (combining-table misses)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define KB __launch_bounds__(256)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

__global__ KB void c_rd16of64(const uint8_t *d, uint32_t *sink, uint64_t n) {
  uint32_t acc = 0;
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull) {
    const uint4 x = *(const uint4 *)(d + u * 64);
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ KB void c_rd64of64(const uint8_t *d, uint32_t *sink, uint64_t n) {
  uint32_t acc = 0;
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull) {
    const uint4 *p = (const uint4 *)(d + u * 64);
    const uint4 a = p[0], b = p[1], c = p[2], e = p[3];
    acc ^= a.x ^ b.y ^ c.z ^ e.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ KB void c_rw16of64(uint8_t *d, uint32_t *sink, uint64_t n) {
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull) {
    uint4 *p = (uint4 *)(d + u * 64);
    uint4 x = p[0];
    x.x += 1;
    p[0] = x;
  }
}

__global__ KB void c_rwfull64(uint8_t *d, uint32_t *sink, uint64_t n) {
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull) {
    uint4 *p = (uint4 *)(d + u * 64);
    uint4 a = p[0], b = p[1], c = p[2], e = p[3];
    a.x += 1;
    p[0] = a;
    p[1] = b;
    p[2] = c;
    p[3] = e;
  }
}

__global__ KB void c_wr4(uint8_t *d, uint32_t *v, uint64_t n) {
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull) v[u] = 3;
}

__global__ KB void c_rd128of2048(const uint8_t *d, uint32_t *sink, uint64_t n) {
  // 8 lanes per slot, 16 B each: one whole 128-B line per 2048-B slot
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n * 8; t += gridDim.x * 256ull) {
    const uint4 x = *(const uint4 *)(d + (t >> 3) * 2048 + (t & 7) * 16);
    acc ^= x.x ^ x.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <uint64_t TABLE>
__global__ KB void c_gather8(const uint8_t *d, uint32_t *sink, uint64_t n) {
  uint64_t acc = 0;
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull)
    acc += *(const uint64_t *)(d + (mix(u) % (TABLE / 8)) * 8);
  if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (uint32_t)acc;
}

__global__ KB void c_wr32of64(uint8_t *d, uint32_t *sink, uint64_t n) {
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull) {
    uint4 *p = (uint4 *)(d + u * 64);
    p[0] = make_uint4((uint32_t)u, 1, 2, 3);
    p[1] = make_uint4((uint32_t)u, 4, 5, 6);
  }
}

__global__ KB void c_atom8_4M(uint8_t *d, uint32_t *sink, uint64_t n) {
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull)
    __hip_atomic_fetch_add((uint64_t *)(d + (mix(u) % ((4ull << 20) / 8)) * 8), 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// the same adds with workgroup scope into a per-XCD copy of the 4 MiB
// region (HW_REG_XCC_ID picks the copy): performed in the XCD's L2, which
// no other XCD shares, instead of at the memory side
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

__global__ KB void c_atom8_4M_xcd(uint8_t *d, uint32_t *sink, uint64_t n) {
  uint8_t *mine = d + (uint64_t)(xcc_id() & 7) * (4ull << 20);
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull)
    __hip_atomic_fetch_add((uint64_t *)(mine + (mix(u) % ((4ull << 20) / 8)) * 8), 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ KB void c_atom8_1M_xcd(uint8_t *d, uint32_t *sink, uint64_t n) {
  uint8_t *mine = d + (uint64_t)(xcc_id() & 7) * (1ull << 20);
  for (uint64_t u = blockIdx.x * 256ull + threadIdx.x; u < n; u += gridDim.x * 256ull)
    __hip_atomic_fetch_add((uint64_t *)(mine + (mix(u) % ((1ull << 20) / 8)) * 8), 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}

// which XCD runs which block: blockIdx.x % 8 under round-robin placement
__global__ KB void c_xcc_map(uint8_t *d, uint32_t *sink, uint64_t n) {
  if (threadIdx.x == 0 && blockIdx.x < 64) sink[blockIdx.x] = xcc_id();
}

int main(int argc, char **argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 24;
  const uint64_t n = 1ull << lg;
  const uint64_t bytes = n * 64 > (1ull << 30) ? n * 64 : (1ull << 30);  // >= 1 GiB: past the L3
  const uint64_t fbytes = 8ull << 30;  // 2^22 2048-B slots: 512 MiB of header lines, past the L3
  uint8_t *d, *t, *f;
  uint32_t *v;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&v, n * 4) != hipSuccess ||
      hipMalloc(&t, 1ull << 30) != hipSuccess || hipMalloc(&f, fbytes) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  hipMemset(d, 0x5a, bytes);
  hipMemset(t, 0x11, 1ull << 30);
  hipMemset(f, 0x22, fbytes);
  hipMemset(v, 0, n * 4);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int REPS = 5;
  const uint32_t grid = 256 * 8;  // 8 blocks per CU
  // name, kernel, data, units, known bytes read per unit, known bytes written per unit
  auto run = [&](const char *name, auto kern, uint8_t *buf, uint64_t units, double rd, double wr) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, buf, v, units);
    hipEventRecord(e0);
    for (int i = 0; i < REPS; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, buf, v, units);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= REPS;
    printf("{\"kernel\": \"%s\", \"units\": %llu, \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"ms\": %.4f, "
           "\"GBps\": %.1f}\n",
           name, (unsigned long long)units, rd * units, wr * units, ms, (rd + wr) * units / ms / 1e6);
  };
  run("c_rd16of64", c_rd16of64, d, n, 16, 0);
  run("c_rd64of64", c_rd64of64, d, n, 64, 0);
  run("c_rw16of64", c_rw16of64, d, n, 16, 16);
  run("c_rwfull64", c_rwfull64, d, n, 64, 64);
  run("c_wr4", c_wr4, d, n, 0, 4);
  run("c_rd128of2048", c_rd128of2048, f, fbytes / 2048, 128, 0);
  run("c_gather8_4M", c_gather8<4ull << 20>, t, n, 8, 0);
  run("c_gather8_64M", c_gather8<64ull << 20>, t, n, 8, 0);
  run("c_gather8_1G", c_gather8<1ull << 30>, t, n, 8, 0);
  run("c_wr32of64", c_wr32of64, d, n, 0, 32);
  run("c_atom8_4M", c_atom8_4M, t, n, 8, 8);
  run("c_atom8_4M_xcd", c_atom8_4M_xcd, t, n, 8, 8);
  run("c_atom8_1M_xcd", c_atom8_1M_xcd, t, n, 8, 8);
  // the per-XCD copies hold every add: their sum over the copies is REPS + 1 adds per unit
  {
    uint64_t *h = (uint64_t *)malloc(32ull << 20);
    hipMemset(t, 0, 32ull << 20);
    hipLaunchKernelGGL(c_atom8_4M_xcd, dim3(grid), dim3(256), 0, 0, t, v, n);
    hipMemcpy(h, t, 32ull << 20, hipMemcpyDeviceToHost);
    uint64_t sum = 0;
    for (uint64_t i = 0; i < (32ull << 20) / 8; i++) sum += h[i];
    printf("{\"check\": \"c_atom8_4M_xcd adds\", \"sum\": %llu, \"want\": %llu}\n", (unsigned long long)sum,
           (unsigned long long)n);
    free(h);
    hipLaunchKernelGGL(c_xcc_map, dim3(64), dim3(256), 0, 0, t, v, 64);
    uint32_t m[64];
    hipMemcpy(m, v, sizeof(m), hipMemcpyDeviceToHost);
    printf("{\"xcc_of_block\": [");
    for (int i = 0; i < 64; i++) printf("%u%s", m[i], i < 63 ? ", " : "");
    printf("]}\n");
  }
  return 0;
}
