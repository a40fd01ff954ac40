// Speed-of-light probe for the xdp-counter access pattern (tools only, not
// product): per 64-B slot read the first 16 B, swap the MACs, write the 16 B
// back, write a 4-B verdict.  Variants: grid-stride with the interpreter's
// grid (16 waves/CU) and U units per lane in flight, or one unit per thread.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int U>
__global__ __launch_bounds__(256) void k_sol(uint8_t *d, uint32_t *v, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t u0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; u0 < n; u0 += step) {
    uint4 x[U];
#pragma unroll
    for (int k = 0; k < U; k++) x[k] = *(const uint4 *)(d + (u0 + 256 * k) * 64);
#pragma unroll
    for (int k = 0; k < U; k++) {
      uint4 y = x[k];
      // bytes 0-5 <-> 6-11
      uint32_t a = x[k].x, b = x[k].y, c = x[k].z;
      y.x = __builtin_amdgcn_perm(b, c, 0x01000706);  // bytes 6,7,8,9
      y.y = __builtin_amdgcn_perm(a, c, 0x05040302 & 0xffffffff);
      y.z = c;
      *(uint4 *)(d + (u0 + 256 * k) * 64) = y;
      v[u0 + 256 * k] = 3;
    }
  }
}

// variants: W=0 read 16 B only + verdict; W=1 16-B store; W=2 full 64-B line
// store (loads 64 B); W=3 16-B nontemporal store; W=4 verdict only
template <int W>
__global__ __launch_bounds__(256) void k_var(uint8_t *d, uint32_t *v, uint64_t n) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < n; u += step) {
    uint4 *p = (uint4 *)(d + u * 64);
    if (W == 4) { v[u] = 3; continue; }
    uint4 x = p[0];
    uint4 y = x;
    y.x = __builtin_amdgcn_perm(x.y, x.z, 0x01000706);
    y.y = __builtin_amdgcn_perm(x.x, x.z, 0x05040302);
    if (W == 0) { v[u] = y.x == 12345 ? 1 : 3; continue; }
    if (W == 1) p[0] = y;
    if (W == 3) { uint32_t *q = (uint32_t *)p; __builtin_nontemporal_store(y.x, q); __builtin_nontemporal_store(y.y, q + 1); __builtin_nontemporal_store(y.z, q + 2); }
    if (W == 2) { uint4 a = p[1], b = p[2], c = p[3]; p[0] = y; p[1] = a; p[2] = b; p[3] = c; }
    v[u] = 3;
  }
}
int main() {
  const uint64_t n = 1ull << 24;
  uint8_t *d; uint32_t *v;
  hipMalloc(&d, n * 64); hipMalloc(&v, n * 4);
  hipMemset(d, 0x5a, n * 64);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char *name, auto kern, uint32_t grid) {
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, v, n);
    hipEventRecord(e0);
    for (int i = 0; i < 20; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, v, n);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 20;
    printf("%-34s grid %7u  %.4f ms  %8.1f Gpps  %6.0f GB/s @100B/pkt\n", name, grid, ms, n / ms / 1e6,
           n * 100.0 / ms / 1e6);
  };
  run("U=1 grid 1024 (16 waves/CU)", k_sol<1>, 1024);
  run("U=2 grid 1024", k_sol<2>, 1024);
  run("U=4 grid 1024", k_sol<4>, 1024);
  run("U=1 grid 2048", k_sol<1>, 2048);
  run("U=1 one unit per thread", k_sol<1>, (uint32_t)(n / 256));
  run("U=4 grid n/1024", k_sol<4>, (uint32_t)(n / 1024));
  run("read 16B + verdict", k_var<0>, 1024);
  run("verdict only", k_var<4>, 1024);
  run("16B store (same as U=1)", k_var<1>, 1024);
  run("full-line 64B store", k_var<2>, 1024);
  run("16B nontemporal store", k_var<3>, 1024);
  run("16B store grid n/256", k_var<1>, (uint32_t)(n / 256));
  run("full-line store grid n/256", k_var<2>, (uint32_t)(n / 256));
  return 0;
}
