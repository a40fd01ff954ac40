// bpftime_amd: the thread grouping of the thread-ordered syscall dispatch
// (common.hpp SeqParams, interp.hip k_sys_seq).
//
// A replay record names its calling thread (96- / 128-B records: the u64
// pid_tgid at +88; struct-of-arrays records: in the exit array,
// include/bpftime_amd.h); the reference runs a thread's
// calls one after another on that thread (syscall_trace_attach_impl.cpp:
// 18-95 runs on the caller).  Grouping = a stable radix sort of (pid_tgid,
// record index) pairs: thread t's records are perm[seg[t] .. seg[t + 1]) in
// record order.  Heads of equal-key runs become the segment starts
// (rocprim select over the head flags); seg[nseg] = n.
#include <hip/hip_runtime.h>

#include <string.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

namespace {

__global__ void k_group_keys(const uint8_t *pid, uint64_t n, uint64_t stride, uint64_t *keys, uint32_t *idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = *(const uint64_t *)(pid + i * stride);
  idx[i] = (uint32_t)i;
}

__global__ void k_group_heads(const uint64_t *keys, uint64_t n, uint8_t *flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = i == 0 || keys[i] != keys[i - 1];
}

__global__ void k_group_tail(uint32_t *seg, const uint32_t *nsel, uint64_t n) { seg[*nsel] = (uint32_t)n; }

struct Layout {
  size_t keys_in, keys_out, idx_in, perm, flags, seg, nsel, temp, total;
  size_t temp_bytes;
};

size_t up(size_t v) { return (v + 255) & ~(size_t)255; }

hipError_t layout(uint64_t n, Layout &l) {
  size_t sort_bytes = 0, sel_bytes = 0;
  hipError_t e = rocprim::radix_sort_pairs(nullptr, sort_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0, 64);
  if (e != hipSuccess) return e;
  e = rocprim::select(nullptr, sel_bytes, rocprim::counting_iterator<uint32_t>(0), (const uint8_t *)nullptr,
                      (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n);
  if (e != hipSuccess) return e;
  l.temp_bytes = sort_bytes > sel_bytes ? sort_bytes : sel_bytes;
  size_t o = 0;
  l.keys_in = o; o += up(8 * n);
  l.keys_out = o; o += up(8 * n);
  l.idx_in = o; o += up(4 * n);
  l.perm = o; o += up(4 * n);
  l.flags = o; o += up(n);
  l.seg = o; o += up(4 * (n + 1));
  l.nsel = o; o += 256;
  l.temp = o; o += up(l.temp_bytes);
  l.total = o;
  return hipSuccess;
}

}  // namespace

// Scratch bytes bpftime_amd_group_threads needs for n records (0 on error).
extern "C" size_t bpftime_amd_group_scratch_bytes(uint64_t n) {
  Layout l;
  if (n == 0 || n > 0xffffffffull || layout(n, l) != hipSuccess) return 0;
  return l.total;
}

// Groups n records by their pid_tgid (record i's at pid + i * stride) into
// `scratch` (bpftime_amd_group_scratch_bytes(n) bytes): *perm / *seg point
// into it; *nseg = the thread count (a synchronous read of the selected count).
extern "C" hipError_t bpftime_amd_group_threads(const void *pid, uint64_t stride, uint64_t n, void *scratch,
                                                uint32_t **perm, uint32_t **seg, uint64_t *nseg,
                                                hipStream_t stream) {
  Layout l;
  if (n == 0 || n > 0xffffffffull || !pid || stride % 8) return hipErrorInvalidValue;
  hipError_t e = layout(n, l);
  if (e != hipSuccess) return e;
  uint8_t *b = (uint8_t *)scratch;
  uint64_t *keys_in = (uint64_t *)(b + l.keys_in), *keys_out = (uint64_t *)(b + l.keys_out);
  uint32_t *idx_in = (uint32_t *)(b + l.idx_in), *pm = (uint32_t *)(b + l.perm), *sg = (uint32_t *)(b + l.seg);
  uint32_t *nsel = (uint32_t *)(b + l.nsel);
  uint8_t *flags = b + l.flags;
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_group_keys, dim3(grid), dim3(256), 0, stream, (const uint8_t *)pid, n, stride, keys_in,
                     idx_in);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  size_t tb = l.temp_bytes;
  e = rocprim::radix_sort_pairs(b + l.temp, tb, (const uint64_t *)keys_in, keys_out, (const uint32_t *)idx_in, pm,
                                (size_t)n, 0, 64, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_group_heads, dim3(grid), dim3(256), 0, stream, (const uint64_t *)keys_out, n, flags);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  tb = l.temp_bytes;
  e = rocprim::select(b + l.temp, tb, rocprim::counting_iterator<uint32_t>(0), (const uint8_t *)flags, sg, nsel,
                      (size_t)n, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_group_tail, dim3(1), dim3(1), 0, stream, sg, (const uint32_t *)nsel, n);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  uint32_t h = 0;
  if ((e = hipMemcpyAsync(&h, nsel, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
  *perm = pm;
  *seg = sg;
  *nseg = h;
  return hipSuccess;
}
