// bpftime_amd: device side of the syscall dispatch's per-record state
// (csrc/syscall_dispatch.cpp): before the programs run, every record's
// override flags are cleared and its return value is what dispatch_syscall
// returns when no program overrides it -- the recorded ret
// (trace_event_raw_sys_exit.ret, syscall_trace_attach_impl.cpp:78-93), 0 for
// a 64-B enter record, which holds none.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpftime_amd {

__global__ void k_sys_init(const uint8_t *exits, uint64_t n, uint64_t xstride, int64_t *out, uint32_t *state) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (state) state[i] = 0;
    if (out) out[i] = exits ? *(const int64_t *)(exits + i * xstride + 16) : 0;
  }
}

}  // namespace bpftime_amd

// exits: record i's trace_event_raw_sys_exit at exits + i * xstride (ret at
// +16), or null (64-B enter records)
extern "C" hipError_t bpftime_amd_launch_sys_init(const void *exits, uint64_t n, uint64_t xstride,
                                                  int64_t *out, uint32_t *state, hipStream_t stream) {
  if (!n) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bpftime_amd::k_sys_init, dim3((uint32_t)blocks), dim3(256), 0, stream,
                     (const uint8_t *)exits, n, xstride, out, state);
  return hipGetLastError();
}
