// bpftime_amd: device side of the syscall dispatch's per-record state
// (csrc/syscall_dispatch.cpp): before the programs run, every record's
// override flags are cleared and its return value is what dispatch_syscall
// returns when no program overrides it -- the recorded ret of a 96- or 128-B record
// (trace_event_raw_sys_exit.ret at +80, syscall_trace_attach_impl.cpp:78-93),
// 0 for a 64-B enter record, which holds none.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpftime_amd {

__global__ void k_sys_init(const uint8_t *records, uint64_t n, uint32_t record_size, int64_t *out,
                           uint32_t *state) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (state) state[i] = 0;
    if (out) out[i] = record_size >= 88 ? *(const int64_t *)(records + i * record_size + 80) : 0;
  }
}

}  // namespace bpftime_amd

extern "C" hipError_t bpftime_amd_launch_sys_init(const void *records, uint64_t n, uint32_t record_size,
                                                  int64_t *out, uint32_t *state, hipStream_t stream) {
  if (!n) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bpftime_amd::k_sys_init, dim3((uint32_t)blocks), dim3(256), 0, stream,
                     (const uint8_t *)records, n, record_size, out, state);
  return hipGetLastError();
}
