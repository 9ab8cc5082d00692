// membench.hip -- BENCH TOOLING: the box's achievable HBM read bandwidth,
// measured in the same process as the rx kernel (GPU-to-GPU variance is
// large enough that cross-run comparisons mislead).  A grid-stride
// dwordx4 read stream with 8 loads in flight per lane, xor-folded so the
// loads cannot be elided; optionally non-temporal.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void read_stream(const u32x4 *p, uint64_t n16, uint32_t *out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  uint64_t i = tid;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = NT ? __builtin_nontemporal_load(p + i + k * stride) : p[i + k * stride];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  for (; i < n16; i += stride) acc ^= p[i];
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) out[tid & 1023] = x;   // practically never: keeps loads alive
}

__global__ __launch_bounds__(256) void copy_stream(const u32x4 *p, u32x4 *q, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) q[i] = p[i];
}

extern "C" int membench_read(const void *p, uint64_t bytes, uint32_t *out, int nt, int grid, void *stream) {
  const uint64_t n16 = bytes / 16;
  if (nt) hipLaunchKernelGGL(read_stream<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const u32x4 *)p, n16, out);
  else hipLaunchKernelGGL(read_stream<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const u32x4 *)p, n16, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int membench_copy(const void *p, void *q, uint64_t bytes, int grid, void *stream) {
  hipLaunchKernelGGL(copy_stream, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const u32x4 *)p, (u32x4 *)q, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
