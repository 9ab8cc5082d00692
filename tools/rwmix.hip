// rwmix.hip -- BENCH TOOLING: how the cost of a small write stream mixed
// into a large read stream depends on the write burst size.  Each wave reads
// tiles of `rb` contiguous bytes (1 KB per load instruction, 8 in flight) in
// grid-strided tile order, exactly like the rx kernel, and after each tile
// writes `wb` contiguous bytes at the tile's output position (one burst).
// Values are garbage; only the time counts.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// INDEP: the burst stores a value that does not depend on the tile's loads
// (so the stores need not wait for them): separates the memory's cost of the
// writes from the wait the dependent stores put on the read stream.
// WRAP: the bursts go to a 32 MiB window reused over and over (they stay in
// the caches; not a real output, an experiment on where the write cost is).
template <bool NT, bool INDEP = false, bool WRAP = false, bool NTST = true, uint32_t WIN = 32u << 20>
__global__ __launch_bounds__(256) void rw_kernel(const u32x4 *in, u32x4 *out, uint64_t ntiles,
                                                 uint32_t rb16, uint32_t wb16, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    const u32x4 *p = in + t * rb16;
    uint32_t k = lane;
    for (; k + 7 * 64 < rb16; k += 8 * 64) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = NT ? __builtin_nontemporal_load(p + k + u * 64) : p[k + u * 64];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= v[u];
    }
    for (; k < rb16; k += 64) acc ^= p[k];
    u32x4 *q = out + (WRAP ? (t * (uint64_t)wb16) & (WIN / 16 - 1) : t * (uint64_t)wb16);
    const u32x4 val = INDEP ? u32x4{(uint32_t)t, (uint32_t)lane, 0u, 0u} : acc;
    for (uint32_t e = lane; e < wb16; e += 64) {
      if (NT && NTST) __builtin_nontemporal_store(val, q + e);
      else q[e] = val;
    }
  }
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) sink[lane] = x;
}

extern "C" int rwmix_run(const void *in, void *out, uint64_t ntiles, uint32_t rb, uint32_t wb,
                         int nt, int grid, uint32_t *sink, void *stream) {
  if (nt == 13)
    hipLaunchKernelGGL((rw_kernel<true, false, true, false, (1u << 20)>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else if (nt == 9)
    hipLaunchKernelGGL((rw_kernel<true, false, false, false>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else if (nt == 5)
    hipLaunchKernelGGL((rw_kernel<true, false, true>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else if (nt == 3)
    hipLaunchKernelGGL((rw_kernel<true, true>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else if (nt)
    hipLaunchKernelGGL(rw_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else
    hipLaunchKernelGGL(rw_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
