// standin.hip -- PROBE TOOLING: a stand-in for RCCL's all-gather kernel with
// its resource footprint on gfx950 (ncclDevKernel_Generic in /opt/rocm's
// librccl: 512 threads per block, 37 664 B of LDS, 248 VGPRs -- so one block
// needs a whole CU), spinning for a given time without memory traffic.
// tools/standin.py runs it beside the rx kernel the way bench.py overlaps a
// batch with the previous batch's gather, to see whether the persistent rx
// grid lets such a kernel run at all.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(512, 1) void standin_kernel(uint64_t ticks, uint32_t *sink,
                                                        uint64_t *trace) {
  __shared__ uint32_t lds[37664 / 4];
  // the VGPR footprint: a clobber of v247 makes the kernel allocate 248
  asm volatile("" ::: "v247");
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = lds[(threadIdx.x + 1) % 512];
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    acc = acc * 2654435761u + 1u;
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
  if (trace && threadIdx.x == 0) {
    // per block: start, XCC_ID, HW_ID (se bits 15:13)
    trace[3 * blockIdx.x] = t0;
    trace[3 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg(20 | (15 << 11));
    trace[3 * blockIdx.x + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  }
}

// The same footprint copying `bytes` from src to dst (the ranks' landing
// bytes and the forwarded reads of a ring all-gather), paced so that it
// takes at least `ticks`: each block copies its contiguous slice in 16-byte
// non-temporal loads and stores, and after every 64 KB waits until the
// clock has reached that fraction of the duration (xGMI-rate arrival).
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512, 1) void standin_copy_kernel(const u32x4s *src, u32x4s *dst,
                                                             uint64_t n16, uint64_t ticks) {
  __shared__ uint32_t lds[37664 / 4];
  asm volatile("" ::: "v247");
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = min(n16, per * blockIdx.x), hi = min(n16, lo + per);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t chunk = 4096;   // 16-byte units: 64 KB
  for (uint64_t c = lo; c < hi; c += chunk) {
    const uint64_t e = min(hi, c + chunk);
    u32x4s v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t i = c + threadIdx.x + k * 512;
      if (i < e) v[k] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t i = c + threadIdx.x + k * 512;
      if (i < e) __builtin_nontemporal_store(v[k], dst + i);
    }
    const uint64_t due = t0 + ticks * (e - lo) / max<uint64_t>(1, hi - lo);
    while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(8);
  }
  if (lds[(threadIdx.x + 1) % 512] == 0xffffffffu) dst[0] = u32x4s{0, 0, 0, 0};
}

extern "C" int standin_copy(int blocks, uint64_t ticks, const void *src, void *dst, uint64_t bytes,
                            void *stream) {
  if (bytes % 16) return -22;
  hipLaunchKernelGGL(standin_copy_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream,
                     (const u32x4s *)src, (u32x4s *)dst, bytes / 16, ticks);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int standin_run(int blocks, uint64_t ticks, uint32_t *sink, uint64_t *trace,
                           void *stream) {
  hipLaunchKernelGGL(standin_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream, ticks, sink,
                     trace);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Which CUs does a CU mask name?  A stream with the given mask runs
// `blocks` blocks of one wave; each records its XCC_ID and HW_ID registers
// (HW_ID: cu_id bits 11:8, sh_id bit 12, se_id bits 15:13).
__global__ void whoami_kernel(uint32_t *out) {
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg(20 | (15 << 11));   // HW_REG_XCC_ID
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg(4 | (31 << 11)); // HW_REG_HW_ID
    __builtin_amdgcn_s_sleep(127);
  }
}

extern "C" int standin_whoami(int nwords, const uint32_t *mask, int blocks, uint32_t *d_out) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return -1;
  hipLaunchKernelGGL(whoami_kernel, dim3(blocks), dim3(64), 0, s, d_out);
  const hipError_t e = hipStreamSynchronize(s);
  hipStreamDestroy(s);
  return e == hipSuccess ? 0 : -2;
}
