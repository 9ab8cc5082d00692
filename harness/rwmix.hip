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

// Blocked tile order: wave w takes runs of B consecutive tiles (run w,
// w + nwaves, ...) and writes each tile's wb bytes right after it (4 KB
// bursts, like the rx kernel, but a wave's reads walk one contiguous span).
template <int B>
__global__ __launch_bounds__(256) void rw_blk_kernel(const u32x4 *in, u32x4 *out, uint64_t ntiles,
                                                     uint32_t rb16, uint32_t wb16, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t r = wid; r * B < ntiles; r += nwaves)
    for (uint64_t t = r * B; t < min(ntiles, r * B + B); ++t) {
      const u32x4 *p = in + t * rb16;
      uint32_t k = lane;
      for (; k + 7 * 64 < rb16; k += 8 * 64) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + k + u * 64);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u];
      }
      for (; k < rb16; k += 64) acc ^= __builtin_nontemporal_load(p + k);
      u32x4 *q = out + t * (uint64_t)wb16;
      for (uint32_t e = lane; e < wb16; e += 64) __builtin_nontemporal_store(acc, q + e);
    }
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) sink[lane] = x;
}

extern "C" int rwblk_run(const void *in, void *out, uint64_t ntiles, uint32_t rb, uint32_t wb,
                         int b, int grid, uint32_t *sink, void *stream) {
  if (b == 64)
    hipLaunchKernelGGL(rw_blk_kernel<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else
    hipLaunchKernelGGL(rw_blk_kernel<8>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)in, (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Speed-of-light kernel for an rx launch's exact traffic (bench.py mix_sol):
// tile t = frames [64t, 64t + 64); its bytes are the contiguous span
// [t * rb, t * rb + rb) (fixed stride) or, for frames packed in batch order
// and described by off/len (CMIX), [off[64t], off[last] + len[last]) read
// after the tile's 64 descriptors; every lane keeps up to U 16-byte loads
// in flight (the whole tile of a small-frame batch at once: a 4 KB C64
// tile is 4 loads per lane), then the tile's wb record bytes are written
// as one burst.  Nothing is parsed or summed beyond a xor that keeps the
// loads alive.
// PH (period > 0): the rx kernel's global write phases -- a tile's record
// bytes held (here: the value they are made of) until the chip-wide clock
// passes the next multiple of `period` ticks, checked after every load
// group, or until the next tile's are ready (rx_kernel.hip "Global write
// phases").
template <bool NT, bool GATHER, int U, bool PH = false>
__global__ __launch_bounds__(256) void sol_kernel(const uint8_t *in, const uint64_t *off,
                                                  const uint16_t *len, uint64_t n, u32x4 *out,
                                                  uint64_t ntiles, uint32_t rb, uint32_t wb16,
                                                  uint32_t *sink, uint32_t period = 0) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 pend = acc;
  uint64_t tpend = ~0ull, deadline = 0;
  auto write = [&](uint64_t t, u32x4 v) {
    u32x4 *q = out + t * (uint64_t)wb16;
    for (uint32_t e = lane; e < wb16; e += 64) {
      if (NT) __builtin_nontemporal_store(v, q + e);
      else q[e] = v;
    }
  };
  for (uint64_t t = wid; t < ntiles; t += nwaves) {
    uint64_t lo, hi;
    if constexpr (GATHER) {
      const uint64_t i = min(t * 64 + (uint64_t)lane, n - 1);
      const uint64_t o = off[i], e = o + len[i];
      lo = __shfl(o, 0) & ~(uint64_t)15;
      hi = __shfl(e, 63);
    } else {
      lo = t * (uint64_t)rb;
      hi = lo + rb;
    }
    const u32x4 *p = (const u32x4 *)(in + lo);
    const uint32_t nch = (uint32_t)((hi - lo + 15) >> 4);
    for (uint32_t k0 = 0; k0 < nch; k0 += U * 64) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t k = min(k0 + (uint32_t)(u * 64 + lane), nch - 1);
        v[u] = NT ? __builtin_nontemporal_load(p + k) : p[k];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
      if (PH && tpend != ~0ull && __builtin_amdgcn_s_memrealtime() >= deadline) {
        write(tpend, pend);
        tpend = ~0ull;
      }
    }
    if (PH) {
      if (tpend != ~0ull) write(tpend, pend);
      tpend = t;
      pend = acc;
      const uint64_t rt = __builtin_amdgcn_s_memrealtime();
      deadline = rt - rt % period + period;
    } else {
      write(t, acc);
    }
  }
  if (PH && tpend != ~0ull) write(tpend, pend);
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) sink[lane] = x;
}

// mode bit 0: non-temporal loads/stores; bit 1: descriptors (off/len);
// bit 2: 4 loads per lane in flight instead of 16; bit 3: global write
// phases of `period` ticks (non-temporal modes)
extern "C" int sol_run_phased(const void *in, const void *off, const void *len, uint64_t n,
                              void *out, uint64_t ntiles, uint32_t rb, uint32_t wb, int mode,
                              int grid, uint32_t *sink, uint32_t period, void *stream) {
  const hipStream_t s = (hipStream_t)stream;
  if (period == 0) return -22;
#define SOL_PH(G, U)                                                                              \
  hipLaunchKernelGGL((sol_kernel<true, G, U, true>), dim3(grid), dim3(256), 0, s,                 \
                     (const uint8_t *)in, (const uint64_t *)off, (const uint16_t *)len, n,        \
                     (u32x4 *)out, ntiles, rb, wb / 16, sink, period)
  switch (mode & 7) {
    case 1: SOL_PH(false, 16); break;
    case 3: SOL_PH(true, 16); break;
    case 5: SOL_PH(false, 4); break;
    case 7: SOL_PH(true, 4); break;
    default: return -22;
  }
#undef SOL_PH
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int sol_run(const void *in, const void *off, const void *len, uint64_t n, void *out,
                       uint64_t ntiles, uint32_t rb, uint32_t wb, int mode, int grid,
                       uint32_t *sink, void *stream) {
  const hipStream_t s = (hipStream_t)stream;
#define SOL_LAUNCH(NT, G, U)                                                                      \
  hipLaunchKernelGGL((sol_kernel<NT, G, U>), dim3(grid), dim3(256), 0, s, (const uint8_t *)in,   \
                     (const uint64_t *)off, (const uint16_t *)len, n, (u32x4 *)out, ntiles, rb,    \
                     wb / 16, sink)
  switch (mode & 7) {
    case 0: SOL_LAUNCH(false, false, 16); break;
    case 1: SOL_LAUNCH(true, false, 16); break;
    case 2: SOL_LAUNCH(false, true, 16); break;
    case 3: SOL_LAUNCH(true, true, 16); break;
    case 4: SOL_LAUNCH(false, false, 4); break;
    case 5: SOL_LAUNCH(true, false, 4); break;
    case 6: SOL_LAUNCH(false, true, 4); break;
    default: SOL_LAUNCH(true, true, 4); break;
  }
#undef SOL_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Deferred record writes: each wave reads G strided tiles (tile t, t +
// nwaves, ...: the rx kernel's tile order) of rb bytes, keeping one 16-byte
// value per tile, and only then writes the G tiles' wb-byte outputs, each at
// its own tile's position (what an rx kernel that staged G tiles' records
// before flushing them would write: clustered in time, not contiguous).
template <int G>
__global__ __launch_bounds__(256) void rw_defer_kernel(const u32x4 *in, u32x4 *out,
                                                       uint64_t ntiles, uint32_t rb16,
                                                       uint32_t wb16, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  u32x4 tot = {0, 0, 0, 0};
  for (uint64_t t0 = wid; t0 < ntiles; t0 += nwaves * G) {
    u32x4 acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      acc[g] = (u32x4){0, 0, 0, 0};
      const uint64_t t = t0 + (uint64_t)g * nwaves;
      if (t >= ntiles) continue;
      const u32x4 *p = in + t * rb16;
      uint32_t k = lane;
      for (; k + 7 * 64 < rb16; k += 8 * 64) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + k + u * 64);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[g] ^= v[u];
      }
      for (; k < rb16; k += 64) acc[g] ^= __builtin_nontemporal_load(p + k);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint64_t t = t0 + (uint64_t)g * nwaves;
      if (t >= ntiles) continue;
      u32x4 *q = out + t * (uint64_t)wb16;
      for (uint32_t e = lane; e < wb16; e += 64) __builtin_nontemporal_store(acc[g], q + e);
      tot ^= acc[g];
    }
  }
  const uint32_t x = tot.x ^ tot.y ^ tot.z ^ tot.w;
  if (x == 0x9e3779b9u) sink[lane] = x;
}

extern "C" int rwdefer_run(const void *in, void *out, uint64_t ntiles, uint32_t rb, uint32_t wb,
                           int g, int grid, uint32_t *sink, void *stream) {
  const hipStream_t s = (hipStream_t)stream;
  if (g == 4)
    hipLaunchKernelGGL(rw_defer_kernel<4>, dim3(grid), dim3(256), 0, s, (const u32x4 *)in,
                       (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else
    hipLaunchKernelGGL(rw_defer_kernel<16>, dim3(grid), dim3(256), 0, s, (const u32x4 *)in,
                       (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Workgroup-staged record writes: a workgroup (4 waves) owns runs of 4*TPW
// consecutive tiles; each wave reads TPW of them (96 KB-style tiles of rb
// bytes) and parks each tile's wb-byte output in LDS; after a barrier the
// whole workgroup flushes the run's 4*TPW*wb bytes as one contiguous burst.
// `pad` bytes of extra dynamic LDS emulate the rx kernel's header images
// (occupancy).  This is the shape an rx kernel staging records in LDS would
// have: bursts of 4*TPW tiles' records instead of one tile's.
template <int TPW>
__global__ __launch_bounds__(256) void rw_stage_kernel(const u32x4 *in, u32x4 *out,
                                                       uint64_t ntiles, uint32_t rb16,
                                                       uint32_t wb16, uint32_t *sink) {
  extern __shared__ u32x4 stage[];
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint64_t runs = ntiles / (4 * TPW);
  u32x4 tot = {0, 0, 0, 0};
  for (uint64_t run = blockIdx.x; run < runs; run += gridDim.x) {
#pragma unroll
    for (int g = 0; g < TPW; ++g) {
      const uint32_t lt = (uint32_t)g * 4 + w;  // tile within the run
      const u32x4 *p = in + (run * 4 * TPW + lt) * rb16;
      u32x4 acc = {0, 0, 0, 0};
      uint32_t k = lane;
      for (; k + 7 * 64 < rb16; k += 8 * 64) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + k + u * 64);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u];
      }
      for (; k < rb16; k += 64) acc ^= __builtin_nontemporal_load(p + k);
      for (uint32_t e = lane; e < wb16; e += 64) stage[lt * wb16 + e] = acc;
      tot ^= acc;
    }
    __syncthreads();
    u32x4 *q = out + run * 4 * TPW * (uint64_t)wb16;
    for (uint32_t e = threadIdx.x; e < 4 * TPW * wb16; e += 256)
      __builtin_nontemporal_store(stage[e], q + e);
    __syncthreads();
  }
  const uint32_t x = tot.x ^ tot.y ^ tot.z ^ tot.w;
  if (x == 0x9e3779b9u) sink[lane] = x;
}

extern "C" int rwstage_run(const void *in, void *out, uint64_t ntiles, uint32_t rb, uint32_t wb,
                           int tpw, uint32_t pad, int grid, uint32_t *sink, void *stream) {
  const hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)4 * tpw * wb + pad;
  if (tpw == 1)
    hipLaunchKernelGGL(rw_stage_kernel<1>, dim3(grid), dim3(256), lds, s, (const u32x4 *)in,
                       (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else if (tpw == 2)
    hipLaunchKernelGGL(rw_stage_kernel<2>, dim3(grid), dim3(256), lds, s, (const u32x4 *)in,
                       (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  else
    hipLaunchKernelGGL(rw_stage_kernel<4>, dim3(grid), dim3(256), lds, s, (const u32x4 *)in,
                       (u32x4 *)out, ntiles, rb / 16, wb / 16, sink);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// XCD-staged record writes (round-4 probe): can records written 4 KB per
// tile still leave the GPU as 256 KB bursts, without LDS?  Runs of 64
// consecutive tiles go to one group of blocks (blockIdx % 8: blocks that
// share an XCD and its L2, observed placement); inside a group the waves
// take the group's tiles grid-strided.  A tile's 4 KB output goes into the
// run's slot of a small per-group staging ring (L2-resident), then the
// wave counts the tile in (agent-scope atomic); the wave completing a run
// copies the run's 256 KB from staging to the output in one burst and frees
// the slot for the run NS later.  A wave whose slot is still busy writes
// its tile directly.  mode bit 0: stage (else: same tile order, direct
// stores); bit 1: non-temporal staging stores.  Values are garbage (the
// real kernel needs the XCC check of the rx kernel's protocol), only the
// time counts.  cnt[] (one word per run) and gen[] (8 * NS words) must be
// zero at launch.
__global__ __launch_bounds__(256) void rw_xstage_kernel(const u32x4 *in, u32x4 *out, u32x4 *stg,
                                                        uint32_t *cnt, uint32_t *gen,
                                                        uint64_t ntiles, uint32_t rb16,
                                                        uint32_t wb16, uint32_t ns, int mode,
                                                        uint32_t *sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint32_t x = blockIdx.x & 7u;                    // group (shared XCD, observed)
  const uint64_t wg = (uint64_t)(gridDim.x / 8) * 4;     // waves per group
  const uint64_t gw = (uint64_t)(blockIdx.x / 8) * 4 + w;
  const uint64_t nruns = (ntiles + 63) / 64;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t s = gw;; s += wg) {
    const uint64_t k = s / 64, run = k * 8 + x, tile = run * 64 + s % 64;
    if (run >= nruns || tile >= ntiles) break;
    const u32x4 *p = in + tile * rb16;
    uint32_t e = lane;
    for (; e + 7 * 64 < rb16; e += 8 * 64) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + e + u * 64);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= v[u];
    }
    for (; e < rb16; e += 64) acc ^= __builtin_nontemporal_load(p + e);
    const uint32_t slot = (uint32_t)(k % ns);
    uint32_t *g = gen + x * ns + slot;
    // bit 2: no protocol at all (always stage; the wave of the run's last
    // tile flushes right after its own tile): the data movement alone
    const bool nosync = mode & 4;
    const bool stage = (mode & 1) &&
        (nosync || __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(k / ns));
    u32x4 *q = stage ? stg + ((uint64_t)(x * ns + slot) * 64 + s % 64) * wb16 : out + tile * wb16;
    for (uint32_t f = lane; f < wb16; f += 64) {
      if (!stage || (mode & 2)) __builtin_nontemporal_store(acc, q + f);
      else q[f] = acc;
    }
    if (!(mode & 1)) continue;
    const uint32_t tir = (uint32_t)min((uint64_t)64, ntiles - run * 64);
    if (nosync) {
      // the flusher rotates over the run's tiles (and so over the waves)
      if (s % 64 != (k * 37 + x * 11) % tir) continue;
    } else {
      // bit 3: no drain of the stores before the count (timing only)
      if (!(mode & 8)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint32_t prev = 0;
      if (lane == 0) prev = __hip_atomic_fetch_add(cnt + run, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      prev = __builtin_amdgcn_readfirstlane(prev);
      if (prev + 1 != tir) continue;
    }
    // last tile of the run: the staged tiles' bytes as one burst (a direct
    // tile is rewritten with garbage too: timing only)
    const u32x4 *src = stg + (uint64_t)(x * ns + slot) * 64 * wb16;
    u32x4 *dst = out + run * 64 * wb16;
    const uint32_t tot = tir * wb16;
    for (uint32_t f = lane; f < tot; f += 8 * 64) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __builtin_nontemporal_load(src + min(f + u * 64, tot - 1));
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (f + u * 64 < tot) __builtin_nontemporal_store(v[u], dst + f + u * 64);
    }
    if (nosync) continue;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_max(g, (uint32_t)(k / ns) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint32_t y = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (y == 0x9e3779b9u) sink[lane] = y;
}

extern "C" int rwxstage_run(const void *in, void *out, void *stg, uint32_t *cnt, uint32_t *gen,
                            uint64_t ntiles, uint32_t rb, uint32_t wb, uint32_t ns, int mode,
                            int grid, uint32_t *sink, void *stream) {
  const hipStream_t s = (hipStream_t)stream;
  const uint64_t nruns = (ntiles + 63) / 64;
  if (grid % 8 || ns == 0) return -22;
  if (hipMemsetAsync(cnt, 0, nruns * 4, s) != hipSuccess || hipMemsetAsync(gen, 0, 8 * ns * 4, s) != hipSuccess)
    return -5;
  hipLaunchKernelGGL(rw_xstage_kernel, dim3(grid), dim3(256), 0, s, (const u32x4 *)in, (u32x4 *)out,
                     (u32x4 *)stg, cnt, gen, ntiles, rb / 16, wb / 16, ns, mode, sink);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Which XCD each block of a grid runs on (HW_REG_XCC_ID), for the
// blockIdx % 8 grouping the staged probe assumes.
__global__ void xcc_census_kernel(uint32_t *out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg(0x1814);
}

extern "C" int xcc_census(uint32_t *out, int grid, void *stream) {
  hipLaunchKernelGGL(xcc_census_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
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
