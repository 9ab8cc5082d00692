// rx_bin.hip -- stable counting sort of frame indices by length group
// (rx_internal.h kGroupMaxLen), so that every wavefront sums frames of
// similar length and pptk_rx_batch_device_mixed can stream each group with
// a kernel shape sized for it (mixed-size batches, SURVEY.md 8(d) CMIX).
// Three small launches:
//   1. per-block histograms over a contiguous index range (bin-major matrix)
//   2. one-block exclusive scan of the matrix
//   3. per-block stable scatter of indices (wave ballots give the rank)
// Reads 2 x 2 bytes and writes 4 bytes per frame: <1 % of the frame bytes
// the transform itself reads.  The scan also leaves the group start table
// (kGroups + 1 entries) behind the counters for the group launches.
#include <algorithm>

#include "rx_internal.h"

namespace pptk {

namespace {

constexpr int NB = kGroups;   // length groups
constexpr int BT = 256;       // threads per block
constexpr int NWARP = BT / 64;

__device__ __forceinline__ int bin_of(uint32_t len, const BinBounds &bb) {
  int b = 0;
#pragma unroll
  for (int k = 0; k < NB - 1; ++k) b += len > bb.b[k];
  return b;
}

// per-thread counts in registers, summed over the wave, one LDS atomic per
// wave and group (an LDS atomic per frame on NB shared counters serialised
// the whole block: 60 us for 16 M lengths)
__global__ __launch_bounds__(BT) void bin_count(const uint16_t *len, uint64_t n,
                                                uint64_t per_block, uint32_t *counts,
                                                BinBounds bb) {
  __shared__ uint32_t h[NB];
  if (threadIdx.x < NB) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t lo = blockIdx.x * per_block;
  const uint64_t hi = min(lo + per_block, n);
  uint32_t c[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) c[k] = 0;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += BT) {
    const int b = bin_of(len[i], bb);
#pragma unroll
    for (int k = 0; k < NB; ++k) c[k] += b == k;
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    uint32_t v = c[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&h[k], v);
  }
  __syncthreads();
  if (threadIdx.x < NB) counts[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of m = NB * nblocks counters (bin-major), one block; then
// table[k] = start of bin k, table[NB] = total, table[NB + 1] = plan (1 =
// bin; adaptive: only when the batch mixes frames of the last group -- jumbo,
// > 1521 bytes -- with shorter ones, else the group whose launch runs the
// whole batch in batch order, rx_internal.h launch_bin)
__global__ __launch_bounds__(1024) void bin_scan(uint32_t *counts, uint32_t m, uint32_t *table,
                                                 uint32_t adaptive) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (m + 1023) / 1024;
  const uint32_t lo = threadIdx.x * per;
  const uint32_t hi = min(lo + per, m);
  uint32_t s = 0;
  for (uint32_t k = lo; k < hi; ++k) s += counts[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint32_t v = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;  // exclusive prefix of this thread's range
  for (uint32_t k = lo; k < hi; ++k) {
    const uint32_t c = counts[k];
    counts[k] = run;
    run += c;
  }
  __syncthreads();
  const uint32_t g = m / NB;
  if (threadIdx.x <= (unsigned)NB)
    table[threadIdx.x] = threadIdx.x < (unsigned)NB ? counts[threadIdx.x * g] : part[1023];
  if (threadIdx.x == 0) {   // the plan (rx_internal.h launch_bin)
    const uint32_t total = part[1023];
    const uint32_t last0 = counts[(NB - 1) * g];   // start of the last group
    uint32_t top = 0;                              // highest non-empty group
    for (int k = 0; k < NB; ++k) {
      const uint32_t lo = counts[k * g], hi = k + 1 < NB ? counts[(k + 1) * g] : total;
      if (hi > lo) top = (uint32_t)k;
    }
    const bool bin = !adaptive || (last0 < total && last0 > 0);
    table[NB + 1] = bin ? 1u : top << 8;
  }
}

// (bdesc: optionally also the frames' descriptors in binned order -- offset
// (or i * stride) and length at the same position as the index -- so the
// group launches read them sequentially instead of gathering them through
// perm: 10 bytes per frame written and later streamed, instead of two
// scattered 8- and 2-byte reads that each fetch a whole 64-byte sector)
__global__ __launch_bounds__(BT) void bin_scatter(const uint16_t *len, uint64_t n,
                                                  uint64_t per_block, const uint32_t *offs,
                                                  uint32_t *perm, BinDesc bdesc,
                                                  BinBounds bb, const uint32_t *plan) {
  __shared__ uint32_t cursor[NB];
  __shared__ uint32_t wcnt[NWARP][NB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (!(*plan & 1u)) {   // not binned: the identity order, no binned descriptors
    const uint64_t lo = blockIdx.x * per_block, hi = min(lo + per_block, n);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += BT) perm[i] = (uint32_t)i;
    return;
  }
  if (threadIdx.x < NB) cursor[threadIdx.x] = offs[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x];
  __syncthreads();
  const uint64_t lo = blockIdx.x * per_block;
  const uint64_t hi = min(lo + per_block, n);
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (uint64_t c0 = lo; c0 < hi; c0 += BT) {
    const uint64_t i = c0 + threadIdx.x;
    const bool ok = i < hi;
    const int b = ok ? bin_of(len[i], bb) : -1;
    uint32_t rank = 0;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const uint64_t mk = __ballot(b == k);
      if (b == k) rank = __popcll(mk & lt_mask);
      if (lane == 0) wcnt[wv][k] = __popcll(mk);
    }
    __syncthreads();
    if (ok) {
      uint32_t before = cursor[b];
      for (int w2 = 0; w2 < wv; ++w2) before += wcnt[w2][b];
      const uint32_t pos = before + rank;
      perm[pos] = (uint32_t)i;
      if (bdesc.boff) {
        bdesc.boff[pos] = bdesc.off ? bdesc.off[i] : i * bdesc.stride;
        bdesc.blen[pos] = len[i];
      }
    }
    __syncthreads();
    if (threadIdx.x < NB) {
      uint32_t add = 0;
      for (int w2 = 0; w2 < NWARP; ++w2) add += wcnt[w2][threadIdx.x];
      cursor[threadIdx.x] += add;
    }
    __syncthreads();
  }
}

}  // namespace

// scratch: counters (NB x grid), the group table (NB + 1) and the plan
// word, then (16-byte aligned) the binned descriptors: n u64 offsets and n
// u16 lengths
static size_t table_end(int grid) {
  return ((((size_t)NB * (size_t)grid + NB + 2) * sizeof(uint32_t)) + 15) & ~(size_t)15;
}

size_t bin_scratch_bytes(uint64_t n, int grid) {
  // + the permutation of a mixed call made without d_perm (16-byte aligned)
  return table_end(grid) + (size_t)n * (sizeof(uint64_t) + sizeof(uint16_t)) + 16 +
         (size_t)n * sizeof(uint32_t);
}

uint32_t *bin_perm(void *scratch, int grid, uint64_t n) {
  const uintptr_t p = (uintptr_t)((uint8_t *)scratch + table_end(grid) +
                                  (size_t)n * (sizeof(uint64_t) + sizeof(uint16_t)));
  return (uint32_t *)((p + 15) & ~(uintptr_t)15);
}

namespace {
__global__ __launch_bounds__(BT) void iota_kernel(uint32_t *perm, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * BT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BT)
    perm[i] = (uint32_t)i;
}
}  // namespace

hipError_t launch_iota(uint32_t *perm, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((n + BT - 1) / BT, 4096);
  hipLaunchKernelGGL(iota_kernel, dim3((unsigned)blocks), dim3(BT), 0, s, perm, n);
  return hipGetLastError();
}

uint64_t *bin_desc_off(void *scratch, int grid) {
  return (uint64_t *)((uint8_t *)scratch + table_end(grid));
}

uint16_t *bin_desc_len(void *scratch, int grid, uint64_t n) {
  return (uint16_t *)(bin_desc_off(scratch, grid) + n);
}

const uint32_t *bin_table(const void *scratch, int grid) {
  return (const uint32_t *)scratch + (size_t)NB * (size_t)grid;
}

hipError_t launch_bin(const uint16_t *len, uint64_t n, uint32_t *perm, void *scratch,
                      hipStream_t s, int grid, const BinDesc &bdesc,
                      const BinBounds &bounds, bool adaptive) {
  if (n == 0) return hipSuccess;
  const uint64_t per_block = ((n + grid - 1) / grid + BT - 1) / BT * BT;
  const int g = (int)((n + per_block - 1) / per_block);
  uint32_t *counts = (uint32_t *)scratch;
  hipLaunchKernelGGL(bin_count, dim3(g), dim3(BT), 0, s, len, n, per_block, counts, bounds);
  uint32_t *table = counts + (size_t)NB * grid;
  hipLaunchKernelGGL(bin_scan, dim3(1), dim3(1024), 0, s, counts, (uint32_t)(NB * g), table,
                     adaptive ? 1u : 0u);
  hipLaunchKernelGGL(bin_scatter, dim3(g), dim3(BT), 0, s, len, n, per_block,
                     (const uint32_t *)counts, perm, bdesc, bounds,
                     (const uint32_t *)table + NB + 1);
  return hipGetLastError();
}

}  // namespace pptk
