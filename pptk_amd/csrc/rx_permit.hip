// rx_permit.hip -- batched ip_permitted / ipv6_permitted token accounting
//  and the batch_timer_fn refill.
//
// The reference rate-limits per source prefix with one token counter per
// hash bucket: ip_permitted()/ipv6_permitted() (iphash/iphash.c:108-197)
// deny when the bucket's counter is 0 and otherwise decrement it and permit;
// the timer (batch_timer_fn, iphash/iphash.c:290-350) adds timer_add tokens
// to a range of buckets, saturating at initial_tokens.  Calling the check once
// per frame in frame order is the semantics to reproduce.  Per bucket b with
// T_b tokens before the batch, frame i (the k-th subject frame of bucket b in
// frame order, k from 0) is permitted iff k < T_b, and afterwards
// T_b' = T_b - min(T_b, count_b): a denied frame consumes nothing, and once
// the counter reaches 0 every later frame of that bucket is denied.  So the
// batch needs, for every frame, its rank among the earlier frames of its
// bucket -- a stable sort of frame indices by bucket:
//   1. keys: bucket of each subject frame (non-subjects get key hash_size
//      and sort last);
//   2. stable LSD radix sort of (key, index) pairs (rocPRIM), only the
//      log2(hash_size) + 1 key bits;
//   3. bucket bounds from the sorted keys: first[b] / end[b] = the sorted
//      positions where bucket b's run starts / ends (0 / 0 when absent);
//   4. verdict of frame i in bucket b: permitted iff it is among the first
//      T_b frames of b's run, i.e. i < lim[b] = (index of the T_b-th frame of
//      the run) + 1 -- everything when the run is no longer than T_b;
//   5. T_b -= min(T_b, end[b] - first[b]).
// (Counting with atomics instead -- device-scope atomics on a 2^16-entry
// array shared by all eight XCDs -- made step 1 take 0.72 of the batch's
// 1.37 ms; the bounds pass reads the 64 MB of sorted keys once.)
// Bucket values come from the records the rx kernel wrote (src_bucket, the
// reference's own hash of the masked source, iphash/iphash.c:157-162).
#include <algorithm>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "rx_internal.h"

namespace pptk {

namespace {

constexpr int PT = 256;

__device__ __forceinline__ void rec_fields(const PermitArgs &a, uint64_t i, uint32_t &flags,
                                           uint32_t &bucket) {
  if (a.recs32) {
    const uint8_t *r = (const uint8_t *)a.recs32 + i * 32u;
    flags = *(const uint16_t *)(r + 20);
    bucket = *(const uint32_t *)(r + 28);
  } else {
    const uint8_t *r = (const uint8_t *)a.recs + i * 64u;
    flags = *(const uint16_t *)(r + 54);
    bucket = *(const uint32_t *)(r + 56);
  }
}

__global__ __launch_bounds__(PT) void permit_keys(PermitArgs a, uint32_t *keys, uint32_t *vals) {
  const uint64_t i = (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (i >= a.n) return;
  uint32_t flags, bucket;
  rec_fields(a, i, flags, bucket);
  const bool v6 = flags & PPTK_RX_F_IPV6;
  bool subj = (flags & PPTK_RX_F_PARSED) && (a.family == 6 ? v6 : !v6);
  if (a.subject) subj = subj && a.subject[i];
  keys[i] = subj ? bucket : a.hash_size;
  vals[i] = (uint32_t)i;
  if (!subj) a.verdict[i] = 2;
}

// Run boundaries of the sorted keys: first[b] and end[b] of every bucket
// present (non-subject keys, == hash_size, sort last and are skipped).
__global__ __launch_bounds__(PT) void permit_bounds(PermitArgs a, const uint32_t *skeys,
                                                    uint32_t *first, uint32_t *end) {
  const uint64_t p = (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (p >= a.n) return;
  const uint32_t b = skeys[p];
  if (b >= a.hash_size) return;
  if (p == 0 || skeys[p - 1] != b) first[b] = (uint32_t)p;
  if (p + 1 == a.n || skeys[p + 1] != b) end[b] = (uint32_t)(p + 1);
}

// lim[b] per bucket: frames of b with index < lim[b] are permitted (the run
// is in frame order: the sort is stable).
__global__ __launch_bounds__(PT) void permit_limits(PermitArgs a, const uint32_t *svals,
                                                    const uint32_t *first, const uint32_t *end,
                                                    uint32_t *lim) {
  const uint64_t b = (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (b >= a.hash_size) return;
  const uint32_t t = a.tokens[b], c = end[b] - first[b];
  lim[b] = c <= t ? 0xffffffffu : t == 0 ? 0u : svals[first[b] + t - 1] + 1u;
}

// Verdicts in frame order (coalesced stores; the sorted-order pass this
// replaces scattered one byte per frame: 0.22 ms per 16 M frames).
__global__ __launch_bounds__(PT) void permit_verdicts(PermitArgs a, const uint32_t *keys,
                                                      const uint32_t *lim) {
  const uint64_t i = (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t b = keys[i];
  if (b >= a.hash_size) return;       // non-subject: verdict 2 already
  a.verdict[i] = (uint32_t)i < lim[b] ? 1 : 0;
}

__global__ __launch_bounds__(PT) void permit_consume(PermitArgs a, const uint32_t *first,
                                                     const uint32_t *end) {
  const uint64_t b = (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (b >= a.hash_size) return;
  const uint32_t t = a.tokens[b], c = end[b] - first[b];
  a.tokens[b] = t > c ? t - c : 0u;
}

// batch_timer_fn restated (iphash/iphash.c:290-350): the u32 sum saturates
// at initial_tokens exactly as the reference's `tokens = e->tokens +
// timer_add; if (tokens >= initial_tokens) tokens = initial_tokens;`
__global__ __launch_bounds__(PT) void tokens_refill(uint32_t *tokens, uint32_t start,
                                                    uint32_t end, uint32_t add,
                                                    uint32_t initial) {
  const uint64_t b = (uint64_t)start + (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (b >= end) return;
  const uint32_t t = tokens[b] + add;
  tokens[b] = t >= initial ? initial : t;
}

int key_bits(uint32_t hash_size) {
  int b = 0;
  while ((1ull << b) <= hash_size) ++b;   // keys 0 .. hash_size inclusive
  return b;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct PermitScratch {
  uint32_t *keys, *vals, *skeys, *svals, *first, *end, *lim;
  void *tmp;
  size_t tmp_bytes, total;
};

hipError_t layout(uint64_t n, uint32_t hash_size, void *base, PermitScratch &s) {
  size_t sort_tmp = 0;
  hipError_t e = rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t *)nullptr,
                                           (uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (uint32_t *)nullptr, (size_t)n, 0,
                                           (unsigned)key_bits(hash_size));
  if (e != hipSuccess) return e;
  uint8_t *p = (uint8_t *)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    uint8_t *q = p ? p + off : nullptr;
    off += align256(bytes);
    return q;
  };
  s.keys = (uint32_t *)take(n * 4);
  s.vals = (uint32_t *)take(n * 4);
  s.skeys = (uint32_t *)take(n * 4);
  s.svals = (uint32_t *)take(n * 4);
  s.first = (uint32_t *)take((size_t)hash_size * 8);   // first[hash_size], then end[]
  s.end = s.first ? s.first + hash_size : nullptr;
  s.lim = (uint32_t *)take((size_t)hash_size * 4);
  s.tmp_bytes = sort_tmp;
  s.tmp = take(s.tmp_bytes);
  s.total = off;
  return hipSuccess;
}

unsigned blocks(uint64_t n) { return (unsigned)((n + PT - 1) / PT); }

}  // namespace

size_t permit_scratch_bytes(uint64_t n, uint32_t hash_size) {
  PermitScratch s;
  if (layout(n, hash_size, nullptr, s) != hipSuccess) return 0;
  return s.total;
}

hipError_t launch_permit(const PermitArgs &a, void *scratch, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  PermitScratch s;
  hipError_t e = layout(a.n, a.hash_size, scratch, s);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(s.first, 0, (size_t)a.hash_size * 8, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(permit_keys, dim3(blocks(a.n)), dim3(PT), 0, st, a, s.keys, s.vals);
  size_t tb = s.tmp_bytes;
  e = rocprim::radix_sort_pairs(s.tmp, tb, s.keys, s.skeys, s.vals, s.svals, (size_t)a.n, 0,
                                (unsigned)key_bits(a.hash_size), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(permit_bounds, dim3(blocks(a.n)), dim3(PT), 0, st, a, s.skeys, s.first,
                     s.end);
  hipLaunchKernelGGL(permit_limits, dim3(blocks(a.hash_size)), dim3(PT), 0, st, a, s.svals,
                     s.first, s.end, s.lim);
  hipLaunchKernelGGL(permit_verdicts, dim3(blocks(a.n)), dim3(PT), 0, st, a, s.keys, s.lim);
  hipLaunchKernelGGL(permit_consume, dim3(blocks(a.hash_size)), dim3(PT), 0, st, a, s.first,
                     s.end);
  return hipGetLastError();
}

hipError_t launch_refill(uint32_t *tokens, uint32_t start, uint32_t end, uint32_t add,
                         uint32_t initial, hipStream_t st) {
  if (end <= start) return hipSuccess;
  hipLaunchKernelGGL(tokens_refill, dim3(blocks(end - start)), dim3(PT), 0, st, tokens, start,
                     end, add, initial);
  return hipGetLastError();
}

}  // namespace pptk
