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
// reference's own hash of the masked source, iphash/iphash.c:157-162), or
// from the dense per-frame key array it can write beside them
// (pptk_rx_dev_batch.d_key: 4 bytes per frame instead of a 16-byte slice of
// each 64-byte record, whose read costs the DRAM the whole 64-byte burst).
//
// That sort is the fallback (hash_size > 2^16).  The main path needs no sort,
// because the verdict of a frame only depends on whether its rank passes
// T_b, and that is decided per BLOCK of frames for all but one block per
// bucket:
//   H. histogram: block c of HB = 65532 consecutive frames counts its
//      subject frames per bucket in LDS (u16 pairs, 128 KB for 2^16
//      buckets) and writes the row bh[c][*]; it also writes each frame's
//      subject key (bucket, or ~0) densely for the later passes;
//   S. per bucket, down the column: count_b, and the block c* holding the
//      T_b-th frame and the rank need_b of that frame inside c*; lim[b] =
//      "all" when count_b <= T_b, 0 when T_b == 0, else pending; T_b -=
//      min(T_b, count_b);
//   R. only blocks that are some bucket's c* (none when no bucket runs out
//      of tokens): list the block's frames of such buckets in frame order
//      and walk the list (one wave ranks them with ballots, LDS counters
//      per bucket): lim[b] = index of the need_b-th frame of b + 1;
//   V. verdicts in frame order from the dense keys and lim[].
// 16 M frames, 2^16 buckets: the histogram table is 32 MB, the passes read
// the keys twice -- no 64 MB x (2 passes x 3 arrays) radix sort.
#include <errno.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <unordered_map>
#include <utility>

#include <hip/hip_ext.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "rx_internal.h"

namespace pptk {

namespace {

constexpr int PT = 256;

// flags and src_bucket of record i: one 16-byte load of the record's
// bytes 48..63 (64-byte records: flags at 54, src_bucket at 56) or 16..31
// (compact: flags at 20, src_bucket at 28) -- the 32-byte sector both fields
// share, in one instruction instead of two narrow strided loads
__device__ __forceinline__ void rec_fields(const PermitArgs &a, uint64_t i, uint32_t &flags,
                                           uint32_t &bucket) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  if (a.recs32) {
    const u32x4 q = __builtin_nontemporal_load((const u32x4 *)((const uint8_t *)a.recs32 + i * 32u) + 1);
    flags = q.y & 0xffffu;
    bucket = q.w;
  } else {
    const u32x4 q = __builtin_nontemporal_load((const u32x4 *)((const uint8_t *)a.recs + i * 64u) + 3);
    flags = q.y >> 16;
    bucket = q.z;
  }
}

// The bucket of frame i if it is a subject of this call, else NOSUBJ:
// from the record, or from the rx kernel's dense key (bucket of a parsed
// IPv4 frame; bucket | 0x80000000 of a parsed IPv6 frame; ~0 otherwise).
constexpr uint32_t NOSUBJ = 0xffffffffu;

__device__ __forceinline__ uint32_t subject_key(const PermitArgs &a, uint64_t i) {
  bool subj;
  uint32_t bucket;
  if (a.keys_in) {
    const uint32_t k = a.keys_in[i];
    subj = k != NOSUBJ && ((k >> 31) == (a.family == 6 ? 1u : 0u));
    bucket = k & 0x7fffffffu;
  } else {
    uint32_t flags;
    rec_fields(a, i, flags, bucket);
    const bool v6 = flags & PPTK_RX_F_IPV6;
    subj = (flags & PPTK_RX_F_PARSED) && (a.family == 6 ? v6 : !v6);
  }
  if (a.subject) subj = subj && a.subject[i];
  // a bucket outside the token array is not a subject (caller-made keys;
  // the rx kernel's buckets are < iphash_size by construction)
  return subj && bucket < a.hash_size ? bucket : NOSUBJ;
}

// (sort fallback: non-subjects get key hash_size, sorted last)
__global__ __launch_bounds__(PT) void permit_keys(PermitArgs a, uint32_t *keys) {
  const uint64_t i = (uint64_t)blockIdx.x * PT + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t k = subject_key(a, i);
  keys[i] = k == NOSUBJ ? a.hash_size : k;   // (verdict 2, written by permit_verdicts)
}

// ---- the sort-free path (hash_size <= 2^16) ------------------------------
constexpr uint32_t HB = 65532;       // frames per histogram block (u16 counts; 4 | HB)
constexpr int HT = 1024;             // threads of the histogram / resolve / verdict blocks
constexpr uint32_t HMAX = 1u << 16;  // largest hash_size of the sort-free path
constexpr uint32_t NOBLK = 0xffffffffu;
// code[b] (u16), what the verdict of a frame of bucket b depends on:
constexpr uint16_t CODE_ALL = 0xffff;    // every frame of b permitted
constexpr uint16_t CODE_NONE = 0xfffe;   // none (T_b == 0)
                                         // else c*: permitted below block c*,
                                         // denied above, lim[b] inside it
constexpr uint32_t MAX_BLOCKS = 0xfffd;  // block ids below CODE_NONE

__device__ __forceinline__ uint32_t hwords(uint32_t hash_size) { return (hash_size + 1) / 2; }

// Subject key of frame i for the passes after the histogram: straight from
// the caller's dense keys, or from the histogram pass's copy (records).
__device__ __forceinline__ uint32_t key_at(const PermitArgs &a, const uint32_t *ckey, uint64_t i) {
  return a.keys_in ? subject_key(a, i) : ckey[i];
}

__device__ __forceinline__ uint32_t filter_key(const PermitArgs &a, uint32_t k) {
  return k != NOSUBJ && ((k >> 31) == (a.family == 6 ? 1u : 0u)) && (k & 0x7fffffffu) < a.hash_size
             ? (k & 0x7fffffffu)
             : NOSUBJ;
}

// Subject keys of frames i .. i + 3 (i + 4 <= n): one 16-byte load when the
// key array allows it (vec), else four.
__device__ __forceinline__ void keys4(const PermitArgs &a, const uint32_t *ckey, uint64_t i,
                                      bool vec, uint32_t k[4]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  if (vec) {
    const u32x4 q = *(const u32x4 *)((a.keys_in ? a.keys_in : ckey) + i);
    k[0] = q.x;
    k[1] = q.y;
    k[2] = q.z;
    k[3] = q.w;
    if (a.keys_in) {
#pragma unroll
      for (int u = 0; u < 4; ++u) k[u] = filter_key(a, k[u]);
      if (a.subject) {
#pragma unroll
        for (int u = 0; u < 4; ++u) k[u] = a.subject[i + u] ? k[u] : NOSUBJ;
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = key_at(a, ckey, i + u);
  }
}

// H: per-block histogram (u16 pairs in LDS, one word = buckets 2w, 2w + 1);
// from records it also writes each frame's subject key densely (ckey), so
// the later passes read 4 bytes per frame instead of the record again
__global__ __launch_bounds__(HT) void permit_hist(PermitArgs a, uint32_t *ckey, uint32_t *bh,
                                                  uint32_t *blk_flag) {
  __shared__ uint32_t h[HMAX / 2];
  const uint32_t words = hwords(a.hash_size);
  for (uint32_t w = threadIdx.x; w < words; w += HT) h[w] = 0;
  if (threadIdx.x == 0) blk_flag[blockIdx.x] = 0;
  __syncthreads();
  const uint64_t lo = (uint64_t)blockIdx.x * HB;
  const uint64_t hi = min(lo + HB, a.n);
  // HU frames per thread and step, their loads issued together (frame
  // base + u * HT + tid: each load instruction reads consecutive frames; a
  // step of four had left the pass waiting on load latency, 37 us)
  constexpr int HU = 16;
  for (uint64_t b0 = lo; b0 < hi; b0 += HU * HT) {
    uint32_t k[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const uint64_t i = b0 + (uint64_t)(u * HT) + threadIdx.x;
      k[u] = i < hi ? subject_key(a, i) : NOSUBJ;
    }
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const uint64_t i = b0 + (uint64_t)(u * HT) + threadIdx.x;
      if (!a.keys_in && i < hi) ckey[i] = k[u];
      if (k[u] != NOSUBJ) atomicAdd(&h[k[u] >> 1], 1u << ((k[u] & 1u) * 16u));
    }
  }
  __syncthreads();
  uint32_t *row = bh + (uint64_t)blockIdx.x * words;
  for (uint32_t w = threadIdx.x; w < words; w += HT) row[w] = h[w];
}

// S: one thread per bucket, down its column of the histogram table
__global__ __launch_bounds__(PT) void permit_scan(PermitArgs a, const uint32_t *bh, uint32_t nblk,
                                                  uint32_t *lim, uint32_t *need, uint16_t *code,
                                                  uint32_t *blk_flag) {
  const uint32_t b = blockIdx.x * PT + threadIdx.x;
  if (b >= a.hash_size) return;
  const uint16_t *col = (const uint16_t *)bh + b;
  const uint64_t pitch = 2ull * hwords(a.hash_size);   // u16 entries per row
  const uint32_t t = a.tokens[b];
  uint32_t acc = 0, cstar = NOBLK, prior = 0;
  uint32_t c = 0;
  for (; c + 16 <= nblk; c += 16) {
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = col[(uint64_t)(c + u) * pitch];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (cstar == NOBLK && acc + v[u] >= t) {
        cstar = c + u;
        prior = acc;
      }
      acc += v[u];
    }
  }
  for (; c < nblk; ++c) {
    const uint32_t v = col[(uint64_t)c * pitch];
    if (cstar == NOBLK && acc + v >= t) {
      cstar = c;
      prior = acc;
    }
    acc += v;
  }
  uint16_t cd = CODE_ALL;
  if (acc > t) {
    if (t == 0) {
      cd = CODE_NONE;
      lim[b] = 0;
    } else {   // the T_b-th frame lies in block cstar: resolved by permit_resolve
      cd = (uint16_t)cstar;
      need[b] = t - prior;
      blk_flag[cstar] = 1;
    }
  }
  code[b] = cd;
  a.tokens[b] = t > acc ? t - acc : 0u;
}

// Stage code[0, hash_size) into LDS (as 32-bit pairs).
__device__ __forceinline__ void stage_code(const PermitArgs &a, const uint16_t *code, uint16_t *tab) {
  const uint32_t words = hwords(a.hash_size);
  const uint32_t *src = (const uint32_t *)code;
  uint32_t *dst = (uint32_t *)tab;
  for (uint32_t w = threadIdx.x; w < words; w += HT) dst[w] = src[w];
}

// R: the blocks holding some bucket's T_b-th frame.  code[] is staged in
// LDS.  A: every thread takes 64 consecutive frames of the block and marks
// its candidates (frames of a bucket b with code[b] == this block); their
// buckets' LDS entries then become rem[b] = need_b; after a block scan of
// the counts the candidates are appended in frame order to the block's
// slice of a list (frame offset in the block << 16 | bucket).  B: every
// wave walks the list, 64 candidates a step, acting on its sixteenth of the
// buckets: per distinct bucket of the step one ballot; the lane at rank
// rem[b] sets lim[b]; rem[b] drops by the step's count (0: resolved).  Only
// the candidates are walked in order, and the walk waits on nothing but
// the list.
constexpr int RPER = 64;   // frames per thread in pass A (HT * RPER >= HB)
static_assert(HT * RPER >= (int)HB, "one pass over a histogram block");

__global__ __launch_bounds__(HT) void permit_resolve(PermitArgs a, const uint32_t *ckey,
                                                     const uint32_t *need, const uint16_t *code,
                                                     const uint32_t *blk_flag, uint32_t *clist,
                                                     uint32_t *lim) {
  if (blk_flag[blockIdx.x] == 0) return;
  __shared__ uint16_t tab[HMAX];   // code[b], then rem[b] for this block's buckets
  __shared__ uint32_t wsum[HT / 64];
  stage_code(a, code, tab);
  const uint32_t c = blockIdx.x;
  const uint64_t lo = (uint64_t)c * HB;
  const uint64_t hi = min(lo + HB, a.n);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t f0 = lo + (uint64_t)threadIdx.x * RPER;
  __syncthreads();
  // A1: this thread's candidates (bit j: frame f0 + j), 16 frames per round
  uint64_t mask = 0;
#pragma unroll
  for (int j0 = 0; j0 < RPER; j0 += 16) {
    uint32_t k[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint64_t i = f0 + (uint64_t)(j0 + u);
      k[u] = i < hi ? key_at(a, ckey, i) : NOSUBJ;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (k[u] != NOSUBJ && tab[k[u]] == (uint16_t)c) mask |= 1ull << (j0 + u);
  }
  __syncthreads();   // every candidate test has read tab[] as code
  for (uint64_t m = mask; m; m &= m - 1) {   // code -> rem (same value from every candidate)
    const uint32_t k = key_at(a, ckey, f0 + (uint64_t)(__ffsll((unsigned long long)m) - 1));
    tab[k] = (uint16_t)need[k];
  }
  // A2: block exclusive scan of the counts
  const uint32_t cnt = (uint32_t)__popcll(mask);
  uint32_t inc = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(inc, d);
    if (lane >= d) inc += v;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < HT / 64; ++w) {
    const uint32_t v = wsum[w];
    base += w < wv ? v : 0u;
    total += v;
  }
  base += inc - cnt;
  // A3: append in frame order
  uint32_t *list = clist + lo;
  for (uint64_t m = mask; m; m &= m - 1) {
    const int j = __ffsll((unsigned long long)m) - 1;
    const uint32_t k = key_at(a, ckey, f0 + (uint64_t)j);
    list[base++] = (uint32_t)(threadIdx.x * RPER + j) << 16 | k;
  }
  __syncthreads();   // (the list and rem[] are complete for the block)
  // B: the ordered walk; wave w takes the buckets b with b % 16 == w (their
  // candidates keep their order), so the per-bucket steps run 16 waves wide
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (uint32_t s0 = 0; s0 < total; s0 += 64) {
    const uint32_t e = s0 + (uint32_t)lane < total ? list[s0 + lane] : NOSUBJ;
    const uint32_t k = e & 0xffffu;
    const bool on = e != NOSUBJ && (k & (HT / 64 - 1)) == (uint32_t)wv;
    uint64_t todo = __ballot(on);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const uint32_t b = __shfl(k, leader);
      const uint64_t m = __ballot(on && k == b);
      const uint32_t r0 = tab[b];
      const uint32_t pc = (uint32_t)__popcll(m);
      if (r0 != 0) {
        if (on && k == b && (uint32_t)__popcll(m & lt) + 1u == r0)
          lim[b] = (uint32_t)(lo + (e >> 16)) + 1u;
        if (lane == leader) tab[b] = (uint16_t)(r0 > pc ? r0 - pc : 0u);
      }
      todo &= ~m;
    }
  }
}

// V: verdicts in frame order, code[] staged in LDS per block (a persistent
// grid: the 128 KB table is read once per CU, not once per 1024 frames):
// key NOSUBJ -> 2; code ALL -> 1; NONE -> 0; else by the frame's block
// against c*, and inside c* against lim[b] (the one global read left, only
// for frames of a bucket's boundary block).  Four frames per thread and
// step: one 4-byte verdict store when the verdict array's alignment allows.
__device__ __forceinline__ uint32_t verdict_code(const PermitArgs &a, const uint16_t *tab,
                                                 const uint32_t *lim, uint64_t i, uint32_t k) {
  if (k == NOSUBJ) return 2u;
  const uint32_t cd = tab[k];
  if (cd == CODE_ALL) return 1u;
  if (cd == CODE_NONE) return 0u;
  const uint32_t blk = (uint32_t)(i / HB);
  if (blk != cd) return blk < cd ? 1u : 0u;
  return (uint32_t)i < lim[k] ? 1u : 0u;
}

__global__ __launch_bounds__(HT) void permit_verdicts_tab(PermitArgs a, const uint32_t *ckey,
                                                          const uint16_t *code,
                                                          const uint32_t *lim) {
  __shared__ uint16_t tab[HMAX];
  stage_code(a, code, tab);
  __syncthreads();
  const bool aligned = ((uintptr_t)a.verdict & 3u) == 0;
  const bool kvec = ((uintptr_t)(a.keys_in ? a.keys_in : ckey) & 15u) == 0;
  // VU groups of four frames per thread and step, their key loads issued
  // together (a step of one group waited on load latency: 22 us)
  constexpr int VU = 4;
  const uint64_t stride = 4 * (uint64_t)gridDim.x * HT;
  for (uint64_t i0 = 4 * ((uint64_t)blockIdx.x * HT + threadIdx.x); i0 < a.n; i0 += VU * stride) {
    uint32_t k[VU][4];
#pragma unroll
    for (int g = 0; g < VU; ++g) {
      const uint64_t i = i0 + (uint64_t)g * stride;
      if (i + 4 <= a.n) {
        keys4(a, ckey, i, kvec, k[g]);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) k[g][u] = i + u < a.n ? key_at(a, ckey, i + u) : NOSUBJ;
      }
    }
#pragma unroll
    for (int g = 0; g < VU; ++g) {
      const uint64_t i = i0 + (uint64_t)g * stride;
      if (i >= a.n) break;
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = verdict_code(a, tab, lim, i + u, k[g][u]);
      if (aligned && i + 4 <= a.n) {
        *(uint32_t *)(a.verdict + i) = v[0] | v[1] << 8 | v[2] << 16 | v[3] << 24;
      } else {
        for (int u = 0; u < 4 && i + u < a.n; ++u) a.verdict[i + u] = (uint8_t)v[u];
      }
    }
  }
}

// ---- the fused path: one persistent launch, every key read once ----------
//
// The four passes above read the keys twice and write + read a 32 MB table
// of u16 per-block bucket counts: 221 MB of HBM traffic for 84 MB of
// algorithmic bytes (16 M dense keys in, 16 M verdicts out), 80 us.  Here
// one workgroup per CU owns a contiguous segment of up to 65 536 frames and
// keeps its keys in registers (64 per thread) through three phases split by
// two grid barriers:
//   1. LDS histogram of the segment's subject keys; the row written to the
//      table as u8 counts (saturated at 255; exact counts of saturated
//      buckets, at most 257 per segment, in a per-segment overflow list);
//   2. per bucket, down its column (the table read once): total, the segment
//      c* holding the T_b-th frame and that frame's rank need_b inside c*;
//      code[b] (all / none / c*) and the new token count;
//   3. only if some bucket ran out (else the speculative verdicts, written
//      at the start of phase 2 as if every subject were permitted, stand and
//      the launch ends): the code table staged in LDS; a segment that is
//      some bucket's c* ranks, round by round in frame order, its frames of
//      such buckets (ballots, as permit_resolve; buckets whose T_b-th frame
//      is their last one here need no ranking) -- the keys are its own
//      registers, no second read -- and every thread rewrites the verdict
//      words that differ.
// HBM: keys once (67 MB), the u8 table twice (2 x 16.8 MB), verdicts (17
// MB): ~118 MB, 1.4 x the algorithmic bytes.  The table and the phase-2
// outputs are handed between workgroups with write-through (sc1) stores and
// sc1 loads; the grid barriers are per-workgroup arrival words holding the
// launch's nonce (no memset before a launch: a stale word never matches)
// (MI355X_MICROARCH.md "inter-workgroup visibility", the
// one-workgroup-per-CU row): no L2 write-back fences.  Co-residency: the
// grid is at most one workgroup per CU and each needs > 80 KB of LDS, so no
// CU holds two; a workgroup not yet resident (a CU busy with another
// stream's kernel) only delays the others.  Two fused launches on two
// streams could each hold part of the CUs and wait for each other's; the
// host orders every fused launch of a device behind the previous one
// (launch_permit), so within a process that cannot happen.  Every spin is
// still bounded (FUSED_SPIN_TICKS, e.g. another process's kernels holding
// the CUs): a workgroup whose barrier times out ABORTS the launch -- it
// publishes an abort word that every other workgroup's barrier also stops
// at -- and marks the status word (PermitFused::out[1], read by
// pptk_rx_permit_status).  The token counts are written only after the
// second barrier has passed, so an aborted launch leaves the tokens as they
// were (the caller repeats the call), never half-updated.
constexpr int FT = 1024;                  // threads per workgroup
constexpr int FKV = 16;                   // 16-byte key loads per thread (64 frames)
constexpr int FKB = 4;                    // of them per batch (two batches in flight)
constexpr uint32_t FSEG = FT * 4 * FKV;   // frames per segment at most (65 536)
constexpr uint32_t FOVF = FSEG / 255 + 1; // saturated buckets per segment at most
constexpr int FSL = 16;                   // phase 2: row slices per word
constexpr uint32_t FMAXBLK = 256;         // segments at most (rows of phase 2: 16 x 16)
constexpr uint32_t FHASH_PASS = 2048;     // phase 3: candidates per hash-table pass at most
constexpr uint32_t FHASH_MAXP = 32;       // hash-table passes at most
constexpr uint32_t FHASH_K = 64;          // frames of one ranked bucket at most, hash path
constexpr uint64_t FUSED_SPIN_TICKS = 200000000ull;   // 2 s of the 100 MHz clock
#ifndef PPTK_PERMIT_CODE_REPL
#define PPTK_PERMIT_CODE_REPL 1
#endif
constexpr uint32_t FCREPL = PPTK_PERMIT_CODE_REPL;   // copies of the code array (A/B)

struct PermitFused {
  uint32_t *table;   // nblk rows x nwords u32 (4 u8 counts each)
  uint32_t *ovf;     // nblk x FOVF (bucket, count) pairs
  uint32_t *novf;    // nblk
  uint32_t *need;    // hash_size
  uint32_t *code;    // ceil(hash_size / 2) words of u16 pairs
  uint32_t *ntok;    // hash_size: the new token counts, until the commit
  uint64_t *arrive;  // FMAXBLK: workgroup c's barrier generation (nonce + k, + 1: its flag)
  uint64_t *out;     // [0] decision (nonce | 2 committed, nonce | 4 aborted: fused_decide);
                     // [1] = nonce | 1: the launch aborted (status)
  uint32_t *stamps;  // FSTAMPS x FMAXBLK phase timestamps (tools/permit_run.py)
  uint64_t nonce;    // this launch's, low three bits clear (never 0)
  uint64_t spin_ticks;   // a barrier's bound (100 MHz ticks)
  uint64_t stall_ticks;  // test builds: hold the last workgroup this long ...
  uint32_t stall_at;     // ... before barrier stall_at (1, 2; 0 = never)
  uint32_t nblk, seg, nwords;
};
constexpr int FSTAMPS = 12;

__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The launch's decision word f.out[0]: nonce | 2 once barrier 2 (the commit
// point) has passed, nonce | 4 once the launch aborted; any other value (a
// word an earlier launch left) is undecided.  Set once per launch by compare-
// and-swap, so every workgroup acts on the same outcome: a workgroup that
// saw every arrival at barrier 2 and one whose wait ran out cannot both win.
// Returns the decided value (ours, or the one another workgroup set first).
// (Each failed swap means another workgroup wrote this launch's decision, so
// the loop ends after at most one retry.)
__device__ __forceinline__ uint64_t fused_decide(uint64_t *out, uint64_t nonce, uint64_t what) {
  uint64_t x = ld_sc1(out);
  for (;;) {
    if ((x & ~7ull) == nonce) return x;
    uint64_t seen = x;
    if (__hip_atomic_compare_exchange_strong(out, &seen, nonce | what, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return nonce | what;
    x = seen;
  }
}

// Grid barrier k (1, 2) of the launch with nonce N: every wave's stores
// complete, workgroup c publishes N + k (+ 1 with `flag`, at k = 2) in
// arrive[c], and wave 0 polls all nblk words (sc1, bounded) until each holds
// N + k or later.  Nothing needs zeroing between launches: a word left by
// another launch (or garbage) never matches this launch's nonce, so there is
// no memset before each launch.  Returns 1 if some workgroup raised its
// flag -- phase 2's "a bucket ran out", carried by the arrival words rather
// than by one word every workgroup would store to (write-through stores to
// one address are served one after another: 10 us for 256 of them) -- else
// 0; or -1: the launch aborted.
// Outcome through the decision word (fused_decide): a workgroup whose wait
// exceeds f.spin_ticks proposes "aborted"; at barrier 2 a workgroup that saw
// every arrival proposes "passed".  Whichever came first holds for all: a
// workgroup that saw "aborted" returns -1 (the status word set), one whose
// own wait ran out after the commit was decided keeps polling (every arrival
// is there) and commits with the others.  Barrier 1 never decides "passed"
// (nothing is committed there), so an abort at barrier 1 always wins, and a
// workgroup that was not resident yet sees it when it arrives.
__device__ __forceinline__ int fused_barrier(const PermitFused &f, uint32_t c, uint64_t k,
                                             bool flag = false) {
  __shared__ int res;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0) st_sc1(f.arrive + c, f.nonce + k + (flag ? 1u : 0u));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool passed = false;   // barrier 2's commit decided (by any workgroup)
    int r = 0;
    for (;;) {
      const uint64_t d = ld_sc1(f.out);
      const bool ours = (d & ~7ull) == f.nonce;
      if (ours && (d & 4ull)) {
        r = -1;
        break;
      }
      passed = passed || (ours && (d & 2ull));
      bool ok = true, fl = false;
      for (uint32_t i = threadIdx.x; i < f.nblk; i += 64) {
        const uint64_t x = ld_sc1(f.arrive + i);
        const bool mine = (x & ~7ull) == f.nonce;
        ok = ok && mine && (x & 3ull) >= k;
        fl = fl || (mine && (x & 3ull) == 3ull);
      }
      if (__all(ok)) {
        uint64_t dec = f.nonce | 2u;
        if (k == 2 && !passed) {
          if (threadIdx.x == 0) dec = fused_decide(f.out, f.nonce, 2u);
          dec = __shfl(dec, 0);
        }
        r = (dec & 4ull) ? -1 : (__any(fl) ? 1 : 0);
        break;
      }
      if (!passed && __builtin_amdgcn_s_memrealtime() - t0 > f.spin_ticks) {
        uint64_t dec = 0;
        if (threadIdx.x == 0) dec = fused_decide(f.out, f.nonce, 4u);
        dec = __shfl(dec, 0);
        if (dec & 4ull) {
          r = -1;
          break;
        }
        passed = true;   // the commit won: wait for the arrivals it saw
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) {
      if (r < 0) st_sc1(f.out + 1, f.nonce | 1u);
      res = r;
    }
  }
  __syncthreads();
  return res;
}

// Test builds (PPTK_RX_TEST_HOOKS) hold the last workgroup before barrier
// f.stall_at for f.stall_ticks, so that the others' barrier times out (the
// fault-injection test of the abort path); a product build never sets it.
__device__ __forceinline__ void fused_stall(const PermitFused &f, uint32_t c, uint32_t k) {
  if (f.stall_ticks == 0 || f.stall_at != k || c + 1 != f.nblk) return;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < f.stall_ticks) __builtin_amdgcn_s_sleep(127);
  }
  __syncthreads();
}

// Subject keys of frames i .. i + 3 of the segment [.., hi).
template <bool KEYS>
__device__ __forceinline__ void fused_keys4(const PermitArgs &a, uint64_t i, uint64_t hi,
                                            bool vec, uint32_t k[4]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  if (KEYS && vec && i + 4 <= hi) {
    const u32x4 q = *(const u32x4 *)(a.keys_in + i);
    k[0] = filter_key(a, q.x);
    k[1] = filter_key(a, q.y);
    k[2] = filter_key(a, q.z);
    k[3] = filter_key(a, q.w);
    if (a.subject) {
#pragma unroll
      for (int u = 0; u < 4; ++u) k[u] = a.subject[i + u] ? k[u] : NOSUBJ;
    }
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = i + u < hi ? subject_key(a, i + u) : NOSUBJ;
  }
}

// Exact count of bucket b in segment r whose u8 table entry saturated.
__device__ __forceinline__ uint32_t fused_ovf(const PermitFused &f, uint32_t r, uint32_t b) {
  const uint32_t m = ld_sc1(f.novf + r);
  const uint32_t *e = f.ovf + (uint64_t)r * FOVF * 2;
  for (uint32_t j = 0; j < m; ++j)
    if (ld_sc1(e + 2 * j) == b) return ld_sc1(e + 2 * j + 1);
  return 255u;   // (unreachable: a saturated entry is always listed)
}

// KEYS: the dense keys (pptk_rx_permit_keys_device), else records.
template <bool KEYS>
__global__ __launch_bounds__(FT) void permit_fused(PermitArgs a, PermitFused f) {
  __shared__ uint32_t tab[HMAX / 2];    // phase 1 histogram (u16 pairs); phase 3 code table
  __shared__ uint32_t rbit[HMAX / 32];  // phase 3: buckets whose c* is this segment
  __shared__ __attribute__((aligned(16))) uint32_t list[FT * 4];   // phase 2 partial sums; phase 3 candidate list
  __shared__ uint32_t wsum[FT / 64 + 1];
  // phase 2: c* found and tokens per (word lane, bucket)
  __shared__ __attribute__((aligned(16))) uint32_t p23[512];
  __shared__ uint32_t out_l;   // phase 2: some bucket of this workgroup ran out
  const uint32_t c = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const uint64_t lo = (uint64_t)c * f.seg;
  const uint64_t hi = min(lo + f.seg, a.n);
  const uint32_t words = hwords(a.hash_size);   // u16-pair words of the histogram / code table
  const bool vec = ((uintptr_t)a.keys_in & 15u) == 0;
  // phase timestamps of every workgroup (100 MHz clock): read by
  // tools/permit_run.py --stamps, nothing else
#define FSTAMP(k)                                                                          \
  do {                                                                                     \
    if (tid == 0) f.stamps[(k) * FMAXBLK + c] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
  FSTAMP(0);

  // ---- phase 1: keys into registers, LDS histogram, the u8 row ------------
  auto clear_tab = [&]() {
    for (uint32_t w = tid; w < words; w += FT) tab[w] = 0;
    __syncthreads();
  };
  // the 64 keys, two 16-bit buckets per register, and which are subjects
  uint32_t kp[FKV * 2];
  uint64_t sm = 0;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // Whole, aligned segment of dense keys: straight-line 16-byte loads, eight
  // rounds in flight (a load under a per-round branch was waited for before
  // the next one issued: 16 serial round trips, 19 us); rounds past the
  // segment re-read round 0 and are dropped; no subject array reads the keys
  // again and ORs in "subject".
  const bool fast = KEYS && vec && hi == lo + f.seg &&
                    (!a.subject || ((uintptr_t)a.subject & 3u) == 0);
  if (fast) {
    const uint32_t nv = f.seg / (FT * 4);
    const bool subj = a.subject != nullptr;
    // Batches of FKB rounds, double-buffered: batch h + 1 is in flight while
    // batch h is counted (2 FKB loads outstanding per thread at most)
    u32x4 qa[FKB], qb[FKB];
    uint32_t sa[FKB], sbb[FKB];
    auto load = [&](u32x4 (&q)[FKB], uint32_t (&sw)[FKB], int h) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < FKB; ++k) {
        const int v = h * FKB + k;
        const uint64_t i = lo + (uint64_t)((uint32_t)v < nv ? v : 0) * FT * 4 + 4 * tid;
        q[k] = *(const u32x4 *)(a.keys_in + i);
        sw[k] = subj ? *(const uint32_t *)(a.subject + i) : 0x01010101u;
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    auto count = [&](const u32x4 (&q)[FKB], const uint32_t (&sw)[FKB], int h)
        __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < FKB; ++k) {
        const int v = h * FKB + k;
        const bool live = (uint32_t)v < nv;
        uint32_t kk[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          kk[u] = live && ((sw[k] >> (8 * u)) & 0xffu) ? filter_key(a, kk[u]) : NOSUBJ;
          if (kk[u] != NOSUBJ) {
            atomicAdd(&tab[kk[u] >> 1], 1u << ((kk[u] & 1u) * 16u));
            sm |= 1ull << (v * 4 + u);
          }
        }
        kp[2 * v] = (kk[0] & 0xffffu) | kk[1] << 16;
        kp[2 * v + 1] = (kk[2] & 0xffffu) | kk[3] << 16;
        asm volatile("" : "+v"(kp[2 * v]), "+v"(kp[2 * v + 1]));
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    static_assert(FKV / FKB == 4, "four batches");
    clear_tab();   // (a barrier after the loads would wait for them all)
    load(qa, sa, 0);
    load(qb, sbb, 1);
    count(qa, sa, 0);
    load(qa, sa, 2);
    count(qb, sbb, 1);
    load(qb, sbb, 3);
    count(qa, sa, 2);
    count(qb, sbb, 3);
  } else {
  clear_tab();
#pragma unroll
  for (int v = 0; v < FKV; ++v) {
    // four rounds of key loads in flight at a time (all sixteen would hold
    // 64 registers of loads at once); one of record loads (16 registers)
    if (v % (KEYS ? 4 : 1) == 0) __builtin_amdgcn_sched_barrier(0);
    uint32_t kk[4];
    fused_keys4<KEYS>(a, lo + (uint64_t)v * FT * 4 + 4 * tid, hi, vec, kk);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (kk[u] != NOSUBJ) {
        atomicAdd(&tab[kk[u] >> 1], 1u << ((kk[u] & 1u) * 16u));
        sm |= 1ull << (v * 4 + u);
      }
    }
    kp[2 * v] = (kk[0] & 0xffffu) | kk[1] << 16;
    kp[2 * v + 1] = (kk[2] & 0xffffu) | kk[3] << 16;
    // opaque: otherwise the compiler keeps the 64 unpacked keys alive for
    // the later phases instead of these 32 registers
    asm volatile("" : "+v"(kp[2 * v]), "+v"(kp[2 * v + 1]));
  }
  }
  FSTAMP(1);
#define FKEY(v, u) ((kp[2 * (v) + ((u) >> 1)] >> (((u) & 1) * 16)) & 0xffffu)
#define FSUBJ(v, u) ((sm >> ((v) * 4 + (u))) & 1ull)
  const uint32_t nsubj = (uint32_t)__popcll(sm);
  // A bucket holding all 65 536 frames of a full segment wraps its u16
  // counter: detected by the segment being all one bucket.
  bool whole = false;
  if (f.seg == FSEG && hi - lo == FSEG) {
    if (tid == 0) wsum[FT / 64] = FSUBJ(0, 0) ? FKEY(0, 0) : NOSUBJ;
    uint32_t s = nsubj;
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if (lane == 0) wsum[wv] = s;
    __syncthreads();
    uint32_t tot = 0;
    for (int w = 0; w < FT / 64; ++w) tot += wsum[w];
    const uint32_t b0 = wsum[FT / 64];
    bool same = true;
#pragma unroll
    for (int v = 0; v < FKV; ++v)
#pragma unroll
      for (int u = 0; u < 4; ++u) same = same && FKEY(v, u) == b0;
    whole = __syncthreads_and(same) && tot == FSEG;
  }
  __syncthreads();
  {
    __shared__ uint32_t novf_l;
    if (tid == 0) novf_l = 0;
    __syncthreads();
    uint32_t *row = f.table + (uint64_t)c * f.nwords;
    uint32_t *ovf = f.ovf + (uint64_t)c * FOVF * 2;
    const uint32_t b0 = whole ? FKEY(0, 0) : NOSUBJ;
    for (uint32_t w = tid; w < f.nwords; w += FT) {
      const uint32_t h0 = whole ? 0u : tab[2 * w];
      const uint32_t h1 = whole || 2 * w + 1 >= words ? 0u : tab[2 * w + 1];
      uint32_t cnt[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
      if (whole && b0 >> 2 == w) cnt[b0 & 3] = FSEG;
      uint32_t packed = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (cnt[q] >= 255u) {
          const uint32_t j = atomicAdd(&novf_l, 1u);
          st_sc1(ovf + 2 * j, 4 * w + q);
          st_sc1(ovf + 2 * j + 1, cnt[q]);
        }
        packed |= min(cnt[q], 255u) << (8 * q);
      }
      st_sc1(row + w, packed);
    }
    __syncthreads();
    if (tid == 0) st_sc1(f.novf + c, novf_l);
  }
  // Speculative verdicts: as if no bucket ran out of tokens (the common
  // case: every subject permitted), written at the end of phase 2 (they
  // drain into the second barrier; phase 1 ends without waiting for them).
  // A workgroup whose buckets do run out raises its flag in that barrier's
  // arrival word; only then does phase 3 write the verdicts that differ.
  const bool valigned = ((uintptr_t)a.verdict & 3u) == 0;
  uint8_t *const vbase = a.verdict + lo;
  const uint32_t nrel = (uint32_t)(hi - lo);
  auto spec_word = [&](int v) {   // subject bits -> 1, else 2
    const uint32_t sv = (uint32_t)(sm >> (4 * v)) & 15u;
    return (sv & 1u ? 1u : 2u) | (sv & 2u ? 1u : 2u) << 8 | (sv & 4u ? 1u : 2u) << 16 |
           (sv & 8u ? 1u : 2u) << 24;
  };
  auto put_word = [&](uint32_t rel, uint32_t word) {
    if (valigned && rel + 4 <= nrel) {
      *(uint32_t *)(vbase + rel) = word;
    } else {
      for (uint32_t u = 0; u < 4 && rel + u < nrel; ++u) vbase[rel + u] = (uint8_t)(word >> (8 * u));
    }
  };
  auto put_spec = [&]() {
#pragma unroll
    for (int v = 0; v < FKV; ++v) {
      const uint32_t rel = (uint32_t)v * FT * 4 + 4 * tid;
      if (rel >= nrel) break;
      put_word(rel, spec_word(v));
    }
  };
  // An aborted launch fails closed: every subject frame of the segment is
  // denied (0), the others stay "not a subject" (2) -- no frame is admitted
  // without a token, as the reference's ip_permitted never does
  // (iphash/iphash.c:164-196) -- while the tokens stay as they were.
  auto put_fail = [&]() {
#pragma unroll
    for (int v = 0; v < FKV; ++v) {
      const uint32_t rel = (uint32_t)v * FT * 4 + 4 * tid;
      if (rel >= nrel) break;
      put_word(rel, spec_word(v) & 0x02020202u);
    }
  };
  FSTAMP(2);
#ifdef PPTK_PERMIT_SPEC_EARLY   // (A/B: the speculative verdicts before the table loads)
  put_spec();
#endif
  fused_stall(f, c, 1);
  if (fused_barrier(f, c, 1) < 0) {   // aborted: no token touched, subjects denied
    put_fail();
    return;
  }
  FSTAMP(3);

  // ---- phase 2: per bucket down its column ---------------------------------
  // Workgroup c takes a range of table words (4 buckets each); its threads
  // are 64 word lanes x 16 row slices (up to 16 rows each, all loads in
  // flight), so a bucket's column is summed by 16 threads at once.
  // The new token counts are committed only after the second barrier (an
  // aborted launch leaves the tokens untouched): slice 0 parks those of its
  // last word batch in LDS (tokl, no longer read), earlier batches (small
  // batches: few segments, many words each) go through f.ntok.
  {
    const uint32_t wpb = (f.nwords + f.nblk - 1) / f.nblk;
    const uint32_t wlo = min(f.nwords, c * wpb), whi = min(f.nwords, wlo + wpb);
    const uint32_t wl = tid & 63, s = tid >> 6;
    // some bucket of this workgroup's words ran out: one flag store per
    // workgroup, not one per word (thousands of write-through stores to one
    // address, all waited for by the barrier)
    if (tid == 0) out_l = 0;
    uint32_t *const cst = p23;          // c* found per (word lane, bucket)
    uint32_t *const tokl = p23 + 256;   // the tokens before the batch
    const uint32_t rs = (f.nblk + FSL - 1) / FSL;          // rows per slice (<= 16)
    uint32_t *part = list;                                  // [FSL][64][4]
    for (uint32_t w0 = wlo; w0 < whi; w0 += 64) {
      const uint32_t w = w0 + wl;
      const bool on = w < whi;
      const uint32_t *col = f.table + (uint64_t)(s * rs) * f.nwords + w;
      // (slice 0 reads the tokens now, beside the table loads: one round
      // trip instead of two)
      uint32_t tk[4] = {0u, 0u, 0u, 0u};
      if (s == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          tk[q] = on && 4 * w + q < a.hash_size ? a.tokens[4 * w + q] : 0u;
      }
      uint32_t p[4] = {0, 0, 0, 0};
      uint64_t sat = 0;   // saturated entries (bit 4 j + q): exact counts below
      uint32_t rowv[16];  // (kept for the boundary walk: no second load)
#pragma unroll
      for (int j = 0; j < 16; ++j)
        rowv[j] = on && (uint32_t)j < rs && s * rs + j < f.nblk
                      ? ld_sc1(col + (uint64_t)j * f.nwords) : 0u;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t x = rowv[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t y = (x >> (8 * q)) & 0xffu;
          sat |= (uint64_t)(y == 255u) << (4 * j + q);
          p[q] += y;
        }
      }
      for (uint64_t m = sat; m; m &= m - 1) {   // (rare: heavy buckets)
        const int e = __ffsll((unsigned long long)m) - 1;
        const int q = e & 3;
        const uint32_t x = fused_ovf(f, s * rs + (e >> 2), 4 * w + q) - 255u;
        p[0] += q == 0 ? x : 0u;
        p[1] += q == 1 ? x : 0u;
        p[2] += q == 2 ? x : 0u;
        p[3] += q == 3 ? x : 0u;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) part[(s * 64 + wl) * 4 + q] = p[q];
      if (s == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          cst[wl * 4 + q] = NOBLK;
          tokl[wl * 4 + q] = tk[q];
        }
      }
      __syncthreads();
      // the four buckets' totals and this slice's prefix (16-byte reads of
      // the partial sums: one per slice, not one per slice and bucket)
      uint32_t pre[4] = {0u, 0u, 0u, 0u}, tot[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (uint32_t s2 = 0; s2 < FSL; ++s2) {
        const u32x4 x = *(const u32x4 *)(part + (s2 * 64 + wl) * 4);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          tot[q] += xs[q];
          pre[q] += s2 < s ? xs[q] : 0u;
        }
      }
      // the slice holding the T_b-th frame finds its segment and rank
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {
        const uint32_t b = 4 * w + q;
        const uint32_t t = tokl[wl * 4 + q];
        // (selects: a register array indexed by the rolled q would go to scratch)
        const uint32_t tq = q == 0 ? tot[0] : q == 1 ? tot[1] : q == 2 ? tot[2] : tot[3];
        const uint32_t prq = q == 0 ? pre[0] : q == 1 ? pre[1] : q == 2 ? pre[2] : pre[3];
        const uint32_t pq = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
        if (on && b < a.hash_size && tq > t && t > 0 && prq < t && t <= prq + pq) {
          uint32_t cum = prq;
          if (((sat >> q) & 0x1111111111111111ull) == 0) {
            // no saturated entry in this bucket's rows: the sixteen rows
            // unrolled, no select chain, no early exit (rows past the slice
            // are 0 and cannot cross t again)
            uint32_t jf = 0xffffffffu, nd = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const uint32_t x = (rowv[j] >> (8 * q)) & 0xffu;
              const bool hit = jf == 0xffffffffu && cum + x >= t;
              nd = hit ? t - cum : nd;
              jf = hit ? (uint32_t)j : jf;
              cum += x;
            }
            st_sc1(f.need + b, nd);
            cst[wl * 4 + q] = s * rs + jf;
          } else {
            for (uint32_t j = 0; j < rs; ++j) {
              uint32_t x = 0;
#pragma unroll
              for (int jj = 0; jj < 16; ++jj) x = (uint32_t)jj == j ? rowv[jj] : x;
              x = (x >> (8 * q)) & 0xffu;
              if (x == 255u) x = fused_ovf(f, s * rs + j, b);
              if (cum + x >= t) {
                st_sc1(f.need + b, t - cum);
                cst[wl * 4 + q] = s * rs + j;
                break;
              }
              cum += x;
            }
          }
        }
      }
      __syncthreads();
      if (s == 0 && on) {   // code pairs and the new token counts
        uint32_t cd[4], ntk[4];
        const bool last = w0 + 64 >= whi;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t b = 4 * w + q;
          const uint32_t t = tokl[wl * 4 + q];
          cd[q] = tot[q] <= t ? CODE_ALL : t == 0 ? CODE_NONE : cst[wl * 4 + q];
          const uint32_t nt = t > tot[q] ? t - tot[q] : 0u;
          if (!last && b < a.hash_size) st_sc1(f.ntok + b, nt);
          ntk[q] = nt;
        }
        // (every read of tokl in this batch is behind the barrier above)
        if (last) {
#pragma unroll
          for (int q = 0; q < 4; ++q) tokl[wl * 4 + q] = ntk[q];
        }
        for (uint32_t r = 0; r < FCREPL; ++r) {
          uint32_t *const cr = f.code + r * ((words + 63u) & ~63u);
          if (2 * w < words) st_sc1(cr + 2 * w, cd[0] | cd[1] << 16);
          if (2 * w + 1 < words) st_sc1(cr + 2 * w + 1, cd[2] | cd[3] << 16);
        }
        if ((cd[0] & cd[1] & cd[2] & cd[3]) != CODE_ALL) out_l = 1u;
      }
      __syncthreads();
    }
    // the speculative verdicts, after the table loads (issued ahead of them
    // they would hold up their first use: loads and stores share one
    // in-order memory counter); they drain into the barrier
#ifndef PPTK_PERMIT_SPEC_EARLY
    put_spec();
#endif
  }
  FSTAMP(4);
  __syncthreads();
  fused_stall(f, c, 2);
  const int b2 = fused_barrier(f, c, 2, out_l != 0);
  if (b2 < 0) {   // aborted: the tokens stay as they were, subjects denied
    put_fail();
    return;
  }
  FSTAMP(5);
  // every workgroup is past phase 2: commit this one's token counts
  if (tid < 64) {
    const uint32_t wpb = (f.nwords + f.nblk - 1) / f.nblk;
    const uint32_t wlo = min(f.nwords, c * wpb), whi = min(f.nwords, wlo + wpb);
    for (uint32_t w0 = wlo; w0 < whi; w0 += 64) {
      const uint32_t w = w0 + tid;
      if (w >= whi) break;
      const bool last = w0 + 64 >= whi;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t b = 4 * w + q;
        if (b < a.hash_size) a.tokens[b] = last ? p23[256 + tid * 4 + q] : ld_sc1(f.ntok + b);
      }
    }
  }
  const bool any_out = b2 > 0;
  // no bucket ran out: the speculative verdicts stand
  if (!any_out) {
    FSTAMP(6);
    return;
  }

  // ---- phase 3: code table in LDS, the boundary ranks, the verdicts --------
  const uint32_t rbw = (a.hash_size + 31) / 32;
  for (uint32_t w = tid; w < rbw; w += FT) rbit[w] = 0;
  if (tid < FHASH_MAXP) p23[128 + tid] = 0;   // (fine class counts, below)
  __syncthreads();
  bool mine = false, many = false;
  uint16_t *const tab16s = (uint16_t *)tab;
  constexpr int SW = HMAX / 2 / FT;   // code words per thread (at most)
  uint32_t cw[SW];                    // all loads in flight at once
#ifdef PPTK_PERMIT_CODE_ROT
  const uint32_t crot = (c >> 3) & (SW - 1);
#else
  const uint32_t crot = 0;
#endif
  auto wof = [&](int j) { return (((uint32_t)j + crot) & (SW - 1)) * FT + tid; };
  const uint32_t *const code_r = f.code + (c % FCREPL) * ((words + 63u) & ~63u);
#pragma unroll
  for (int j = 0; j < SW; ++j) {
    const uint32_t w = wof(j);
    cw[j] = w < words ? ld_sc1(code_r + w) : 0u;
  }
  // the codes into LDS; this segment's c* buckets (bit 2 j + h) get, in a
  // second pass, the rank to find
  uint64_t cs = 0;
#pragma unroll
  for (int j = 0; j < SW; ++j) {
    const uint32_t w = wof(j);
    if (w >= words) continue;
    const uint32_t x = cw[j];
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (2 * w + h < a.hash_size && ((x >> (16 * h)) & 0xffffu) == c) cs |= 1ull << (2 * j + h);
    // in LDS, the verdict of every frame of the bucket here (1: T_b falls
    // in a later segment, or CODE_ALL; 0: an earlier one, or CODE_NONE); a
    // c* bucket's entry is rewritten below
    const uint32_t lo16 = x & 0xffffu, hi16 = x >> 16;
    tab[w] = (lo16 != CODE_NONE && c < lo16 ? 1u : 0u) | (hi16 != CODE_NONE && c < hi16 ? 1u : 0u) << 16;
  }
  // The rank to find, as a u16.  The T_b-th frame being b's last frame here
  // (its count in this segment's row) means every frame of b here is
  // permitted: verdict 1, no ranking -- with few frames per bucket and
  // segment the common case.  The segment's c* buckets are compacted into
  // the list (4 096 at a time) and spread evenly over the threads, so a
  // segment that is c* for thousands of buckets costs one round trip of
  // loads per 4 096 of them, not one per batch of a thread's words.
  {
    const uint32_t ncs = (uint32_t)__popcll(cs);
    uint32_t inc = ncs;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d);
      if (lane >= d) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t base = inc - ncs, tcs = 0;
    for (int w = 0; w < FT / 64; ++w) {
      const uint32_t y = wsum[w];
      base += w < wv ? y : 0u;
      tcs += y;
    }
    constexpr uint32_t CH = FT * 4;
#pragma unroll 1
    for (uint32_t ch = 0; ch < tcs; ch += CH) {
      __syncthreads();   // (the previous chunk's list reads are done)
      // (over the set bits only, in bit order: a few per thread)
      uint32_t pos = base;
      for (uint64_t m = cs; m; m &= m - 1) {
        const uint32_t bit = (uint32_t)__ffsll((unsigned long long)m) - 1u;
        if (pos >= ch && pos < ch + CH) list[pos - ch] = 2 * wof((int)(bit >> 1)) + (bit & 1u);
        ++pos;
      }
      __syncthreads();
      const uint32_t nch = min(CH, tcs - ch);
      uint32_t nd[CH / FT], rw[CH / FT];
#pragma unroll
      for (int k = 0; k < (int)(CH / FT); ++k) {   // all loads first
        const uint32_t i = tid + (uint32_t)k * FT;
        const uint32_t b = i < nch ? list[i] : 0u;
        nd[k] = ld_sc1(f.need + b);
        rw[k] = ld_sc1(f.table + (uint64_t)c * f.nwords + (b >> 2));
      }
#pragma unroll
      for (int k = 0; k < (int)(CH / FT); ++k) {
        if (tid + (uint32_t)k * FT >= nch) continue;
        const uint32_t b = list[tid + (uint32_t)k * FT];
        uint32_t kb = (rw[k] >> (8 * (b & 3u))) & 0xffu;
        if (kb == 255u) kb = fused_ovf(f, c, b);
        uint32_t e = 1u;   // (every frame here permitted)
        if (nd[k] < kb) {
          atomicOr(&rbit[b >> 5], 1u << (b & 31));
          e = nd[k];
          mine = true;
          many = many || kb > FHASH_K;
        }
        tab16s[b] = (uint16_t)e;
      }
    }
  }
  mine = __syncthreads_or(mine);
  many = __syncthreads_or(many);
  FSTAMP(7);
  // (16-bit accesses: the two buckets of a word are walked by different waves)
  uint16_t *const tab16 = (uint16_t *)tab;
  auto tabh = [&](uint32_t b) { return (uint32_t)tab16[b]; };
  auto isc = [&](uint32_t b) { return (rbit[b >> 5] >> (b & 31)) & 1u; };
  // Candidate frames of this thread (bit 4 v + u): subjects of a bucket
  // whose c* is this segment.  The ordered walk below leaves, for each such
  // bucket, tab16[b] = the segment offset of its T_b-th frame (the last one
  // permitted) and clears its rbit bit: the verdicts need no global limit.
  uint64_t cm = 0;
  if (mine) {
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    // Candidates, counted by fine class (the top 5 bits of a 16-bit bucket
    // hash: FHASH_MAXP classes); pmh = those of the lower 16 fine classes
    auto hash1 = [](uint32_t b) { return b * 0x9E3779B1u; };
    uint32_t *const fcnt = p23 + 128;
    uint64_t pmh = 0;
#pragma unroll
    for (int v = 0; v < FKV; ++v) {
      __builtin_amdgcn_sched_barrier(0);   // (else all 64 LDS lookups are hoisted)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (FSUBJ(v, u) && isc(FKEY(v, u))) {
          const uint32_t fc = (hash1(FKEY(v, u)) >> 8 & 0xffffu) >> 11;
          atomicAdd(&fcnt[fc], 1u);
          cm |= 1ull << (4 * v + u);
          if (fc < FHASH_MAXP / 2) pmh |= 1ull << (4 * v + u);
        }
    }
    // the segment's candidate count
    uint32_t ncand = (uint32_t)__popcll(cm);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) ncand += __shfl_xor(ncand, d);
    if (lane == 0) wsum[wv] = ncand;
    __syncthreads();
    ncand = 0;
    for (int w = 0; w < FT / 64; ++w) ncand += wsum[w];
    __syncthreads();   // (wsum is reused below)
    // Ranking by hash tables when no ranked bucket has more than FHASH_K
    // frames here (counting along a probe sequence costs a bucket's frames
    // once per frame): the candidates go in passes by bucket class, a pass
    // being at most FHASH_PASS of them in the list's 4 096 slots (load <=
    // 1/2, double hashing: short probe sequences for every lane of a wave).
    // In a pass each candidate is inserted as (offset << 16 | bucket), then
    // counts the frames of its bucket at smaller offsets along its bucket's
    // probe sequence (its rank, in frame order), and the one whose rank + 1
    // is the bucket's rank to find is the boundary frame.  More classes than
    // FHASH_MAXP, or a class over FHASH_PASS: the ordered walk below.
    // The pass count is a power of two, so a pass is a run of fine classes
    // (pass = fine class >> (5 - log2 npass)) and its size is known from
    // the fine counts without another sweep; with two passes pmh is pass 0.
    const uint32_t npr = max(1u, (ncand + FHASH_PASS * 3 / 4 - 1) / (FHASH_PASS * 3 / 4));
    uint32_t npass = 1;
    while (npass < npr && npass <= FHASH_MAXP) npass <<= 1;
    bool hashed = !many && npass <= FHASH_MAXP;
    auto cls = [&](uint32_t b) { return (((hash1(b) >> 8) & 0xffffu) * npass) >> 16; };   // (no division)
    if (hashed && npass > 1) {
      const uint32_t per = FHASH_MAXP / npass;
      bool over = false;
      for (uint32_t p = 0; p < npass; ++p) {
        uint32_t n = 0;
        for (uint32_t i = 0; i < per; ++i) n += fcnt[p * per + i];
        over = over || n > FHASH_PASS;
      }
      hashed = !over;
    }
    if (hashed) {
      constexpr uint32_t HC = FT * 4;
      uint32_t *const occ = p23;        // slot occupancy, 128 words
      uint32_t *const ent = rbit;       // the pass's candidates, compacted (no longer needed as rbit)
      auto off_at = [&](int v, int u) { return (uint32_t)v * FT * 4 + 4 * tid + (uint32_t)u; };
      uint64_t t_part = 0, t_rank = 0, t0 = 0;   // (diagnostics: wave 0's time)
      uint64_t left = cm;   // candidates of the passes still to come
#pragma unroll 1
      for (uint32_t pass = 0; pass < npass; ++pass) {
        if (tid == 0) t0 = __builtin_amdgcn_s_memrealtime();
        // (opaque per pass: else the 64 keys and classes are hoisted out of
        // the pass loop into 64 more registers)
#pragma unroll
        for (int q = 0; q < FKV * 2; ++q) asm volatile("" : "+v"(kp[q]));
        for (uint32_t i = tid; i < HC / 32; i += FT) occ[i] = 0;
        // this pass's candidates of the thread, compacted block-wide (frame
        // order does not matter here: ranks come from the offsets), so each
        // thread then handles at most two entries -- a wave runs two probe
        // loops, not one per round and lane that holds a candidate
        // (the last pass takes what is left, and of two passes the first is
        // pmh: no class sweep of their own)
        uint64_t pm = 0;
        if (pass + 1 == npass) {
          pm = left;
        } else if (pass == 0 && npass == 2) {
          pm = pmh;
        } else {
#pragma unroll
          for (int v = 0; v < FKV; ++v) {
            if (((left >> (4 * v)) & 15ull) == 0) continue;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (((left >> (4 * v + u)) & 1ull) && cls(FKEY(v, u)) == pass) pm |= 1ull << (4 * v + u);
          }
        }
        left &= ~pm;
        const uint32_t pc = (uint32_t)__popcll(pm);
        uint32_t inc = pc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(inc, d);
          if (lane >= d) inc += y;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint32_t pos = inc - pc, ptot = 0;
        for (int w = 0; w < FT / 64; ++w) {
          const uint32_t y = wsum[w];
          pos += w < wv ? y : 0u;
          ptot += y;
        }
#pragma unroll
        for (int v = 0; v < FKV; ++v) {
          if (((pm >> (4 * v)) & 15ull) == 0) continue;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if ((pm >> (4 * v + u)) & 1ull) ent[pos++] = off_at(v, u) << 16 | FKEY(v, u);
        }
        __syncthreads();
        if (tid == 0) {
          const uint64_t t = __builtin_amdgcn_s_memrealtime();
          t_part += t - t0;
          t0 = t;
        }
        auto step_of = [](uint32_t hv) { return ((hv >> 7) | 1u) & (HC - 1); };   // odd: visits every slot
        for (uint32_t i = tid; i < ptot; i += FT) {
          const uint32_t e = ent[i], hv = hash1(e & 0xffffu), step = step_of(hv);
          for (uint32_t h = hv >> 20;; h = (h + step) & (HC - 1)) {
            const uint32_t bit = 1u << (h & 31);
            if (!(atomicOr(&occ[h >> 5], bit) & bit)) {
              list[h] = e;
              break;
            }
          }
        }
        __syncthreads();
        uint32_t bnd[FHASH_PASS / FT];   // this thread's boundary entries (or NOSUBJ)
#pragma unroll
        for (int k = 0; k < (int)(FHASH_PASS / FT); ++k) {
          const uint32_t i = tid + (uint32_t)k * FT;
          bnd[k] = NOSUBJ;
          if (i >= ptot) continue;
          const uint32_t e = ent[i], b = e & 0xffffu, off = e >> 16;
          const uint32_t hv = hash1(b), step = step_of(hv);
          uint32_t rank = 0;
          for (uint32_t h = hv >> 20; (occ[h >> 5] >> (h & 31)) & 1u; h = (h + step) & (HC - 1)) {
            const uint32_t x = list[h];
            rank += (x & 0xffffu) == b && (x >> 16) < off ? 1u : 0u;
          }
          if (rank + 1u == tabh(b)) bnd[k] = e;
        }
        __syncthreads();   // (every rank read before a limit replaces it)
#pragma unroll
        for (int k = 0; k < (int)(FHASH_PASS / FT); ++k)
          if (bnd[k] != NOSUBJ) tab16[bnd[k] & 0xffffu] = (uint16_t)(bnd[k] >> 16);
        __syncthreads();   // (ent, occ and wsum are rewritten by the next pass)
        if (tid == 0) t_rank += __builtin_amdgcn_s_memrealtime() - t0;
      }
      if (tid == 0) {
        f.stamps[9 * FMAXBLK + c] = (uint32_t)t_part;
        f.stamps[10 * FMAXBLK + c] = (uint32_t)t_rank;
        f.stamps[11 * FMAXBLK + c] = npass;
      }
    } else {
    // (diagnostics: wave 0's time in the list building and in the walk)
    uint64_t t_list = 0, t_walk = 0, tr0 = 0, tw0 = 0;
#pragma unroll 1
    for (int v = 0; v < FKV; ++v) {
      if (tid == 0) tr0 = __builtin_amdgcn_s_memrealtime();
      const uint32_t base_off = (uint32_t)v * FT * 4 + 4 * tid;
      const uint32_t m = (uint32_t)(cm >> (4 * v)) & 15u;
      // this round's two key registers (a select: the array stays in registers)
      uint32_t k01 = 0, k23 = 0;
#pragma unroll
      for (int vv = 0; vv < FKV; ++vv) {
        k01 = vv == v ? kp[2 * vv] : k01;
        k23 = vv == v ? kp[2 * vv + 1] : k23;
      }
      // block exclusive scan of the candidate counts (frame order)
      const uint32_t cnt = (uint32_t)__popc(m);
      uint32_t inc = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d);
        if (lane >= d) inc += y;
      }
      if (lane == 63) wsum[wv] = inc;
      __syncthreads();
      uint32_t basep = 0, total = 0;
      for (int w = 0; w < FT / 64; ++w) {
        const uint32_t y = wsum[w];
        basep += w < wv ? y : 0u;
        total += y;
      }
      basep += inc - cnt;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (m & (1u << u))
          list[basep++] = (base_off + u) << 16 | (((u < 2 ? k01 : k23) >> ((u & 1) * 16)) & 0xffffu);
      __syncthreads();
      // the ordered walk: wave wv takes the buckets with b % 16 == wv, one
      // distinct bucket of a 64-entry step per ballot
      if (tid == 0) tw0 = __builtin_amdgcn_s_memrealtime();
      for (uint32_t s0 = 0; s0 < total; s0 += 64) {
        const uint32_t e = s0 + (uint32_t)lane < total ? list[s0 + lane] : NOSUBJ;
        const uint32_t b = e & 0xffffu;
        const bool on = e != NOSUBJ && (b & (FT / 64 - 1)) == (uint32_t)wv;
        uint64_t todo = __ballot(on);
        while (todo) {
          const int leader = __ffsll((unsigned long long)todo) - 1;
          const uint32_t bb = __shfl(b, leader);
          const uint64_t mm = __ballot(on && b == bb);
          if (isc(bb)) {   // (else its frame was found in an earlier step)
            const uint32_t r0 = tabh(bb);   // rank still to find, >= 1
            const uint32_t pc = (uint32_t)__popcll(mm);
            if (r0 <= pc) {
              if (on && b == bb && (uint32_t)__popcll(mm & lt) + 1u == r0) {
                tab16[bb] = (uint16_t)(e >> 16);
                atomicAnd(&rbit[bb >> 5], ~(1u << (bb & 31)));
              }
            } else if (lane == leader) {
              tab16[bb] = (uint16_t)(r0 - pc);
            }
          }
          todo &= ~mm;
        }
      }
      if (tid == 0) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        t_walk += t - tw0;
        t_list += tw0 - tr0;
      }
      __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
      f.stamps[9 * FMAXBLK + c] = (uint32_t)t_list;
      f.stamps[10 * FMAXBLK + c] = (uint32_t)t_walk;
    }
    }
  }
  FSTAMP(8);
  // (32-bit offsets from the segment start: the 64-bit frame index of
  // every round would be hoisted into 32 registers)
  const bool aligned = valigned;
#pragma unroll
  for (int v = 0; v < FKV; ++v) {
#ifndef PPTK_PERMIT_VERDICT_FREE
    __builtin_amdgcn_sched_barrier(0);
#endif
    const uint32_t rel = (uint32_t)v * FT * 4 + 4 * tid;
    if (rel >= nrel) break;
    uint32_t vd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t kk = FKEY(v, u);
      if (!FSUBJ(v, u)) {
        vd[u] = 2u;
      } else if ((cm >> (4 * v + u)) & 1ull) {   // up to its T_b-th frame
        vd[u] = rel + u <= tabh(kk) ? 1u : 0u;
      } else {
        vd[u] = tabh(kk);
      }
    }
    // (only the words that differ from the speculative ones)
    const uint32_t word = vd[0] | vd[1] << 8 | vd[2] << 16 | vd[3] << 24;
    if (word != spec_word(v)) {
      if (aligned && rel + 4 <= nrel) {
        *(uint32_t *)(vbase + rel) = word;
      } else {
        for (uint32_t u = 0; u < 4 && rel + u < nrel; ++u) vbase[rel + u] = (uint8_t)vd[u];
      }
    }
  }
  FSTAMP(6);
#undef FKEY
#undef FSUBJ
#undef FSTAMP
}

// Run boundaries of the sorted keys: first[b] and end[b] of every bucket
// present (non-subject keys, == hash_size, sort last and are skipped).  Four
// keys per thread (one 16-byte load); the neighbours across a thread's
// edge come from the adjacent lanes, or from memory at a wave's edge.
__device__ __forceinline__ void bound_at(const PermitArgs &a, uint32_t *first, uint32_t *end,
                                         uint64_t p, uint32_t prev, uint32_t b, uint32_t next) {
  if (b >= a.hash_size) return;
  if (p == 0 || prev != b) first[b] = (uint32_t)p;
  if (p + 1 == a.n || next != b) end[b] = (uint32_t)(p + 1);
}

__global__ __launch_bounds__(PT) void permit_bounds(PermitArgs a, const uint32_t *skeys,
                                                    uint32_t *first, uint32_t *end) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t t = (uint64_t)blockIdx.x * PT + threadIdx.x;
  const uint64_t p = 4 * t;
  const int lane = threadIdx.x & 63;
  const bool whole = p + 4 <= a.n;
  u32x4 q = (u32x4){0u, 0u, 0u, 0u};
  if (whole) q = *(const u32x4 *)(skeys + p);
  // neighbours (every lane takes part in the shuffles)
  uint32_t prev = __shfl_up(q.w, 1), next = __shfl_down(q.x, 1);
  if (!whole) {
    for (uint64_t k = p; k < a.n; ++k)    // the ragged last group
      bound_at(a, first, end, k, k ? skeys[k - 1] : 0u, skeys[k], k + 1 < a.n ? skeys[k + 1] : 0u);
    return;
  }
  if (lane == 0 && p > 0) prev = skeys[p - 1];
  if ((lane == 63 || p + 8 > a.n) && p + 4 < a.n) next = skeys[p + 4];   // (lane + 1: ragged)
  bound_at(a, first, end, p, prev, q.x, q.y);
  bound_at(a, first, end, p + 1, q.x, q.y, q.z);
  bound_at(a, first, end, p + 2, q.y, q.z, q.w);
  bound_at(a, first, end, p + 3, q.z, q.w, next);
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
// replaces scattered one byte per frame: 0.22 ms per 16 M frames), the
// non-subject frames' 2 included.  Four frames per thread: one 16-byte key
// load, one 4-byte verdict store when the verdict array's alignment allows.
__device__ __forceinline__ uint32_t verdict_of(const PermitArgs &a, const uint32_t *lim,
                                               uint64_t i, uint32_t b) {
  return b >= a.hash_size ? 2u : ((uint32_t)i < lim[b] ? 1u : 0u);   // key hash_size: not subject
}

__global__ __launch_bounds__(PT) void permit_verdicts(PermitArgs a, const uint32_t *keys,
                                                      const uint32_t *lim) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t i = 4 * ((uint64_t)blockIdx.x * PT + threadIdx.x);
  if (i >= a.n) return;
  if (i + 4 <= a.n && ((uintptr_t)(a.verdict + i) & 3u) == 0) {
    const u32x4 q = *(const u32x4 *)(keys + i);
    *(uint32_t *)(a.verdict + i) = verdict_of(a, lim, i, q.x) | verdict_of(a, lim, i + 1, q.y) << 8 |
                                   verdict_of(a, lim, i + 2, q.z) << 16 |
                                   verdict_of(a, lim, i + 3, q.w) << 24;
    return;
  }
  for (uint64_t k = i; k < i + 4 && k < a.n; ++k)
    a.verdict[k] = (uint8_t)verdict_of(a, lim, k, keys[k]);
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

// Onesweep with 9-bit digits: the keys (log2(hash_size) + 1 bits, 17 for
// 2^16 buckets) sort in two passes instead of the default 8-bit digits'
// three; the values are the frame indices, read from a counting iterator
// (no index array is written).  Blocks of 1024 threads x 8 keys: 16 M
// records 0.529 ms per batch, against 0.61 with 512 x 16, 0.76 with
// 256 x 16, 0.67 with 512 x 8, 0.60 with 1024 x 12, 0.57 with 1024 x 16
// and 0.66 with 1024 x 4 (tools/opbench.py permit).
template <unsigned BS, unsigned IPT>
using OnesweepConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                        rocprim::kernel_config<BS, IPT>, 9,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <class Cfg>
hipError_t sort_pairs_cfg(void *tmp, size_t &tb, const uint32_t *keys, uint32_t *skeys,
                          uint32_t *svals, size_t n, unsigned bits, hipStream_t st) {
  return rocprim::radix_sort_pairs<Cfg>(tmp, tb, keys, skeys,
                                        rocprim::counting_iterator<uint32_t>(0), svals, n, 0,
                                        bits, st);
}

// (tmp == nullptr: the temporary size of the chosen shape into tb)
hipError_t sort_pairs(void *tmp, size_t &tb, const uint32_t *keys, uint32_t *skeys,
                      uint32_t *svals, size_t n, unsigned bits, hipStream_t st) {
  return sort_pairs_cfg<OnesweepConfig<1024, 8>>(tmp, tb, keys, skeys, svals, n, bits, st);
}

int key_bits(uint32_t hash_size) {
  int b = 0;
  while ((1ull << b) <= hash_size) ++b;   // keys 0 .. hash_size inclusive
  return b;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// sort-free path scratch: dense keys, the histogram table, per-bucket lim /
// need / pend, per-block flags
struct HistScratch {
  uint32_t *ckey, *bh, *lim, *need, *blk_flag, *clist;
  uint16_t *code;
  uint32_t nblk;
  size_t total;
};

void hist_layout(uint64_t n, uint32_t hash_size, void *base, HistScratch &s) {
  uint8_t *p = (uint8_t *)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    uint8_t *q = p ? p + off : nullptr;
    off += align256(bytes);
    return (uint32_t *)q;
  };
  s.nblk = (uint32_t)((n + HB - 1) / HB);
  const size_t words = (hash_size + 1) / 2;
  s.ckey = take(n * 4);
  s.bh = take((size_t)s.nblk * words * 4);
  s.lim = take((size_t)hash_size * 4);
  s.need = take((size_t)hash_size * 4);
  s.code = (uint16_t *)take((size_t)hash_size * 2 + 4);
  s.blk_flag = take((size_t)s.nblk * 4);
  s.clist = take(n * 4);
  s.total = off;
}

struct PermitScratch {
  uint32_t *keys, *skeys, *svals, *first, *end, *lim;
  void *tmp;
  size_t tmp_bytes, total;
};

hipError_t layout(uint64_t n, uint32_t hash_size, void *base, PermitScratch &s) {
  size_t sort_tmp = 0;
  hipError_t e = sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, (size_t)n,
                            (unsigned)key_bits(hash_size), 0);
  if (e != hipSuccess) return e;
  uint8_t *p = (uint8_t *)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    uint8_t *q = p ? p + off : nullptr;
    off += align256(bytes);
    return q;
  };
  s.keys = (uint32_t *)take(n * 4);
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

// Fused path geometry: nblk segments of seg frames (a multiple of 4096,
// at most FSEG), at most one workgroup per CU.
struct FusedGeom {
  uint32_t nblk, seg;
};

bool fused_geom(uint64_t n, uint32_t hash_size, int ncu, FusedGeom &g) {
  if (hash_size > HMAX || ncu < 1 || n == 0) return false;
  const uint64_t maxblk = std::min<uint64_t>((uint64_t)ncu, FMAXBLK);
  if (n > maxblk * FSEG) return false;
  const uint64_t want = std::min<uint64_t>(maxblk, (n + 4095) / 4096);
  const uint64_t seg = ((n + want - 1) / want + 4095) / 4096 * 4096;
  g.seg = (uint32_t)seg;
  g.nblk = (uint32_t)((n + seg - 1) / seg);
  return true;
}

void fused_layout(uint32_t nblk, uint32_t seg, uint32_t hash_size, void *base, PermitFused &f,
                  size_t &total) {
  uint8_t *p = (uint8_t *)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    uint32_t *q = p ? (uint32_t *)(p + off) : nullptr;
    off += align256(bytes);
    return q;
  };
  f.nblk = nblk;
  f.seg = seg;
  f.nwords = (hash_size + 3) / 4;
  f.arrive = (uint64_t *)take(FMAXBLK * 8);
  f.out = (uint64_t *)take(16);
  f.stamps = take(FSTAMPS * FMAXBLK * 4);
  f.table = take((size_t)nblk * f.nwords * 4);
  f.ovf = take((size_t)nblk * FOVF * 8);
  f.novf = take((size_t)nblk * 4);
  f.need = take((size_t)hash_size * 4);
  f.code = take((size_t)FCREPL * ((((hash_size + 1) / 2) + 63) & ~63u) * 4);
  f.ntok = take((size_t)hash_size * 4);
  total = off;
}
// (f.out sits at this offset of the scratch for every geometry)
constexpr size_t kFusedOutOff = (FMAXBLK * 8 + 255) / 256 * 256;

// Barrier nonces: base + 8 k for the k-th fused launch of this process
// (distinct per launch; the base is random, so a word another process left
// in a reused scratch buffer never matches), low three bits clear for the
// barrier generation and the abort bit.
uint64_t nonce_base() {
  static const uint64_t base = [] {
    std::random_device rd;
    uint64_t z = ((uint64_t)rd() << 32 ^ rd()) ^
                 (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (z ^ (z >> 31)) & ~7ull;
  }();
  return base;
}
std::atomic<uint64_t> g_nonce_ctr{1};
uint64_t nonce_of(uint64_t k) { return nonce_base() + 8 * k; }

// Per scratch buffer: the first launch counter since its status was last
// read (pptk_rx_permit_status reports whether any launch since then
// aborted).  Small: one entry per scratch buffer in use.
std::mutex g_status_mu;
std::unordered_map<const void *, std::pair<uint64_t, uint64_t>> g_status;   // first, last k

// At most this many scratch buffers are tracked: a caller that never queries
// the status (or allocates a fresh scratch per call) does not grow the map
// without bound; the entry whose last launch is oldest goes first (a later
// status query on it reports 0).
constexpr size_t kMaxStatus = 1024;

void note_launch(const void *scratch, uint64_t k) {
  std::lock_guard<std::mutex> sl(g_status_mu);
  auto it = g_status.find(scratch);
  if (it != g_status.end()) {
    it->second.second = k;
    return;
  }
  if (g_status.size() >= kMaxStatus) {
    auto old = g_status.begin();
    for (auto j = g_status.begin(); j != g_status.end(); ++j)
      if (j->second.second < old->second.second) old = j;
    g_status.erase(old);
  }
  g_status.emplace(scratch, std::make_pair(k, k));
}

// The previous fused launch of each device, which the next one on another
// stream waits for: two fused grids running at once could split the CUs
// between them and each wait at its barrier for workgroups that cannot
// become resident.  An event per device, the stop event of
// every fused launch (hipExtLaunchKernelGGL's own, 2.2 us per call), so a
// launch from a new stream only waits for that event -- never for the whole
// device, which would also wait for other streams' gathers and batches.
// (A/B builds: PPTK_PERMIT_ORDER=0, no order)
#ifndef PPTK_PERMIT_ORDER
#define PPTK_PERMIT_ORDER 1
#endif
struct FusedOrder {
  std::mutex mu;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
  bool any = false;     // a fused launch was made on this device (ev records its end)
};
FusedOrder g_order[64];

// Test builds only (PPTK_RX_TEST_HOOKS): fault injection for the abort path.
void test_hooks(PermitFused &f) {
#ifdef PPTK_RX_TEST_HOOKS
  // (read at every launch: a test sets and clears them between calls)
  auto knob = [](const char *name, long dflt) {
    const char *e = getenv(name);
    return e ? atol(e) : dflt;
  };
  // (milliseconds, or microseconds through the _US forms, which win)
  const long stall_us = knob("PPTK_RX_TEST_PERMIT_STALL_US",
                             knob("PPTK_RX_TEST_PERMIT_STALL_MS", 0) * 1000);
  const long stall_at = knob("PPTK_RX_TEST_PERMIT_STALL_AT", 1);
  const long spin_us = knob("PPTK_RX_TEST_PERMIT_SPIN_US",
                            knob("PPTK_RX_TEST_PERMIT_SPIN_MS", 0) * 1000);
  if (spin_us > 0) f.spin_ticks = (uint64_t)spin_us * 100ull;
  if (stall_us > 0) {
    f.stall_ticks = (uint64_t)std::min(stall_us, 10000000l) * 100ull;
    f.stall_at = (uint32_t)stall_at;
  }
#else
  (void)f;
#endif
}

// The fused kernel fits one workgroup per CU (its registers and 150 KB of
// LDS); checked once.
bool fused_fits() {
  static const bool ok = [] {
    int nb = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, permit_fused<true>, FT, 0) ==
               hipSuccess &&
           nb >= 1;
  }();
  return ok;
}

}  // namespace

size_t permit_scratch_bytes(uint64_t n, uint32_t hash_size) {
  size_t fused = 0;
  FusedGeom g;
  if (fused_geom(n, hash_size, (int)FMAXBLK, g)) {
    // (every geometry the fused path may pick for n takes at most this:
    // its table grows with the segment count, at most FMAXBLK)
    PermitFused f;
    fused_layout(FMAXBLK, FSEG, hash_size, nullptr, f, fused);
  }
  if (hash_size <= HMAX && (n + HB - 1) / HB <= MAX_BLOCKS) {
    HistScratch h;
    hist_layout(n, hash_size, nullptr, h);
    return std::max(h.total, fused);
  }
  PermitScratch s;
  if (layout(n, hash_size, nullptr, s) != hipSuccess) return 0;
  return s.total;
}

hipError_t launch_permit(const PermitArgs &a, void *scratch, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  FusedGeom g;
  // (records: the four passes -- their 1 GB read dominates, and the fused
  // kernel's records loads, one round in flight for its register budget,
  // measured slower: 0.351 vs 0.238 ms per 16 M records)
  int dev = -1;
  if (!a.force_passes && a.keys_in && fused_geom(a.n, a.hash_size, a.ncu, g) && fused_fits() &&
      hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
    PermitFused f{};
    size_t total = 0;
    fused_layout(g.nblk, g.seg, a.hash_size, scratch, f, total);
    f.spin_ticks = FUSED_SPIN_TICKS;
    test_hooks(f);
    FusedOrder &o = g_order[dev];
    std::lock_guard<std::mutex> lk(o.mu);
    hipError_t e = hipSuccess;
    // (a device-scope release is all the stream wait needs: no system-scope
    // fence -- an L2 write-back -- behind every launch)
    if (!o.ev && hipEventCreateWithFlags(&o.ev, hipEventDisableTiming |
                                                    hipEventDisableSystemFence) != hipSuccess &&
        (e = hipEventCreateWithFlags(&o.ev, hipEventDisableTiming)) != hipSuccess)
      return e;
    if (PPTK_PERMIT_ORDER && o.any && o.last != st &&
        (e = hipStreamWaitEvent(st, o.ev, 0)) != hipSuccess)
      return e;
    const uint64_t k = g_nonce_ctr.fetch_add(1);
    f.nonce = nonce_of(k);
    note_launch(scratch, k);
    if (PPTK_PERMIT_ORDER) {
      // the order event as the launch's own stop event (2.2 us per call;
      // a separate hipEventRecord behind the kernel cost 3.6)
      hipExtLaunchKernelGGL(permit_fused<true>, dim3(g.nblk), dim3(FT), 0, st, nullptr, o.ev, 0,
                            a, f);
    } else {
      hipLaunchKernelGGL(permit_fused<true>, dim3(g.nblk), dim3(FT), 0, st, a, f);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    o.last = st;
    o.any = true;
    return hipSuccess;
  }
  if (a.hash_size <= HMAX && (a.n + HB - 1) / HB <= MAX_BLOCKS) {
    HistScratch h;
    hist_layout(a.n, a.hash_size, scratch, h);
    hipLaunchKernelGGL(permit_hist, dim3(h.nblk), dim3(HT), 0, st, a, h.ckey, h.bh, h.blk_flag);
    hipLaunchKernelGGL(permit_scan, dim3(blocks(a.hash_size)), dim3(PT), 0, st, a, h.bh, h.nblk,
                       h.lim, h.need, h.code, h.blk_flag);
    hipLaunchKernelGGL(permit_resolve, dim3(h.nblk), dim3(HT), 0, st, a, h.ckey, h.need, h.code,
                       h.blk_flag, h.clist, h.lim);
    // one block per CU holds the 128 KB table (a persistent grid)
    const unsigned vb = (unsigned)std::min<uint64_t>((a.n + 4 * HT - 1) / (4 * HT),
                                                     (uint64_t)std::max(1, a.ncu));
    hipLaunchKernelGGL(permit_verdicts_tab, dim3(vb), dim3(HT), 0, st, a, h.ckey, h.code, h.lim);
    return hipGetLastError();
  }
  PermitScratch s;
  hipError_t e = layout(a.n, a.hash_size, scratch, s);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(s.first, 0, (size_t)a.hash_size * 8, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(permit_keys, dim3(blocks(a.n)), dim3(PT), 0, st, a, s.keys);
  size_t tb = s.tmp_bytes;
  e = sort_pairs(s.tmp, tb, s.keys, s.skeys, s.svals, (size_t)a.n,
                 (unsigned)key_bits(a.hash_size), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(permit_bounds, dim3(blocks((a.n + 3) / 4)), dim3(PT), 0, st, a, s.skeys,
                     s.first, s.end);
  hipLaunchKernelGGL(permit_limits, dim3(blocks(a.hash_size)), dim3(PT), 0, st, a, s.svals,
                     s.first, s.end, s.lim);
  hipLaunchKernelGGL(permit_verdicts, dim3(blocks((a.n + 3) / 4)), dim3(PT), 0, st, a, s.keys,
                     s.lim);
  hipLaunchKernelGGL(permit_consume, dim3(blocks(a.hash_size)), dim3(PT), 0, st, a, s.first,
                     s.end);
  return hipGetLastError();
}

int permit_status(const void *scratch, hipStream_t st) {
  std::pair<uint64_t, uint64_t> r;
  {
    std::lock_guard<std::mutex> sl(g_status_mu);
    auto it = g_status.find(scratch);
    if (it == g_status.end()) return 0;   // no fused launch on it since the last query
    r = it->second;
    g_status.erase(it);
  }
  if (hipStreamSynchronize(st) != hipSuccess) return -EIO;
  uint64_t w = 0;
  if (hipMemcpy(&w, (const uint8_t *)scratch + kFusedOutOff + 8, 8, hipMemcpyDeviceToHost) !=
      hipSuccess)
    return -EIO;
  if (!(w & 1u)) return 0;
  const uint64_t k = ((w & ~7ull) - nonce_base()) / 8;
  return k >= r.first && k <= r.second ? -ETIMEDOUT : 0;
}

hipError_t launch_refill(uint32_t *tokens, uint32_t start, uint32_t end, uint32_t add,
                         uint32_t initial, hipStream_t st) {
  if (end <= start) return hipSuccess;
  hipLaunchKernelGGL(tokens_refill, dim3(blocks(end - start)), dim3(PT), 0, st, tokens, start,
                     end, add, initial);
  return hipGetLastError();
}

}  // namespace pptk
