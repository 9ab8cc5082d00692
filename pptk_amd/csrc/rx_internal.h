// rx_internal.h -- shared between the kernels and the C-ABI shim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/pptk_rx.h"

namespace pptk {

// Every C-ABI entry point works on its context's device and gives the
// calling thread its current device back on return: a drop-in C library
// must not move a multi-GPU rx thread's later hipMalloc or launches to
// another GPU.
struct DeviceScope {
  int prev = -1;
  bool ok = false;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = prev == dev || hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope &) = delete;
  DeviceScope &operator=(const DeviceScope &) = delete;
};

// Context internals shared with the multi-GPU module (rx_comm.hip).
int ctx_device(const pptk_rx_ctx *c);
std::atomic<void *> *ctx_comm_slot(pptk_rx_ctx *c);
uint32_t ctx_comm_timeout_ms(const pptk_rx_ctx *c);   // opts.comm_timeout_ms (0 -> default)
// CUs of the collective stream pptk_rx_stream_split left the context (0: no
// split): the channel cap (ncclConfig_t.maxCTAs) of a communicator created on it
int ctx_coll_cap(const pptk_rx_ctx *c);
void comm_release(pptk_rx_ctx *c);   // destroys the context's communicator, if any

// Diagnostic tune bits (RxKArgs::tune 3, 4, 7, 9: skip record stores, the
// per-frame phase, half the record bytes, the tx writes -- output invalid,
// for profiling) and the A/B environment knobs of the host code exist only
// in experiment builds (`make abvariant NAME=exp DEFS=-DPPTK_RX_EXPERIMENTS`):
// in the product library the branches are compiled out and the knobs are
// constants (INTEGRATION.md section 6 lists the knobs a product build reads).
#if defined(PPTK_RX_EXPERIMENTS) || defined(PPTK_RX_DIAG)
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif

// Kernel arguments (by value; a handful of SGPRs).
struct RxKArgs {
  const uint8_t *frames;
  const uint64_t *off;   // nullable -> fixed stride
  const uint16_t *len;   // nullable -> fixed_len
  const uint32_t *perm;  // nullable -> identity
  uint64_t stride;
  uint64_t n;
  pptk_rx_rec *recs;
  pptk_rx_rec32 *recs32; // nullable: compact records instead of recs
  uint64_t *hash;        // nullable
  pptk_rx_frag *frag;    // nullable: fragment side records
  uint32_t *key;         // nullable: dense rate-limiter keys (pptk_rx_dev_batch.d_key)
  uint64_t k0, k1;       // SipHash key words (LE loads of key[0..7], key[8..15])
  uint64_t mask6_0, mask6_1;  // ipv6_permitted prefix mask over the 16 address bytes
  uint32_t mask4;        // ip_permitted prefix mask (host order)
  uint32_t hash_mask;    // iphash_size - 1
  uint32_t fixed_len;
  uint32_t bucket4, bucket6;  // 1 = compute src_bucket for that family
  uint32_t tune;         // A/B knobs (PPTK_RX_TUNE): bit0 nt frame loads, bit1 no LDS record staging
  const void *zero;      // >= 16 zeroed device bytes (owned by the context)
  uint8_t *frames_w;     // tx batches: frames (writable) whose checksums are set
  // tx, two passes: the fields go to txside[i] (u16 offset, u16 value, twice;
  // offset 0xffff = none) instead of the frames, and launch_tx_apply writes
  // them after the streaming pass
  uint64_t *txside;
  // Derived by launch_rx for the GATHER kernels: branch-free descriptor
  // loads.  An absent array is read at index 0 of `zero` (msk = 0) and its
  // arithmetic stand-in (identity, i * stride_g, fixed_g) is added instead.
  const uint32_t *perm_ld;
  const uint64_t *off_ld;
  const uint16_t *len_ld;
  uint32_t perm_msk, off_msk, len_msk, fixed_g;
  uint64_t stride_g;
  // nullable (GATHER + perm): process perm[*range_lo .. *range_hi) only
  const uint32_t *range_lo, *range_hi;
  // 1: off/len are indexed by processing position (binned descriptors,
  // pptk_rx_batch_device_mixed), perm only gives the record index
  uint32_t by_pos;
  // header rewrite (pptk_tx_rewrite_device): rw[rw_one ? 0 : i], status
  const pptk_rewrite *rw;
  uint32_t rw_one;
  uint8_t *rw_status;
  // MSS clamping (pptk_tcp_mss_clamp_device): new MSS, PPTK_MSS_* flags;
  // the per-frame status goes to rw_status
  uint32_t mss, mss_flags;
  // binned launches of pptk_rx_batch_device_mixed: the binning's plan word
  // (device; bit 0 = binned; else bits 8-15 = the group whose launch runs
  // the whole batch in batch order), the caller's own descriptors for that
  // case (off0 nullable: stride), and this launch's group
  const uint32_t *plan;
  const uint64_t *off0;
  const uint16_t *len0;
  uint32_t plan_group;
  // global write phases of the streaming shapes (rx_kernel.hip): the period
  // in s_memrealtime ticks (10 ns); 0 = each tile's records at its end
  uint32_t phase_ticks;
  // oversubscribed grids (rx_capi.hip grid_for): blocks from tail_block on
  // (0: none) take the tiles from tail_tile on, in fewer tiles per wave, so
  // that the launch's last blocks are short
  uint32_t tail_block;
  uint64_t tail_tile;
#ifdef PPTK_RX_WAVE_TIMES
  uint64_t *wave_times;   // probe build: per wave (start, end) of the last launch
#endif
};

// Kernel variants: T lanes per frame in the streaming checksum phase, S
// 16-byte chunks per lane kept in registers (frames up to 16*T*S - 15
// bytes are summed without a tail loop).
enum RxVariant {
  RX_T4S1 = 0, RX_T4S2, RX_T16S2, RX_T16S6, RX_T32S3, RX_T64S2,
  RX_T16S7L, RX_T32S4L,   // chunk grid on 128-byte lines
  RX_T32S3D7, RX_T16S6D1, // prefetch-depth experiments
  RX_T8S2, RX_T16S4,      // length-group shapes (256 and 1024 bytes)
  RX_L4,                  // lane kernel: fixed stride, 16-byte aligned frames <= 64 bytes
  RX_M6,                  // mixed shapes: lanes binned by length inside each tile
  RX_NVARIANTS
};

// Wavefronts per block of the receive kernels (every wave works on its own
// tiles; no block-wide barrier).  PPTK_RX_WPB builds another size (A/B).
#ifndef PPTK_RX_WPB
#define PPTK_RX_WPB 4
#endif
constexpr int kWavesPerBlock = PPTK_RX_WPB;

// The lane kernel reads a batch packed at a 64-byte stride whose frames all
// span four chunks as contiguous 4 KB tiles (rx_kernel.hip lane_load);
// PPTK_RX_LANE_COAL=0 builds the per-frame loads only (A/B).
#ifndef PPTK_RX_LANE_COAL
#define PPTK_RX_LANE_COAL 1
#endif
__host__ __device__ inline bool lane_coalesced(uint64_t stride, uint32_t fixed_len) {
  return PPTK_RX_LANE_COAL && stride == 64 && ((fixed_len + 15u) >> 4) == 4;
}

// Length groups of pptk_rx_batch_device_mixed: group g holds the frames with
// len <= kGroupMaxLen[g] (and above the previous bound) and is streamed by
// kGroupVariant[g], whose 16*T*S-byte shape covers len + 15 bytes of chunk
// misalignment; the last group takes everything longer (tail loop).  Three
// groups: every finer split measured slower on CMIX (six groups 3.54 ms,
// 64..241 / rest 3.20, 64..113 / rest 3.13, one group 3.03, batch order
// 2.82; DESIGN.md "Binned CMIX"): each group launch sweeps the whole buffer
// for its frames, and the team-streamed kernel has no per-lane length
// divergence for binning to remove.
constexpr int kGroups = 3;
constexpr uint32_t kGroupMaxLen[kGroups] = {113, 1521, 0xffffffffu};
constexpr int kGroupVariant[kGroups] = {RX_T4S2, RX_T16S6, RX_T64S2};

hipError_t launch_rx(int variant, const RxKArgs &a, int grid, hipStream_t s);
// whether a variant's kernel holds records for the write phases (the
// streaming team shapes; RxKArgs::phase_ticks)
bool rx_variant_phased(int variant);
// tx second pass: frames[base(i) + off] = value (big-endian) for the
// fields txside[i] names; base(i) = off ? off[i] : i * stride
hipError_t launch_tx_apply(const uint64_t *txside, uint8_t *frames, const uint64_t *off,
                           uint64_t stride, uint64_t n, hipStream_t s);
hipError_t launch_rewrite(const RxKArgs &a, int grid, hipStream_t s);
hipError_t launch_mss_clamp(const RxKArgs &a, int grid, hipStream_t s);
int rx_variant_blocks_per_cu(int variant);

// Stable counting sort of 0..n-1 into kGroups length groups.  After it,
// bin_table(scratch, grid)[g] is the first position of group g in perm,
// [kGroups] = n and [kGroups + 1] the plan word (device memory, written by
// the launch).  With `adaptive` the binning first decides whether the batch
// is worth binning at all: only when it mixes frames of the last group
// (> 1521 bytes: batch order would stream every frame with the jumbo shape)
// with shorter ones.  Splitting 64..1521 B frames into groups was measured
// slower than batch order for every mix tried (CMIX, IMIX; DESIGN.md "Binned
// order"), so otherwise the plan word sends the whole batch, in batch order,
// to the launch of its highest non-empty group (perm = identity).
constexpr int kBinGrid = 2048;   // blocks of the binning sort (scratch layout)
// Optional binned copy of the descriptors (boff/blen null: perm only).
struct BinDesc {
  const uint64_t *off;   // nullable: frame i at i * stride
  uint64_t stride;
  uint64_t *boff;        // binned offsets (scratch), or null
  uint16_t *blen;        // binned lengths (scratch)
};
// Upper length bounds of groups 0 .. kGroups-2 (the last takes the rest):
// kGroupMaxLen, or a coarser grouping (equal neighbours = empty groups).
struct BinBounds {
  uint32_t b[kGroups - 1];
};
hipError_t launch_bin(const uint16_t *len, uint64_t n, uint32_t *perm,
                      void *scratch, hipStream_t s, int grid, const BinDesc &bdesc,
                      const BinBounds &bounds, bool adaptive);
// perm[i] = i (the processing order of a mixed call that runs batch order)
hipError_t launch_iota(uint32_t *perm, uint64_t n, hipStream_t s);
// the permutation inside the scratch (mixed calls without d_perm)
uint32_t *bin_perm(void *scratch, int grid, uint64_t n);
size_t bin_scratch_bytes(uint64_t n, int grid);
const uint32_t *bin_table(const void *scratch, int grid);
uint64_t *bin_desc_off(void *scratch, int grid);
uint16_t *bin_desc_len(void *scratch, int grid, uint64_t n);

// Batched ip_permitted / ipv6_permitted (rx_permit.hip).
struct PermitArgs {
  const pptk_rx_rec *recs;      // one of recs / recs32
  const pptk_rx_rec32 *recs32;
  const uint32_t *keys_in;      // or the rx kernel's dense keys (pptk_rx_dev_batch.d_key)
  uint64_t n;
  const uint8_t *subject;       // nullable: every parsed frame of the family
  uint32_t *tokens;             // hash_size counters
  uint8_t *verdict;             // 1 permitted, 0 denied, 2 not subject
  uint32_t hash_size;
  int family;                   // 4 or 6
  int ncu;                      // compute units (grid of the persistent verdict pass)
  int force_passes;             // 1: the four-pass path even where the fused one applies (tests)
};
size_t permit_scratch_bytes(uint64_t n, uint32_t hash_size);
hipError_t launch_permit(const PermitArgs &a, void *scratch, hipStream_t s);
// 0, or -ETIMEDOUT if a fused launch on this scratch since the last query
// aborted (synchronises s); -EIO on a HIP error
int permit_status(const void *scratch, hipStream_t s);
hipError_t launch_refill(uint32_t *tokens, uint32_t start, uint32_t end, uint32_t add,
                         uint32_t initial, hipStream_t s);

}  // namespace pptk
