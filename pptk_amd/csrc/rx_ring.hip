// rx_ring.hip -- library-owned device rings, placed (include/pptk_rx.h,
// "Device rings").
//
// What the memory charges for the receive transform's record writes beside
// its frame-read stream depends on where the frame buffer and the record
// buffer sit physically in HBM: the same C1500 launch runs 4.0 ms on one
// (frames, records) pair and 4.8-5.1 ms on another, and a buffer keeps its
// class for its lifetime (DESIGN.md section 7 "Placement").  The class is a
// property of physical regions that a user process cannot see, and no
// kernel-side write pattern that fits on the chip avoids it (records staged
// in L2 and flushed as 256 KB runs, round 4: as slow as the direct 4 KB
// stores, profiles/r04/xstage/).  So a long-lived rx queue -- an LDP/netmap
// ring lives for the process (reference ldp/ldpnetmap.c:163-185) -- gets its
// device rings from this allocator, which measures the placement once: frame
// and record candidates are allocated behind spacers (so that they land in
// different regions), a synthetic batch of the ring's geometry is run on
// every (frames, records) pair, the fastest pair is kept and everything else
// freed.  The product path's default allocation is then the placed one.
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "rx_internal.h"

using namespace pptk;

namespace {

// Probe frames: Ethernet + IPv4 (DF, no options) + TCP (20 bytes) + a payload
// pattern, frame i at i * len, every field varying with i the way a real
// stream's do (ip_id, source address, source port, sequence number).  The
// checksum fields are left zero: the transform verifies them, and verifying
// a wrong checksum is the same work as verifying a right one.  One thread per
// output dword; bytes are computed one at a time (frames need not be 4-byte
// aligned).
__device__ __forceinline__ uint32_t probe_byte(uint64_t i, uint32_t k, uint32_t len) {
  const uint32_t tl = len - 14;
  switch (k) {
    case 0: case 6: return 0x02;
    case 5: return 0x01;
    case 11: return 0x02;
    case 12: return 0x08;
    case 14: return 0x45;
    case 16: return tl >> 8;
    case 17: return tl & 0xff;
    case 18: return (uint32_t)(i >> 8) & 0xff;
    case 19: return (uint32_t)i & 0xff;
    case 20: return 0x40;
    case 22: return 64;
    case 23: return 6;
    case 26: return 10;
    case 28: return (uint32_t)(i >> 8) & 0xff;
    case 29: return (uint32_t)i & 0xff;
    case 30: return 10;
    case 31: return 1;
    case 33: return 1;
    case 34: return 0x04 + (uint32_t)((i % 50000) >> 8);
    case 35: return (uint32_t)(i % 50000) & 0xff;
    case 37: return 80;
    case 38: return (uint32_t)(i >> 24) & 0xff;
    case 39: return (uint32_t)(i >> 16) & 0xff;
    case 40: return (uint32_t)(i >> 8) & 0xff;
    case 41: return (uint32_t)i & 0xff;
    case 46: return 0x50;
    case 47: return 0x10;
    case 48: return 0xff;
    case 49: return 0xff;
    default: return k >= 54 ? (uint32_t)(i * 131u + k) & 0xff : 0u;
  }
}

__global__ __launch_bounds__(256) void ring_fill_kernel(uint32_t *dst, uint64_t ndw, uint32_t len) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < ndw; w += (uint64_t)gridDim.x * 256) {
    const uint64_t o = w * 4;
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint64_t ob = o + b;
      v |= probe_byte(ob / len, (uint32_t)(ob % len), len) << (8 * b);
    }
    dst[w] = v;
  }
}

constexpr uint64_t kGiB = 1ull << 30;
constexpr double kScrubBytesPerS = 20e9;   // the driver's scrub of freed memory

void free_all(std::vector<void *> &v) {
  for (void *p : v)
    if (p) (void)hipFree(p);
  v.clear();
}

// One placement probe at a time per device: several rx queues of one GPU
// (a context each, reference ldp/ldprecvmt.c:16-67) setting up their rings
// at once would otherwise size their candidate sets from the same free
// memory, then fail each other's allocations and time their probes beside
// each other's.  Each call sees the memory the previous ones kept.
std::mutex g_place_mu[64];
std::mutex &place_mutex(int dev) { return g_place_mu[(unsigned)dev % 64u]; }

// The memory a call's candidates (and spacers) may take beyond the pair it
// keeps: `budget` if given, else `frac` of the device's free memory.
double cand_budget(uint64_t budget, size_t free_b, double frac) {
  return budget ? (double)std::min<uint64_t>(budget, free_b) : frac * (double)free_b;
}

}  // namespace

extern "C" {

int pptk_rx_ring_alloc(struct pptk_rx_ctx *c, const struct pptk_rx_ring_spec *sp,
                       struct pptk_rx_ring *out, void *stream) {
  if (!c || !sp || !out) return -EINVAL;
  memset(out, 0, sizeof(*out));
  const uint32_t rb = sp->rec_bytes;
  const uint32_t plen = sp->probe_len ? sp->probe_len : 1500;
  const uint32_t nf0 = sp->frame_cands ? sp->frame_cands : 3;
  const uint32_t nr0 = sp->rec_cands ? sp->rec_cands : 8;
  const uint32_t reps = sp->reps ? sp->reps : 3;
  if ((rb != 64 && rb != 32) || sp->frame_bytes == 0 || sp->nrec == 0 || plen < 64 ||
      plen > 1536 || nf0 > 8 || nr0 > 16 || reps > 20 || sp->nrec > 0xffffffffull ||
      (sp->flags & ~(uint32_t)(PPTK_RX_RING_SETTLE | PPTK_RX_RING_PROBE_HASH)) || sp->reserved)
    return -EINVAL;
  // the probe batch: fixed-stride frames of probe_len bytes over the frame
  // ring (up to nrec of them)
  const uint64_t n = std::min<uint64_t>(sp->nrec, sp->frame_bytes / plen);
  if (n == 0) return -EINVAL;
  DeviceScope dg(ctx_device(c));
  if (!dg.ok) return -EIO;
  std::lock_guard<std::mutex> plk(place_mutex(ctx_device(c)));
  const hipStream_t s = (hipStream_t)stream;
  // The frame ring is readable 64 bytes past its end (the kernels' 16-byte
  // chunk reads of a last frame, pptk_rx.h "Frames").
  const uint64_t fbytes = sp->frame_bytes + 64;
  const uint64_t rbytes = sp->nrec * rb;
  const uint64_t spacer_f = std::min<uint64_t>(8 * kGiB, std::max<uint64_t>(kGiB, fbytes / 2));
  const uint64_t spacer_r = std::min<uint64_t>(4 * kGiB, std::max<uint64_t>(256ull << 20, 4 * rbytes));
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return -EIO;
  if (fbytes + rbytes > free_b) return -ENOMEM;
  // candidates beyond the first pair only as far as the budget (default
  // 60 % of the free memory) allows
  uint32_t nf = nf0, nr = nr0;
  auto need = [&](uint32_t f, uint32_t r) {
    return (f - 1) * (fbytes + spacer_f) + r * (rbytes + spacer_r) + fbytes;
  };
  const double budget = cand_budget(sp->budget_bytes, free_b, 0.6);
  while (nf > 1 && (double)need(nf, nr) > budget) --nf;
  while (nr > 1 && (double)need(nf, nr) > budget) --nr;

  std::vector<void *> spacers, fc, rc;
  uint64_t allocated = 0;
  auto alloc = [&allocated](uint64_t bytes, std::vector<void *> &into) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    into.push_back(p);
    allocated += bytes;
    return true;
  };
  // frame candidate 0 and record candidate 0 are what a plain allocation
  // would give; every later candidate sits behind a spacer.  A candidate
  // that does not fit ends its list (the probe runs on the ones there are).
  for (uint32_t k = 0; k < nf; ++k)
    if ((k > 0 && !alloc(spacer_f, spacers)) || !alloc(fbytes, fc)) break;
  for (uint32_t k = 0; k < nr && !fc.empty(); ++k)
    if ((k > 0 && !alloc(spacer_r, spacers)) || !alloc(rbytes, rc)) break;
  if (fc.empty() || rc.empty()) {
    free_all(spacers);
    free_all(fc);
    free_all(rc);
    return -ENOMEM;
  }
  int err = 0;
  nf = (uint32_t)fc.size();
  nr = (uint32_t)rc.size();
  // the probe's dense hashes (PPTK_RX_RING_PROBE_HASH), allocated after the
  // candidates and freed with them
  void *hbuf = nullptr;
  if ((sp->flags & PPTK_RX_RING_PROBE_HASH) && alloc(n * 8, spacers)) hbuf = spacers.back();
  const uint64_t freed = allocated - fbytes - rbytes;   // all but the pair kept

  const uint64_t ndw = (n * plen + 3) / 4;
  for (void *f : fc) {
    hipLaunchKernelGGL(ring_fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t *)f, ndw, plen);
    if (hipGetLastError() != hipSuccess) err = -EIO;
  }
  std::vector<const uint8_t *> fptr(fc.size());
  for (size_t k = 0; k < fc.size(); ++k) fptr[k] = (const uint8_t *)fc[k];
  int bf = 0, br = 0;
  std::vector<float> ms((size_t)nf * nr, 0.f);
  if (err == 0) {
    pptk_rx_dev_batch b;
    memset(&b, 0, sizeof(b));
    b.d_frames = fptr[0];
    b.stride = plen;
    b.fixed_len = plen;
    b.max_len = plen;
    b.n = n;
    if (rb == 64) b.d_recs = (pptk_rx_rec *)rc[0];
    else b.d_recs32 = (pptk_rx_rec32 *)rc[0];
    b.d_hash = (uint64_t *)hbuf;
    err = pptk_rx_place_buffers(c, &b, fptr.data(), (int)nf, rc.data(), (int)nr, (int)reps, &bf,
                                &br, ms.data(), stream);
  }
  if (err != 0) {
    (void)hipStreamSynchronize(s);
    free_all(spacers);
    free_all(fc);
    free_all(rc);
    return err;
  }
  // keep the chosen pair, free the rest
  void *keep_f = fc[(size_t)bf], *keep_r = rc[(size_t)br];
  fc[(size_t)bf] = nullptr;
  rc[(size_t)br] = nullptr;
  free_all(spacers);
  free_all(fc);
  free_all(rc);
  out->d_frames = (uint8_t *)keep_f;
  out->frame_bytes = sp->frame_bytes;
  out->d_recs = keep_r;
  out->nrec = sp->nrec;
  out->rec_bytes = rb;
  out->device = ctx_device(c);
  out->frame_cands = nf;
  out->rec_cands = nr;
  out->chosen_frames = bf;
  out->chosen_recs = br;
  out->chosen_ms = ms[(size_t)bf * nr + br];
  out->first_ms = ms[0];
  out->probe_frames = n;
  out->freed_bytes = freed;
  if (sp->flags & PPTK_RX_RING_SETTLE) {
    // batches beside the driver's scrub of the freed candidates run up to
    // 9 % slower: wait it out
    const double sec = (double)freed / kScrubBytesPerS;
    std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(sec * 1e6)));
    out->settle_ms = (uint32_t)(sec * 1e3);
  }
  return 0;
}

int pptk_rx_ring_free(struct pptk_rx_ring *r) {
  if (!r) return -EINVAL;
  DeviceScope dg(r->device);
  if (r->d_frames) (void)hipFree(r->d_frames);
  if (r->d_recs) (void)hipFree(r->d_recs);
  memset(r, 0, sizeof(*r));
  return 0;
}

// The multi-GPU gather buffers, placed.  Per batch the all-gather lands
// (nranks - 1) shards of hashes in this GPU's HBM while the next batch
// streams its frames, and the kernel writes its own hashes into its slice:
// what those writes cost beside the frame stream depends on where the
// buffer sits, as for the records (one GPU, C1500: 4.62 vs 5.19 ms per
// batch with 940 MB of emulated gather writes beside it).  The
// two double-buffered gather buffers are the two halves of one region
// (placements come in runs of several GB, so both halves share the
// region's class).  Per candidate region (allocated behind spacers): the
// caller's batch is run with its hashes into each half's own slice in turn
// and, beside each launch on a second stream, a device copy of the bytes
// the gather would land in the rest of that half; the fastest region is
// kept, the rest freed.
int pptk_rx_gather_alloc(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b,
                         const struct pptk_rx_gather_spec *sp, struct pptk_rx_gather *out,
                         void *stream) {
  if (!c || !b || !sp || !out) return -EINVAL;
  memset(out, 0, sizeof(*out));
  const uint32_t ncand0 = sp->cands ? sp->cands : 8;
  const uint32_t reps = sp->reps ? sp->reps : 5;
  if (sp->nranks < 1 || sp->rank < 0 || sp->rank >= sp->nranks || sp->per_rank == 0 ||
      b->n > sp->per_rank || ncand0 > 16 || reps > 20 || sp->reserved ||
      (sp->flags & ~(uint32_t)PPTK_RX_RING_SETTLE) ||
      sp->per_rank > (1ull << 40) / (uint64_t)sp->nranks)
    return -EINVAL;
  DeviceScope dg(ctx_device(c));
  if (!dg.ok) return -EIO;
  std::lock_guard<std::mutex> plk(place_mutex(ctx_device(c)));
  const hipStream_t s = (hipStream_t)stream;
  const uint64_t nb = (uint64_t)sp->nranks * sp->per_rank * 8;   // one gather buffer
  const uint64_t lo = (uint64_t)sp->rank * sp->per_rank * 8, hi = lo + sp->per_rank * 8;
  const uint64_t spacer = std::min<uint64_t>(4 * kGiB, std::max<uint64_t>(256ull << 20, 4 * nb));
  const uint64_t srcb = std::max<uint64_t>(std::max(lo, nb - hi), 16);
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return -EIO;
  if (2 * nb + srcb > free_b) return -ENOMEM;
  uint32_t nc = ncand0;
  const double budget = cand_budget(sp->budget_bytes, free_b, 0.5);
  while (nc > 1 && (double)(nc * (2 * nb + spacer) + srcb) > budget) --nc;

  std::vector<void *> spacers, cands;
  void *src = nullptr;
  auto alloc = [](uint64_t bytes, std::vector<void *> &into) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    into.push_back(p);
    return true;
  };
  for (uint32_t k = 0; k < nc; ++k)
    if ((k > 0 && !alloc(spacer, spacers)) || !alloc(2 * nb, cands)) break;
  hipStream_t side = nullptr;
  hipEvent_t ev = nullptr, te[3] = {nullptr, nullptr, nullptr};
  int err = 0;
  if (cands.empty() || hipMalloc(&src, srcb) != hipSuccess) err = -ENOMEM;
  if (!err && (hipMemsetAsync(src, 0, srcb, s) != hipSuccess ||
               hipStreamCreateWithFlags(&side, hipStreamNonBlocking) != hipSuccess ||
               hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess))
    err = -EIO;
  for (int k = 0; k < 3 && !err; ++k)
    if (hipEventCreate(&te[k]) != hipSuccess) err = -EIO;
  nc = (uint32_t)cands.size();
  // One batch into half h of candidate k, then (second stream) the bytes the
  // gather would land in the rest of that half, beside the NEXT launch -- as
  // in an rx loop, where batch k's gather overlaps batch k + 1.
  auto batch = [&](uint32_t k, int h) {
    uint8_t *half = (uint8_t *)cands[k] + (uint64_t)h * nb;
    pptk_rx_dev_batch bb = *b;
    bb.d_hash = (uint64_t *)(half + lo);
    int e = pptk_rx_batch_device(c, &bb, stream);
    if (e) return e;
    if (hipEventRecord(ev, s) != hipSuccess || hipStreamWaitEvent(side, ev, 0) != hipSuccess ||
        (lo && hipMemcpyAsync(half, src, lo, hipMemcpyDeviceToDevice, side) != hipSuccess) ||
        (nb > hi &&
         hipMemcpyAsync(half + hi, src, nb - hi, hipMemcpyDeviceToDevice, side) != hipSuccess))
      return -EIO;
    return 0;
  };
  auto drain = [&]() {
    return hipStreamSynchronize(s) == hipSuccess && hipStreamSynchronize(side) == hipSuccess
               ? 0 : -EIO;
  };
  // Warm-up: clocks ramp over the first few hundred ms of sustained load;
  // without it the first candidates probed look slower than the rest.
  {
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; !err; ++r) {
      err = batch(0, r & 1);
      if (!err && (r & 7) == 7) {
        err = drain();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(300)) break;
      }
    }
  }
  // Rounds over the candidates (drift falls on all alike); per visit one
  // untimed batch (the previous candidate's gather copies are beside it),
  // then two timed by events on the batch stream: kernel durations with
  // this candidate's gather writes beside them.  Median per candidate.
  std::vector<std::vector<float>> samp(nc);
  for (uint32_t r = 0; r < reps && !err; ++r) {
    for (uint32_t k = 0; k < nc && !err; ++k) {
      if ((err = batch(k, 0)) != 0) break;
      if (hipEventRecord(te[0], s) != hipSuccess) err = -EIO;
      if (!err) err = batch(k, 1);
      if (!err && hipEventRecord(te[1], s) != hipSuccess) err = -EIO;
      if (!err) err = batch(k, 0);
      if (!err && hipEventRecord(te[2], s) != hipSuccess) err = -EIO;
      if (!err) err = drain();
      float m1 = 0.f, m2 = 0.f;
      if (!err && (hipEventElapsedTime(&m1, te[0], te[1]) != hipSuccess ||
                   hipEventElapsedTime(&m2, te[1], te[2]) != hipSuccess))
        err = -EIO;
      samp[k].push_back(m1);
      samp[k].push_back(m2);
    }
  }
  std::vector<float> ms(nc, 0.f);
  for (uint32_t k = 0; k < nc && !err; ++k) {
    std::vector<float> &v = samp[k];
    std::sort(v.begin(), v.end());
    ms[k] = v.empty() ? 0.f : v[v.size() / 2];
  }
  for (hipEvent_t x : te)
    if (x) (void)hipEventDestroy(x);
  if (side) {
    (void)hipStreamSynchronize(side);
    (void)hipStreamDestroy(side);
  }
  (void)hipStreamSynchronize(s);
  if (ev) (void)hipEventDestroy(ev);
  if (src) (void)hipFree(src);
  if (err) {
    free_all(spacers);
    free_all(cands);
    return err;
  }
  const uint32_t best = (uint32_t)(std::min_element(ms.begin(), ms.end()) - ms.begin());
  void *keep = cands[best];
  cands[best] = nullptr;
  uint64_t freed = (uint64_t)spacers.size() * spacer + (uint64_t)(nc - 1) * 2 * nb + srcb;
  free_all(spacers);
  free_all(cands);
  // the buffers start zeroed (the padding past the last rank's frames too)
  if (hipMemsetAsync(keep, 0, 2 * nb, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(keep);
    return -EIO;
  }
  out->d_out[0] = (uint64_t *)keep;
  out->d_out[1] = (uint64_t *)((uint8_t *)keep + nb);
  out->per_rank = sp->per_rank;
  out->nranks = sp->nranks;
  out->rank = sp->rank;
  out->device = ctx_device(c);
  out->cands = nc;
  out->chosen = (int32_t)best;
  out->chosen_ms = ms[best];
  out->first_ms = ms[0];
  out->freed_bytes = freed;
  for (uint32_t k = 0; k < nc; ++k) out->cand_ms[k] = ms[k];
  if (sp->flags & PPTK_RX_RING_SETTLE) {
    const double sec = (double)freed / kScrubBytesPerS;
    std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(sec * 1e6)));
    out->settle_ms = (uint32_t)(sec * 1e3);
  }
  return 0;
}

int pptk_rx_gather_free(struct pptk_rx_gather *g) {
  if (!g) return -EINVAL;
  DeviceScope dg(g->device);
  if (g->d_out[0]) (void)hipFree(g->d_out[0]);
  memset(g, 0, sizeof(*g));
  return 0;
}

}  // extern "C"
