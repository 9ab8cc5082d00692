// rx_capi.hip -- the C-ABI shim of libpptkrx.so (include/pptk_rx.h).
//
// Host side of the drop-in: a context per rx thread (own stream, own pinned
// staging), the device-resident batch entry point, the host-buffer batch
// entry point that an LDP rx loop calls between ldp_in_nextpkts() and
// ldp_in_deallocate_some() (reference ldp/ldprecv.c:60-70), and the
// length-binning helper.  Error convention: 0 or -errno, never abort on
// packet content.
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "../../include/hashseed.h"
#include "rx_internal.h"

using namespace pptk;

namespace {

constexpr uint32_t kStageAlign = 16;

}  // namespace

struct pptk_rx_ctx {
  int device = 0;
  pptk_rx_opts opts{};
  RxKArgs tmpl{};      // key/iphash part of the kernel arguments
  int ncu = 256;
  int bpc[RX_NVARIANTS] = {};
  int forced_variant = -1;
  int forced_flags = -1;
  // host-batch staging (pptk_rx_batch)
  hipStream_t stream = nullptr;
  size_t cap_pkts = 0, cap_bytes = 0;
  uint8_t *h_frames = nullptr, *d_frames = nullptr;
  uint64_t *h_off = nullptr, *d_off = nullptr;
  uint16_t *h_len = nullptr, *d_len = nullptr;
  pptk_rx_rec *h_recs = nullptr, *d_recs = nullptr;
};

static int hip_err(hipError_t e) { return e == hipSuccess ? 0 : -EIO; }

static uint64_t le64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

extern "C" {

const char *pptk_rx_version(void) { return "pptk_amd rx 0.1 gfx950"; }

void pptk_rx_opts_default(struct pptk_rx_opts *o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->device = 0;
  if (hash_seed_inited) memcpy(o->key, hash_seed, 16);
  o->iphash_size = 1;
  o->max_batch = 8192;
  o->max_frame = 9216;
}

int pptk_rx_ctx_create(struct pptk_rx_ctx **out, const struct pptk_rx_opts *opts) {
  if (!out || !opts) return -EINVAL;
  *out = nullptr;
  if (opts->iphash_bits4 > 32 || opts->iphash_bits6 > 128) return -EINVAL;
  if ((opts->iphash_bits4 || opts->iphash_bits6) &&
      (opts->iphash_size == 0 || (opts->iphash_size & (opts->iphash_size - 1))))
    return -EINVAL;
  if (opts->max_frame > 65535) return -EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || opts->device < 0 || opts->device >= ndev)
    return -EINVAL;
  pptk_rx_ctx *c = new (std::nothrow) pptk_rx_ctx();
  if (!c) return -ENOMEM;
  c->device = opts->device;
  c->opts = *opts;
  if (hipSetDevice(c->device) != hipSuccess) {
    delete c;
    return -EIO;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) c->ncu = prop.multiProcessorCount;
  for (int v = 0; v < RX_NVARIANTS; ++v) c->bpc[v] = rx_variant_blocks_per_cu(v);

  RxKArgs &t = c->tmpl;
  t.k0 = le64(opts->key);
  t.k1 = le64(opts->key + 8);
  t.bucket4 = opts->iphash_bits4 ? 1u : 0u;
  t.bucket6 = opts->iphash_bits6 ? 1u : 0u;
  t.hash_mask = opts->iphash_size ? opts->iphash_size - 1u : 0u;
  const uint32_t b4 = opts->iphash_bits4;
  t.mask4 = b4 >= 32 ? 0xffffffffu : (b4 == 0 ? 0u : ~((1u << (32 - b4)) - 1u));
  uint8_t m6[16];
  for (int b = 0; b < 16; ++b) {
    const int kept = std::min(std::max((int)opts->iphash_bits6 - 8 * b, 0), 8);
    m6[b] = (uint8_t)((0xff00u >> kept) & 0xffu);
  }
  t.mask6_0 = le64(m6);
  t.mask6_1 = le64(m6 + 8);
  *out = c;
  return 0;
}

static void free_staging(pptk_rx_ctx *c) {
  if (c->stream) (void)hipStreamDestroy(c->stream);
  (void)hipHostFree(c->h_frames);
  (void)hipHostFree(c->h_off);
  (void)hipHostFree(c->h_len);
  (void)hipHostFree(c->h_recs);
  (void)hipFree(c->d_frames);
  (void)hipFree(c->d_off);
  (void)hipFree(c->d_len);
  (void)hipFree(c->d_recs);
  c->stream = nullptr;
  c->h_frames = c->d_frames = nullptr;
  c->h_off = c->d_off = nullptr;
  c->h_len = c->d_len = nullptr;
  c->h_recs = c->d_recs = nullptr;
  c->cap_pkts = c->cap_bytes = 0;
}

void pptk_rx_ctx_destroy(struct pptk_rx_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  free_staging(c);
  delete c;
}

static int pick_variant(uint32_t span) {
  if (span <= 64) return RX_T4S1;
  if (span <= 128) return RX_T4S2;
  if (span <= 512) return RX_T16S2;
  if (span <= 1536) return RX_T16S6;
  return RX_T64S2;
}

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) {
    const uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

int pptk_rx_batch_device(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b,
                         void *stream) {
  if (!c || !b) return -EINVAL;
  if (b->n == 0) return 0;
  if (!b->d_frames || !b->d_recs) return -EINVAL;
  if (b->n > 0xffffffffull) return -EINVAL;  // indices are 32-bit (d_perm)
  if (!b->d_off && b->stride == 0 && b->n > 1) return -EINVAL;
  if (!b->d_len && b->fixed_len > 65535) return -EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return -EIO;

  // worst misalignment of a frame start inside a 16-byte chunk
  uint32_t mmax = 15;
  if (!b->d_off) {
    const uint64_t p = (uint64_t)(uintptr_t)b->d_frames;
    const uint64_t gg = gcd64(b->stride % 16 ? b->stride % 16 : 16, 16);
    mmax = (uint32_t)((p % gg) + 16 - gg);
  }
  uint32_t maxlen = b->d_len ? (b->max_len ? b->max_len : 65535u) : b->fixed_len;
  int variant = pick_variant(maxlen + mmax);
  static int force = -2;   // PPTK_RX_VARIANT: A/B override (results never change)
  if (force == -2) {
    const char *e = getenv("PPTK_RX_VARIANT");
    force = e ? atoi(e) : -1;
  }
  if (force >= 0 && force < RX_NVARIANTS) variant = force;
  if (c->forced_variant >= 0) variant = c->forced_variant;

  RxKArgs a = c->tmpl;
  a.frames = b->d_frames;
  a.off = b->d_off;
  a.len = b->d_len;
  a.perm = b->d_perm;
  a.stride = b->stride;
  a.fixed_len = b->fixed_len;
  a.n = b->n;
  a.recs = b->d_recs;
  a.hash = b->d_hash;

  // Memory policy (PPTK_RX_TUNE_*).  Default: non-temporal frame loads and
  // record stores for the streaming variants (frames are read once, records
  // written once: measured 4.47 -> 4.25 ms on C1500 in one process, see
  // DESIGN.md "Measurement log"), plain for the small-frame variants (nt
  // measured slower on C64).  PPTK_RX_TUNE overrides for A/B runs.
  static int tune = -2;
  if (tune == -2) {
    const char *e = getenv("PPTK_RX_TUNE");
    tune = e ? atoi(e) : -1;
  }
  a.tune = tune >= 0 ? (uint32_t)tune : (variant >= RX_T16S2 ? 33u : 0u);
  if (c->forced_flags >= 0) a.tune = (uint32_t)c->forced_flags;
  const uint64_t ntiles = (b->n + 63) / 64;
  const uint64_t want_blocks = (ntiles + 3) / 4;
  static int grid_mult = -1;
  if (grid_mult < 0) {
    const char *e = getenv("PPTK_RX_GRID_MULT");
    grid_mult = e ? std::max(1, atoi(e)) : 1;
  }
  const uint64_t cap = (uint64_t)c->ncu * (uint64_t)c->bpc[variant] * (uint64_t)grid_mult;
  const int grid = (int)std::min<uint64_t>(want_blocks, cap);
  return hip_err(launch_rx(variant, a, grid, (hipStream_t)stream));
}

int pptk_rx_set_tuning(struct pptk_rx_ctx *c, int variant, int flags) {
  if (!c || variant < -1 || variant >= RX_NVARIANTS || flags < -1 || flags > 255) return -EINVAL;
  c->forced_variant = variant;
  c->forced_flags = flags;
  return 0;
}

int pptk_rx_variant_count(void) { return RX_NVARIANTS; }

size_t pptk_rx_bin_scratch_bytes(uint64_t n) { return bin_scratch_bytes(n, 2048); }

int pptk_rx_bin_device(struct pptk_rx_ctx *c, const uint16_t *d_len, uint64_t n,
                       uint32_t *d_perm, void *d_scratch, void *stream) {
  if (!c || (n && (!d_len || !d_perm || !d_scratch))) return -EINVAL;
  if (n > 0xffffffffull) return -EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return -EIO;
  return hip_err(launch_bin(d_len, n, d_perm, d_scratch, (hipStream_t)stream, 2048));
}

static int ensure_staging(pptk_rx_ctx *c, size_t pkts, size_t bytes) {
  if (pkts <= c->cap_pkts && bytes <= c->cap_bytes) return 0;
  free_staging(c);
  pkts = std::max(pkts, (size_t)c->opts.max_batch);
  bytes = std::max(bytes, (size_t)c->opts.max_batch * ((c->opts.max_frame + 15) & ~15u));
  bytes += 64;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void **)&c->h_frames, bytes, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&c->h_off, pkts * 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&c->h_len, pkts * 2, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&c->h_recs, pkts * 64, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void **)&c->d_frames, bytes) != hipSuccess ||
      hipMalloc((void **)&c->d_off, pkts * 8) != hipSuccess ||
      hipMalloc((void **)&c->d_len, pkts * 2) != hipSuccess ||
      hipMalloc((void **)&c->d_recs, pkts * 64) != hipSuccess) {
    free_staging(c);
    return -ENOMEM;
  }
  c->cap_pkts = pkts;
  c->cap_bytes = bytes;
  return 0;
}

int pptk_rx_batch(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num,
                  struct pptk_rx_rec *recs) {
  if (!c || num < 0 || (num > 0 && (!pkts || !recs))) return -EINVAL;
  if (num == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -EIO;
  const uint32_t maxf = c->opts.max_frame ? c->opts.max_frame : 65535u;
  // gather: frames packed at 16-byte aligned offsets; over-long frames are
  // staged with length 0, which yields a MALFORMED-only record.
  size_t bytes = 0;
  for (int i = 0; i < num; ++i)
    if (pkts[i].data && pkts[i].sz <= maxf)
      bytes += (pkts[i].sz + kStageAlign - 1) & ~(size_t)(kStageAlign - 1);
  int rc = ensure_staging(c, (size_t)num, bytes);
  if (rc) return rc;
  size_t pos = 0;
  uint32_t maxlen = 0;
  for (int i = 0; i < num; ++i) {
    const bool ok = pkts[i].data && pkts[i].sz <= maxf;
    const uint32_t sz = ok ? pkts[i].sz : 0u;
    c->h_off[i] = pos;
    c->h_len[i] = (uint16_t)sz;
    if (sz) memcpy(c->h_frames + pos, pkts[i].data, sz);
    pos += (sz + kStageAlign - 1) & ~(size_t)(kStageAlign - 1);
    maxlen = std::max(maxlen, sz);
  }
  hipStream_t s = c->stream;
  if (hipMemcpyAsync(c->d_frames, c->h_frames, std::max<size_t>(pos, 16), hipMemcpyHostToDevice, s) !=
          hipSuccess ||
      hipMemcpyAsync(c->d_off, c->h_off, (size_t)num * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(c->d_len, c->h_len, (size_t)num * 2, hipMemcpyHostToDevice, s) != hipSuccess)
    return -EIO;
  pptk_rx_dev_batch b;
  memset(&b, 0, sizeof(b));
  b.d_frames = c->d_frames;
  b.d_off = c->d_off;
  b.d_len = c->d_len;
  b.max_len = maxlen;
  b.n = (uint64_t)num;
  b.d_recs = c->d_recs;
  rc = pptk_rx_batch_device(c, &b, s);
  if (rc) return rc;
  if (hipMemcpyAsync(c->h_recs, c->d_recs, (size_t)num * 64, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return -EIO;
  memcpy(recs, c->h_recs, (size_t)num * 64);
  return 0;
}

}  // extern "C"
