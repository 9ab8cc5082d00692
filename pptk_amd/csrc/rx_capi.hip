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

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/hashseed.h"
#include "rx_internal.h"

using namespace pptk;

// One part of a host chunk's descriptors (pptk_rx_batch): the staging bytes
// its frames take and where they start, a ring chunk's span and frame bytes,
// the longest frame.
struct PartDesc {
  size_t bytes = 0, base = 0;
  size_t lo = SIZE_MAX, hi = 0, fbytes = 0;
  uint32_t maxlen = 0;
  // uniform frames: every frame of the part sz0 bytes (same), and at
  // p0 + k * stride (uni; k = its index in the part); each cleared at the
  // first frame that is not.  A staged chunk needs only `same` (the staging
  // puts equal frames at one stride), a ring chunk both.
  bool same = true, uni = true;
  uint32_t sz0 = 0;
  const uint8_t *p0 = nullptr;
  int64_t stride = 0;
  bool outside = false;   // a frame not (wholly) inside the candidate ring
};

// One half of the host-batch double buffer: pinned staging, device copies,
// and the chunk currently in flight on its stream.
struct RxSlot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  size_t cap_pkts = 0, cap_bytes = 0;
  size_t dev_cap = 0;   // d_frames bytes (grown for registered-ring spans)
  uint8_t *h_frames = nullptr, *d_frames = nullptr;
  uint64_t *h_off = nullptr, *d_off = nullptr;
  uint16_t *h_len = nullptr, *d_len = nullptr;
  pptk_rx_rec *h_recs = nullptr, *d_recs = nullptr;
  // device addresses of the pinned h_* buffers (direct small chunks)
  uint8_t *hd_frames = nullptr;
  uint64_t *hd_off = nullptr;
  uint16_t *hd_len = nullptr;
  pptk_rx_rec *hd_recs = nullptr;
  void *out = nullptr;   // caller's records of the chunk in flight
  size_t count = 0;
  size_t rec_bytes = 64;   // of the chunk in flight: 64 (pptk_rx_rec) or 32 (pptk_rx_rec32)
  bool busy = false;
  std::vector<PartDesc> parts;  // pptk_rx_batch's per-part descriptor sums
  std::unique_ptr<std::atomic<size_t>[]> run;   // the parts' running staging totals
  size_t run_cap = 0;
};

// The context's host worker threads (opts.gather_threads - 1 of them, started
// on the first host batch and kept): parallel_for(n, f) runs f(0..n-1)
// across them and the calling thread and returns when all are done.  The
// staged path's frame gather and record copy-out use it; starting threads
// per chunk instead cost more than the copies for small frames.
class WorkerPool {
 public:
  explicit WorkerPool(size_t nworkers) {
    try {
      for (size_t t = 0; t < nworkers; ++t) th_.emplace_back([this] { loop(); });
    } catch (...) {   // a thread could not be started: stop the others
      shutdown();
      throw;
    }
  }
  ~WorkerPool() { shutdown(); }
  size_t size() const { return th_.size() + 1; }
  void parallel_for(size_t n, const std::function<void(size_t)> &f) {
    if (n == 0) return;
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f;
      n_ = n;
      next_ = 0;
      left_ = n;
      gen = ++gen_;
    }
    cv_.notify_all();
    work(gen);
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  // Items are claimed under the mutex together with the job they belong to:
  // a worker still finishing generation k can never claim an index of
  // generation k + 1 (which starts only after every item of k completed) or
  // run one with a stale job pointer.  Items are ~256 frames or 1 MiB of
  // copying, so a lock per claim costs nothing measurable.
  void work(uint64_t gen) {
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      if (gen_ != gen || next_ >= n_) return;
      const size_t i = next_++;
      const std::function<void(size_t)> *job = job_;
      g.unlock();
      (*job)(i);
      g.lock();
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work(seen);
    }
  }
  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread &t : th_) t.join();
    th_.clear();
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)> *job_ = nullptr;
  size_t n_ = 0, left_ = 0, next_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// A host rx ring registered for zero-copy reads (hipHostRegister, mapped).
struct RxRing {
  uint8_t *host;
  size_t bytes;
  const uint8_t *dev;
};

struct pptk_rx_ctx {
  int device = 0;
  pptk_rx_opts opts{};
  RxKArgs tmpl{};      // key/iphash part of the kernel arguments
  void *d_zero = nullptr;  // 64 zeroed device bytes (RxKArgs::zero)
  // two-pass tx side arrays (8 B per frame): per call from this stream-
  // ordered pool (allocated and freed on the call's stream, so concurrent
  // tx calls on different streams never share one), or the caller's buffer
  hipMemPool_t txpool = nullptr;
  std::mutex txpool_mu;   // tx calls of one context may run on several threads
  uint64_t *d_txuser = nullptr;   // pptk_tx_set_side_buffer
  uint64_t txuser_n = 0;
  int ncu = 256;
  int coll_cus = 0;   // pptk_rx_stream_split: CUs the grids leave to the collective now
  // pptk_rx_stream_split's two streams, owned by the context: created by the
  // first split (or a split to another CU count before any communicator),
  // kept across pptk_rx_stream_split(0), destroyed by pptk_rx_ctx_destroy
  // after the communicator; split_cus = the collective stream's CUs
  hipStream_t split_rx = nullptr, split_coll = nullptr;
  int split_cus = 0;
  int bpc[RX_NVARIANTS] = {};
  int forced_variant = -1;
  int forced_flags = -1;   // the receive transform's memory policy, -1 automatic
  bool permit_passes = false;   // PPTK_RX_TUNE_PERMIT_PASSES set by pptk_rx_set_tuning
  int last_variant = -1;
  // pptk_rx_autotune's choice per automatic variant, for fixed-stride [0]
  // and offset-described [1] batches (-1: the automatic variant itself)
  int tuned[2][RX_NVARIANTS];
  // host-batch pipeline: pptk_rx_batch double-buffers over slots 0 and 1,
  // pptk_rx_batch_submit rotates over all of them (allocated on first use)
  RxSlot slot[PPTK_RX_MAX_INFLIGHT];
  int async_head = 0;  // slot of the oldest outstanding submission
  int async_n = 0;     // outstanding submissions (0..PPTK_RX_MAX_INFLIGHT)
  std::vector<RxRing> rings;
  WorkerPool *pool = nullptr;   // started by the first host batch
  // RCCL communicator (rx_comm.hip), or null; atomic: pptk_rx_comm_abort
  // may read it from another rx thread while this one creates it
  std::atomic<void *> comm{nullptr};
};

namespace pptk {
int ctx_device(const pptk_rx_ctx *c) { return c->device; }
std::atomic<void *> *ctx_comm_slot(pptk_rx_ctx *c) { return &c->comm; }
uint32_t ctx_comm_timeout_ms(const pptk_rx_ctx *c) {
  return c->opts.comm_timeout_ms ? c->opts.comm_timeout_ms : PPTK_RX_COMM_TIMEOUT_MS;
}
int ctx_coll_cap(const pptk_rx_ctx *c) { return c->split_coll ? c->split_cus : 0; }
}  // namespace pptk

// Streams pptk_rx_stream_split handed out, by owner (pptk_rx_stream_destroy
// refuses them: -EBUSY), and the ones a context destroy has since destroyed
// (a caller following the old contract -- destroy them after the context --
// gets 0 for those instead of a second hipStreamDestroy).
static std::mutex g_split_mu;
static std::unordered_map<hipStream_t, const pptk_rx_ctx *> g_split_owned;
static std::unordered_set<hipStream_t> g_split_retired;

// Destroy the context's split streams (after their work; the communicator
// that may have used the collective stream is gone or never existed).
static void drop_split_streams(pptk_rx_ctx *c) {
  hipStream_t s[2] = {c->split_rx, c->split_coll};
  {
    std::lock_guard<std::mutex> g(g_split_mu);
    for (hipStream_t x : s)
      if (x) {
        g_split_owned.erase(x);
        g_split_retired.insert(x);
      }
  }
  for (hipStream_t x : s)
    if (x) {
      (void)hipStreamSynchronize(x);
      (void)hipStreamDestroy(x);
    }
  c->split_rx = c->split_coll = nullptr;
  c->split_cus = 0;
}

static int hip_err(hipError_t e) { return e == hipSuccess ? 0 : -EIO; }

// An integer environment knob, read once (the callers keep it in a function-
// local static: initialised once, thread-safe, as rx threads may race on
// their first batches).
static long env_long(const char *name, long dflt) {
  const char *e = getenv(name);
  return e ? atol(e) : dflt;
}

// An A/B knob: read from the environment in experiment builds only
// (rx_internal.h kDiag); a product build uses the default.
#ifdef PPTK_RX_EXPERIMENTS
#define EXP_KNOB(name, dflt) env_long(name, dflt)
#else
#define EXP_KNOB(name, dflt) ((long)(dflt))
#endif

static uint64_t le64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

extern "C" {

const char *pptk_rx_version(void) { return "pptk_amd rx 0.6 gfx950"; }

int pptk_rx_abi(void) { return PPTK_RX_ABI; }

void pptk_rx_opts_default(struct pptk_rx_opts *o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->device = 0;
  if (hash_seed_inited) memcpy(o->key, hash_seed, 16);
  o->iphash_size = 1;
  o->max_batch = 8192;
  o->max_frame = 9216;
  o->comm_timeout_ms = PPTK_RX_COMM_TIMEOUT_MS;
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
  DeviceScope dg(c->device);
  if (!dg.ok) {
    delete c;
    return -EIO;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) c->ncu = prop.multiProcessorCount;
  for (int v = 0; v < RX_NVARIANTS; ++v) {
    c->bpc[v] = rx_variant_blocks_per_cu(v);
    c->tuned[0][v] = c->tuned[1][v] = -1;
  }
  if (hipMalloc(&c->d_zero, 64) != hipSuccess || hipMemset(c->d_zero, 0, 64) != hipSuccess) {
    (void)hipFree(c->d_zero);
    delete c;
    return -ENOMEM;
  }

  RxKArgs &t = c->tmpl;
  t.zero = c->d_zero;
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

static void free_slot(RxSlot &sl) {
  if (sl.stream) (void)hipStreamSynchronize(sl.stream);
  if (sl.done) (void)hipEventDestroy(sl.done);
  if (sl.stream) (void)hipStreamDestroy(sl.stream);
  (void)hipHostFree(sl.h_frames);
  (void)hipHostFree(sl.h_off);
  (void)hipHostFree(sl.h_len);
  (void)hipHostFree(sl.h_recs);
  (void)hipFree(sl.d_frames);
  (void)hipFree(sl.d_off);
  (void)hipFree(sl.d_len);
  (void)hipFree(sl.d_recs);
  sl = RxSlot();
}

static void free_staging(pptk_rx_ctx *c) {
  for (RxSlot &sl : c->slot) free_slot(sl);
}

void pptk_rx_ctx_destroy(struct pptk_rx_ctx *c) {
  if (!c) return;
  DeviceScope dg(c->device);
  comm_release(c);
  drop_split_streams(c);   // after the communicator that may have used them
  free_staging(c);
  delete c->pool;
  (void)hipFree(c->d_zero);
  if (c->txpool) {   // its frees are queued on the callers' streams
    (void)hipDeviceSynchronize();
    (void)hipMemPoolDestroy(c->txpool);
  }
  for (const RxRing &r : c->rings) (void)hipHostUnregister(r.host);
  delete c;
}

static int pick_variant(uint32_t span) {
  if (span <= 64) return RX_T4S1;
  if (span <= 128) return RX_T4S2;
  if (span <= 256) return RX_T8S2;
  if (span <= 512) return RX_T16S2;
  if (span <= 1024) return RX_T16S4;
  if (span <= 1536) return RX_T16S6;
  return RX_T64S2;
}

// The result-preserving memory-policy bits (pptk_rx.h).  The kernels also
// know diagnostic bits that skip work (record stores, the per-frame phase,
// half the record bytes, tx writes) for profiling; they are accepted only by
// a -DPPTK_RX_DIAG build, so a product library can never produce wrong
// records through pptk_rx_set_tuning or PPTK_RX_TUNE.
#ifdef PPTK_RX_DIAG
static constexpr uint32_t kTuneMask = 0xffffu;
#else
static constexpr uint32_t kTuneMask = PPTK_RX_TUNE_NT_LOADS | PPTK_RX_TUNE_NO_STAGING |
                                      PPTK_RX_TUNE_NT_STORES | PPTK_RX_TUNE_SC1_STORES |
                                      PPTK_RX_TUNE_BLOCKED | PPTK_RX_TUNE_PERMIT_PASSES;
#endif

// Memory policy (PPTK_RX_TUNE_*), from in-process A/B runs (DESIGN.md
// "Measurement log"): non-temporal record stores always (C64 0.468 -> 0.463
// ms, CMIX 3.05 -> 2.97 ms); non-temporal frame loads only for fixed-stride
// batches with the streaming variants (C1500 4.47 -> 4.25 ms; they cost 14 %
// on C64 and 10 % on offset-described CMIX).  PPTK_RX_TUNE overrides.
static long env_tune() {
  static const long tune = env_long("PPTK_RX_TUNE", -1);
  return tune;
}

static uint32_t pick_tune(const pptk_rx_ctx *c, int variant, bool gather, bool coal = false) {
  constexpr uint32_t rx_bits = kTuneMask & ~(uint32_t)PPTK_RX_TUNE_PERMIT_PASSES;
  if (c->forced_flags >= 0) return (uint32_t)c->forced_flags & rx_bits;
  // (an environment word holding only the rate limiter's bit leaves the
  // memory policy automatic, as pptk_rx_set_tuning does; any other word,
  // 0 included, forces the policy it names)
  const long tune = env_tune();
  if (tune >= 0 && tune != PPTK_RX_TUNE_PERMIT_PASSES) return (uint32_t)tune & rx_bits;
  // (the lane kernel on a packed run of 64-byte slots reads its tiles as
  // contiguous 1 KB runs, rx_kernel.hip lane_load: there non-temporal loads
  // pay, C64 0.3815 -> 0.3723 ms; on its per-frame loads they cost 22 %)
  const bool small = variant == RX_T4S1 || variant == RX_T4S2 || variant == RX_T8S2 ||
                     (variant == RX_L4 && !coal);
  return (small || gather) ? PPTK_RX_TUNE_NT_STORES
                           : (PPTK_RX_TUNE_NT_STORES | PPTK_RX_TUNE_NT_LOADS);
}

static int forced_variant(const pptk_rx_ctx *c) {
  // PPTK_RX_VARIANT: A/B override (results never change)
  static const long force = env_long("PPTK_RX_VARIANT", -1);
  if (c->forced_variant >= 0) return c->forced_variant;
  return force >= 0 && force < RX_NVARIANTS ? (int)force : -1;
}

// Blocks a launch may keep resident (the persistent grid).
static uint64_t resident_blocks(const pptk_rx_ctx *c, int variant);

// Grid of a launch: by default persistent (every block resident, its waves
// striding over the tiles).  tpw > 0: enough blocks that each wave takes
// about tpw tiles -- more than are resident, so the dispatcher hands out
// the later blocks as earlier ones finish (tiles_per_wave).
static int grid_for(const pptk_rx_ctx *c, int variant, uint64_t n, uint32_t tpw = 0) {
  const uint64_t ntiles = (n + 63) / 64;
  const uint64_t want_blocks = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
  if (tpw > 0) {
    const uint64_t per_block = (uint64_t)kWavesPerBlock * tpw;
    const uint64_t blocks = (ntiles + per_block - 1) / per_block;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(want_blocks,
                                                         std::max(blocks, resident_blocks(c, variant))));
  }
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(want_blocks, resident_blocks(c, variant)));
}

static uint64_t resident_blocks(const pptk_rx_ctx *c, int variant) {
  static const long grid_mult = std::max(1l, EXP_KNOB("PPTK_RX_GRID_MULT", 1));
  // the CUs pptk_rx_stream_split left to the collective (the batches'
  // stream cannot use them); PPTK_RX_RESERVE_CUS: that many CUs' worth of
  // resident blocks fewer without a mask (on its own it leaves no CU free:
  // the dispatcher spreads the smaller grid over every CU)
  static const int reserve_knob = (int)std::max(0l, EXP_KNOB("PPTK_RX_RESERVE_CUS", 0));
  const int reserve = std::max(reserve_knob, c->coll_cus);
  const uint64_t ncu = (uint64_t)std::max(1, c->ncu - std::min(reserve, c->ncu - 1));
  // (PPTK_RX_BPC: resident blocks per CU for every variant, A/B only)
  static const long bpc_knob = EXP_KNOB("PPTK_RX_BPC", 0);
  const uint64_t bpc = bpc_knob > 0 ? (uint64_t)bpc_knob : (uint64_t)c->bpc[variant];
  return ncu * bpc * (uint64_t)grid_mult;
}

// An oversubscribed launch's grid with its tail region (RxKArgs::tail_block):
// the last PPTK_RX_TAIL_PCT % of the tiles in blocks of PPTK_RX_TAIL_TPW
// tiles per wave, dispatched last, so that the launch does not end on a few
// long blocks (A/B knobs; 0 % = one region).
static int plan_grid(const pptk_rx_ctx *c, int variant, uint64_t n, uint32_t tpw, RxKArgs &a);

// Tiles per wave of an oversubscribed grid (grid_for), 0 = persistent.  The
// lane kernel, and the streaming shapes on offset-described batches (tiles
// of uneven duration), run faster when the dispatcher hands out blocks of a
// few tiles per wave than when every wave owns a fixed share of the batch:
// in-process A/B (profiles/r06/grid/), C64 0.3764 -> 0.3580 ms (8 tiles)
// and 0.3972 -> 0.3615 (4), CMIX T16S6 2.5245 -> 2.4591 (8) and 2.5189 ->
// 2.4509 (4), M6 on CMIX 2.5563 -> 2.4439 and on IMIX 1.3977 -> 1.3385 (8);
// C1500 (fixed stride, T32S3) is unchanged and T16S6 on it is slower
// (4.1465 -> 4.3680), so fixed-stride streaming stays persistent, as does
// the jumbo shape T64S2 (JMIX 3.9191 -> 4.0169 with 4 tiles, equal with 8).
static uint32_t tiles_per_wave(int variant, bool gather) {
  static const long lane = EXP_KNOB("PPTK_RX_LANE_TPW", 4);
  static const long strm = EXP_KNOB("PPTK_RX_GATHER_TPW", 8);
  static const long jumbo = EXP_KNOB("PPTK_RX_JUMBO_TPW", 0);   // T64S2 (A/B)
  static const long fixed = EXP_KNOB("PPTK_RX_FIXED_TPW", 0);   // fixed stride (A/B)
  if (variant == RX_L4) return (uint32_t)std::max(0l, lane);
  if (!gather) return (uint32_t)std::max(0l, fixed);
  return (uint32_t)std::max(0l, variant == RX_T64S2 ? jumbo : strm);
}

static int plan_grid(const pptk_rx_ctx *c, int variant, uint64_t n, uint32_t tpw, RxKArgs &a) {
  a.tail_block = 0;
  a.tail_tile = 0;
  const int grid = grid_for(c, variant, n, tpw);
  static const long pct = EXP_KNOB("PPTK_RX_TAIL_PCT", 0);
  static const long ttpw = EXP_KNOB("PPTK_RX_TAIL_TPW", 1);
  if (tpw == 0 || pct <= 0 || pct >= 100 || ttpw <= 0) return grid;
  const uint64_t ntiles = (n + 63) / 64;
  const uint64_t t2 = ntiles * (uint64_t)pct / 100, t1 = ntiles - t2;
  const uint64_t w1 = (uint64_t)kWavesPerBlock * tpw, w2 = (uint64_t)kWavesPerBlock * (uint64_t)ttpw;
  const uint64_t b1 = (t1 + w1 - 1) / w1, b2 = (t2 + w2 - 1) / w2;
  // (a batch too small to fill the chip twice over keeps one region)
  if (t2 == 0 || b1 < 2 * resident_blocks(c, variant) || b1 + b2 > 0x7fffffffull) return grid;
  a.tail_block = (uint32_t)b1;
  a.tail_tile = t1;
  return (int)(b1 + b2);
}

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) {
    const uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

static int check_batch(const pptk_rx_ctx *c, const pptk_rx_dev_batch *b) {
  if (!c || !b) return -EINVAL;
  if (b->n == 0) return 0;
  if (!b->d_frames || (!b->d_recs && !b->d_recs32)) return -EINVAL;
  if (b->n > 0xffffffffull) return -EINVAL;  // indices are 32-bit (d_perm)
  if (!b->d_off && b->stride == 0 && b->n > 1) return -EINVAL;
  if (!b->d_len && b->fixed_len > 65535) return -EINVAL;
  return 0;
}

static RxKArgs batch_args(const pptk_rx_ctx *c, const pptk_rx_dev_batch *b) {
  RxKArgs a = c->tmpl;
  a.frames = b->d_frames;
  a.off = b->d_off;
  a.len = b->d_len;
  a.perm = b->d_perm;
  a.stride = b->stride;
  a.fixed_len = b->fixed_len;
  a.n = b->n;
  a.recs = b->d_recs;
  a.recs32 = b->d_recs32;
  a.hash = b->d_hash;
  a.frag = b->d_frag;
  a.key = b->d_key;
  return a;
}

// The automatic kernel variant for a device batch: the lane kernel for
// fixed-stride 16-byte-aligned frames of at most 64 bytes, else the team
// shape sized for the longest frame plus its worst misalignment.
static int auto_variant(const pptk_rx_dev_batch *b, bool *lane_ok_out) {
  // worst misalignment of a frame start inside a 16-byte chunk
  uint32_t mmax = 15;
  if (!b->d_off) {
    const uint64_t p = (uint64_t)(uintptr_t)b->d_frames;
    const uint64_t gg = gcd64(b->stride % 16 ? b->stride % 16 : 16, 16);
    mmax = (uint32_t)((p % gg) + 16 - gg);
  }
  const uint32_t maxlen = b->d_len ? (b->max_len ? b->max_len : 65535u) : b->fixed_len;
  // the lane kernel takes fixed-stride batches of small frames that all
  // start on a 16-byte boundary (mmax == 0: aligned buffer and stride)
  // (and write no fragment side records: those come from lane_generic)
  // (an empty frame reads only the chunk holding its start, as the header
  // allows)
  const bool lane_ok = !b->d_off && !b->d_len && !b->d_perm && !b->d_frag && mmax == 0 &&
                       b->fixed_len <= 64;
  if (lane_ok_out) *lane_ok_out = lane_ok;
  return lane_ok ? RX_L4 : pick_variant(maxlen + mmax);
}

// The write-phase period of a launch (rx_kernel.hip "Global write phases"):
// ~0.75 of the time one wave takes for one 64-frame tile, estimated from the
// tile's frame bytes (fixed-stride batches: 64 strides; offset-described
// ones: 64 frames of half the max_len hint, as for lengths spread evenly up
// to it), the waves of the grid, and ~5.5 TB/s of frame stream.  Measured:
// the best periods lie at 0.6-0.9 of a tile (profiles/r05/w: C1500 30-40 us
// against 47-51 us tiles, CMIX 15-20 us against 20 us).  0 (off) for the
// small-frame shapes, permuted batches (records scatter) and tx batches.
static uint32_t phase_ticks_for(const pptk_rx_dev_batch *b, int variant, int grid) {
  static const long force = EXP_KNOB("PPTK_RX_PHASE_TICKS", -1);
  if (force >= 0) return (uint32_t)force;
  if (!rx_variant_phased(variant) || b->d_perm || (!b->d_recs && !b->d_recs32)) return 0;
  const uint64_t maxlen = b->d_len ? (b->max_len ? b->max_len : 1518u) : b->fixed_len;
  // (a stride far past any frame only lengthens the estimate; capped so the
  // product below cannot overflow)
  const uint64_t tile_bytes =
      64 * (b->d_off ? std::max<uint64_t>(64, maxlen / 2)
                     : std::min<uint64_t>(std::max<uint64_t>(b->stride, 64), 1u << 20));
  const uint64_t waves = (uint64_t)grid * kWavesPerBlock;
  const uint64_t ticks = tile_bytes * waves * 3 / 4 / 55000;   // 5.5 TB/s = 55 000 B per tick
  return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ticks, 100), 1000000);
}

#ifdef PPTK_RX_WAVE_TIMES
// probe build (tools/wave_times.py): every wave's (start, end) clock of the
// last launch
static uint64_t *g_wave_times = nullptr;
static int g_wave_count = 0;
extern "C" int pptk_rx_wave_times(uint64_t *host, int max_waves) {
  if (!g_wave_times) return -EINVAL;
  const int n = std::min(max_waves, g_wave_count);
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(host, g_wave_times, (size_t)n * 16, hipMemcpyDeviceToHost) != hipSuccess)
    return -EIO;
  return n;
}
#endif

static int launch_batch(pptk_rx_ctx *c, const pptk_rx_dev_batch *b, int variant, void *stream) {
  RxKArgs a = batch_args(c, b);
  a.tune = pick_tune(c, variant, b->d_off || b->d_len || b->d_perm,
                     variant == RX_L4 && lane_coalesced(b->stride, b->fixed_len));
  c->last_variant = variant;
  const bool gather = b->d_off || b->d_len || b->d_perm;
  const int grid = plan_grid(c, variant, b->n, tiles_per_wave(variant, gather), a);
  // (the period follows the waves resident at once, not the whole grid)
  a.phase_ticks = phase_ticks_for(
      b, variant, (int)std::min<uint64_t>((uint64_t)grid, resident_blocks(c, variant)));
#ifdef PPTK_RX_WAVE_TIMES
  if (!g_wave_times && hipMalloc(&g_wave_times, (size_t)65536 * 16) != hipSuccess) return -ENOMEM;
  if (grid * kWavesPerBlock > 65536) return -EINVAL;
  a.wave_times = g_wave_times;
  g_wave_count = grid * kWavesPerBlock;
#endif
  return hip_err(launch_rx(variant, a, grid, (hipStream_t)stream));
}

int pptk_rx_batch_device(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b,
                         void *stream) {
  int rc = check_batch(c, b);
  if (rc || b->n == 0) return rc;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  bool lane_ok = false;
  int variant = auto_variant(b, &lane_ok);
  const int tv = c->tuned[b->d_off || b->d_len || b->d_perm ? 1 : 0][variant];
  if (tv >= 0) variant = tv;                  // pptk_rx_autotune's choice
  const int fv = forced_variant(c);
  if (fv >= 0) variant = fv;
  if (variant == RX_L4 && !lane_ok) variant = auto_variant(b, nullptr);   // (a team shape)
  return launch_batch(c, b, variant, stream);
}

// Interchangeable shapes per automatic variant (same frame capacity, same
// results: every variant is parity-tested on every fixture).  Which is
// fastest depends on what the record writes cost (which follows the record
// buffer's placement): where they are expensive (the
// read/write-mix speed of light ~4.8 ms for C1500) T32S3D7 ran C1500 6 %
// faster than T16S6; T16S6 was chosen where the mix costs ~4.0 ms.  The
// 1536-byte class is the one measured.
static int autotune_candidates(int variant, bool gather, int cand[8]) {
  int n = 0;
  cand[n++] = variant;
  if (variant == RX_T16S6) {
    cand[n++] = RX_T32S3;
    cand[n++] = RX_T32S3D7;
    cand[n++] = RX_T16S7L;
    if (gather) cand[n++] = RX_M6;   // mixed lengths: lanes binned inside the tile
  }
  return n;
}

int pptk_rx_autotune(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b, int reps,
                     void *stream) {
  int rc = check_batch(c, b);
  if (rc || b->n == 0) return rc;
  if (reps < 1 || reps > 100) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  const int base = auto_variant(b, nullptr);
  const int g = b->d_off || b->d_len || b->d_perm ? 1 : 0;
  int cand[8];
  const int nc = autotune_candidates(base, g == 1, cand);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return -EIO;
  }
  const hipStream_t s = (hipStream_t)stream;
  // Candidates interleaved round by round (two untimed warm-up rounds), so
  // that clock and thermal drift during the probe fall on all of them alike;
  // the fastest median wins, but a shape other than the automatic one must
  // beat it by 1 % (noise never moves the choice away from candidate 0).
  std::vector<std::vector<float>> ms((size_t)nc);
  for (int r = 0; r < reps + 2 && rc == 0; ++r) {
    for (int k = 0; k < nc && rc == 0; ++k) {
      if (hipEventRecord(e0, s) != hipSuccess) rc = -EIO;
      if (rc == 0) rc = launch_batch(c, b, cand[k], stream);
      if (rc == 0 && (hipEventRecord(e1, s) != hipSuccess ||
                      hipEventSynchronize(e1) != hipSuccess))
        rc = -EIO;
      float t = 0.f;
      if (rc == 0 && r >= 2 && hipEventElapsedTime(&t, e0, e1) == hipSuccess)
        ms[(size_t)k].push_back(t);
    }
  }
  int best = base;
  if (rc == 0 && !ms[0].empty()) {
    std::vector<float> med((size_t)nc, 1e30f);
    for (int k = 0; k < nc; ++k) {
      if (ms[(size_t)k].empty()) continue;
      std::sort(ms[(size_t)k].begin(), ms[(size_t)k].end());
      med[(size_t)k] = ms[(size_t)k][ms[(size_t)k].size() / 2];
    }
    int kb = 0;
    for (int k = 1; k < nc; ++k)
      if (med[(size_t)k] < med[(size_t)kb]) kb = k;
    if (kb != 0 && med[(size_t)kb] < 0.99f * med[0]) best = cand[kb];
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc == 0) c->tuned[g][base] = best == base ? -1 : best;
  return rc;
}

int pptk_rx_place_buffers(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b,
                          const uint8_t *const *fr, int nf, void *const *rc_, int nr, int reps,
                          int *best_f, int *best_r, float *ms_out, void *stream) {
  if (!c || !b || !fr || !rc_ || !best_f || !best_r || nf < 1 || nf > 16 || nr < 1 ||
      nr > 64 || nf * nr > 256 || reps < 1 || reps > 100)
    return -EINVAL;
  for (int k = 0; k < nf; ++k)
    if (!fr[k]) return -EINVAL;
  for (int k = 0; k < nr; ++k)
    if (!rc_[k]) return -EINVAL;
  pptk_rx_dev_batch t = *b;
  const bool c32 = b->d_recs32 != nullptr;
  t.d_frames = fr[0];
  t.d_recs = c32 ? nullptr : (pptk_rx_rec *)rc_[0];
  t.d_recs32 = c32 ? (pptk_rx_rec32 *)rc_[0] : nullptr;
  int rc = check_batch(c, &t);
  if (rc || b->n == 0) {
    if (rc == 0) *best_f = *best_r = 0;
    return rc;
  }
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return -EIO;
  }
  const hipStream_t s = (hipStream_t)stream;
  const int np = nf * nr;
  std::vector<std::vector<float>> ms((size_t)np);
  // pairs interleaved round by round, so that clock drift during the probe
  // falls on all of them alike; round 0 is the warm-up
  for (int r = 0; r <= reps && rc == 0; ++r) {
    for (int p = 0; p < np && rc == 0; ++p) {
      t.d_frames = fr[p / nr];
      if (c32) t.d_recs32 = (pptk_rx_rec32 *)rc_[p % nr];
      else t.d_recs = (pptk_rx_rec *)rc_[p % nr];
      if (hipEventRecord(e0, s) != hipSuccess) rc = -EIO;
      if (rc == 0) rc = pptk_rx_batch_device(c, &t, stream);
      if (rc == 0 && (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess))
        rc = -EIO;
      float x = 0.f;
      if (rc == 0 && r > 0 && hipEventElapsedTime(&x, e0, e1) == hipSuccess)
        ms[(size_t)p].push_back(x);
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc) return rc;
  int bp = 0;
  float bm = 1e30f;
  for (int p = 0; p < np; ++p) {
    std::vector<float> &v = ms[(size_t)p];
    std::sort(v.begin(), v.end());
    const float med = v.empty() ? 1e30f : v[v.size() / 2];
    if (ms_out) ms_out[p] = med;
    if (med < bm) {
      bm = med;
      bp = p;
    }
  }
  *best_f = bp / nr;
  *best_r = bp % nr;
  return 0;
}

int pptk_rx_place_records(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b,
                          void *const *cands, int ncand, int reps, int *best, float *ms_out,
                          void *stream) {
  if (!b || !best) return -EINVAL;
  const uint8_t *f0 = b->d_frames;
  int bf = 0;
  return pptk_rx_place_buffers(c, b, &f0, 1, cands, ncand, reps, &bf, best, ms_out, stream);
}

// Tx in two passes (fixed-stride batches): the streaming pass records each
// frame's checksum fields in a side array (8 B per frame) and a second
// kernel writes them, so that the 2-byte field writes do not land beside
// the 25 GB read stream (DESIGN.md "Secondary kernels").
// PPTK_TX_TWO_PASS=0: the fields are stored in place by the streaming pass
// (A/B).
static bool tx_two_pass() {
  static const long v = EXP_KNOB("PPTK_TX_TWO_PASS", 1);
  return v != 0;
}

int pptk_tx_cksum_device(struct pptk_rx_ctx *c, uint8_t *d_frames, const uint64_t *d_off,
                         const uint16_t *d_len, uint64_t stride, uint32_t fixed_len,
                         uint64_t n, uint32_t max_len, void *stream) {
  if (!c || n > 0xffffffffull) return -EINVAL;
  if (n == 0) return 0;
  if (!d_frames || (!d_off && stride == 0 && n > 1) || (!d_len && fixed_len > 65535))
    return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  pptk_rx_dev_batch b;
  memset(&b, 0, sizeof(b));
  b.d_frames = d_frames;
  b.d_off = d_off;
  b.d_len = d_len;
  b.stride = stride;
  b.fixed_len = fixed_len;
  b.max_len = max_len;
  b.n = n;
  uint32_t mmax = 15;
  if (!d_off) {
    const uint64_t p = (uint64_t)(uintptr_t)d_frames;
    const uint64_t gg = gcd64(stride % 16 ? stride % 16 : 16, 16);
    mmax = (uint32_t)((p % gg) + 16 - gg);
  }
  const uint32_t maxlen = d_len ? (max_len ? max_len : 65535u) : fixed_len;
  int variant = pick_variant(maxlen + mmax);
  const bool two_pass = !d_off && tx_two_pass();
  if (two_pass) {
    // the streaming pass of a two-pass batch moves what the receive
    // transform moves minus most of the writes: pptk_rx_autotune's choice
    // for this shape applies (T32S3D7 5.14 ms vs T16S6 5.30 on C1500,
    // DESIGN.md "Secondary kernels")
    const int tv = c->tuned[0][variant];
    if (tv >= 0 && tv != RX_L4) variant = tv;
  }
  const int fv = forced_variant(c);
  if (fv >= 0 && fv != RX_L4) variant = fv;   // the lane kernel has no tx mode
  RxKArgs a = batch_args(c, &b);
  a.frames_w = d_frames;
  c->last_variant = variant;
  a.tune = c->forced_flags >= 0 ? (uint32_t)c->forced_flags & kTuneMask
                                : pick_tune(c, variant, d_off || d_len) &
                                      ~(uint32_t)PPTK_RX_TUNE_NT_LOADS;
  hipStream_t s = (hipStream_t)stream;
  if (two_pass) {
    // Fixed-stride batches: the streaming pass writes nothing into the
    // frames (so it may use non-temporal loads, as the receive transform
    // does); the fields go to the context's side array and a second pass
    // writes them.  Offset-described batches keep the in-place stores:
    // their streaming pass is slower with non-temporal loads, and the
    // fields stored beside it cost less than the second pass.
    if (c->forced_flags < 0)
      a.tune = pick_tune(c, variant, false);
    uint64_t *side = c->d_txuser && c->txuser_n >= n ? c->d_txuser : nullptr;
    const bool pooled = side == nullptr;
    if (pooled) {   // stream-ordered: this call's own array, freed behind it
      hipMemPool_t pool;
      {
        // created once, by whichever tx call comes first (two threads'
        // first calls may race)
        std::lock_guard<std::mutex> g(c->txpool_mu);
        if (!c->txpool) {
          hipMemPoolProps pp;
          memset(&pp, 0, sizeof(pp));
          pp.allocType = hipMemAllocationTypePinned;
          pp.location.type = hipMemLocationTypeDevice;
          pp.location.id = c->device;
          hipMemPool_t np = nullptr;
          if (hipMemPoolCreate(&np, &pp) != hipSuccess) return -ENOMEM;
          uint64_t keep = UINT64_MAX;   // keep freed blocks for the next call
          (void)hipMemPoolSetAttribute(np, hipMemPoolAttrReleaseThreshold, &keep);
          c->txpool = np;
        }
        pool = c->txpool;
      }
      if (hipMallocFromPoolAsync((void **)&side, n * 8, pool, s) != hipSuccess)
        return -ENOMEM;
    }
    a.txside = side;
    hipError_t e = launch_rx(variant, a, grid_for(c, variant, n), s);
    if (e == hipSuccess) e = launch_tx_apply(side, d_frames, d_off, stride, n, s);
    if (pooled && hipFreeAsync(side, s) != hipSuccess && e == hipSuccess) e = hipErrorUnknown;
    return hip_err(e);
  }
  return hip_err(launch_rx(variant, a, grid_for(c, variant, n), s));
}

int pptk_tx_set_side_buffer(struct pptk_rx_ctx *c, void *d_side, uint64_t frames) {
  if (!c || (!d_side && frames) || ((uintptr_t)d_side & 7u)) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  c->d_txuser = (uint64_t *)d_side;
  c->txuser_n = d_side ? frames : 0;
  return 0;
}

int pptk_tx_rewrite_device(struct pptk_rx_ctx *c, uint8_t *d_frames, const uint64_t *d_off,
                           const uint16_t *d_len, uint64_t stride, uint32_t fixed_len,
                           uint64_t n, const struct pptk_rewrite *d_rw, uint64_t rw_count,
                           uint8_t *d_status, void *stream) {
  if (!c || n > 0xffffffffull) return -EINVAL;
  if (n == 0) return 0;
  if (!d_frames || !d_rw || (rw_count != 1 && rw_count != n) ||
      (!d_off && stride == 0 && n > 1) || (!d_len && fixed_len > 65535))
    return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  RxKArgs a = c->tmpl;
  a.frames = d_frames;
  a.frames_w = d_frames;
  a.off = d_off;
  a.len = d_len;
  a.stride = stride;
  a.fixed_len = fixed_len;
  a.n = n;
  a.rw = d_rw;
  a.rw_one = rw_count == 1 ? 1u : 0u;
  a.rw_status = d_status;
  const uint64_t blocks = (n + 255) / 256;
  const int grid = (int)std::min<uint64_t>(blocks, (uint64_t)c->ncu * 8);
  return hip_err(launch_rewrite(a, grid, (hipStream_t)stream));
}

int pptk_tcp_mss_clamp_device(struct pptk_rx_ctx *c, uint8_t *d_frames, const uint64_t *d_off,
                              const uint16_t *d_len, uint64_t stride, uint32_t fixed_len,
                              uint64_t n, uint16_t mss, uint32_t flags, uint8_t *d_status,
                              void *stream) {
  if (!c || n > 0xffffffffull) return -EINVAL;
  if (n == 0) return 0;
  if (!d_frames || (flags & ~PPTK_MSS_SYN_ONLY) || (!d_off && stride == 0 && n > 1) ||
      (!d_len && fixed_len > 65535))
    return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  RxKArgs a = c->tmpl;
  a.frames = d_frames;
  a.frames_w = d_frames;
  a.off = d_off;
  a.len = d_len;
  a.stride = stride;
  a.fixed_len = fixed_len;
  a.n = n;
  a.mss = mss;
  a.mss_flags = flags;
  a.rw_status = d_status;
  const uint64_t blocks = (n + 255) / 256;
  const int grid = (int)std::min<uint64_t>(blocks, (uint64_t)c->ncu * 8);
  return hip_err(launch_mss_clamp(a, grid, (hipStream_t)stream));
}

// The length groups of the mixed path: kGroupMaxLen, or (A/B experiment)
// PPTK_RX_BIN_BOUNDS="b0,b1", non-decreasing upper bounds of groups 0 and 1
// (equal neighbours leave a group empty; it is not launched).
static const BinBounds &bin_bounds() {
  static const BinBounds bb = [] {
    BinBounds r;
    for (int k = 0; k < kGroups - 1; ++k) r.b[k] = kGroupMaxLen[k];
#ifdef PPTK_RX_EXPERIMENTS
    const char *e = getenv("PPTK_RX_BIN_BOUNDS");
#else
    const char *e = nullptr;
#endif
    if (!e) return r;
    BinBounds t = r;
    for (int k = 0; k < kGroups - 1; ++k) {
      char *end = nullptr;
      const unsigned long v = strtoul(e, &end, 10);
      if (end == e || v > 65535 || (k && v < t.b[k - 1])) return r;
      t.b[k] = (uint32_t)v;
      e = *end == ',' ? end + 1 : end;
    }
    return t;
  }();
  return bb;
}

static bool default_bounds(const BinBounds &bb) {
  for (int k = 0; k < kGroups - 1; ++k)
    if (bb.b[k] != kGroupMaxLen[k]) return false;
  return true;
}

int pptk_rx_batch_device_mixed(struct pptk_rx_ctx *c, const struct pptk_rx_dev_batch *b,
                               uint32_t *d_perm, void *d_scratch, void *stream) {
  int rc = check_batch(c, b);
  if (rc || b->n == 0) return rc;
  if (!b->d_len || !d_scratch) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  const hipStream_t s = (hipStream_t)stream;
  const BinBounds &bb = bin_bounds();
  const bool dflt = default_bounds(bb);
  if (b->max_len && b->max_len <= bb.b[kGroups - 2]) {
    // Every frame fits the 1536-byte shape (by the hint; a wrong hint costs
    // speed, never results): no length group is worth a launch of its own
    // (DESIGN.md "Binned order"), so batch order, as pptk_rx_batch_device.
    pptk_rx_dev_batch t = *b;
    t.d_perm = nullptr;
    if ((rc = pptk_rx_batch_device(c, &t, stream)) != 0) return rc;
    return d_perm ? hip_err(launch_iota(d_perm, b->n, s)) : 0;
  }
  uint32_t *perm = d_perm ? d_perm : bin_perm(d_scratch, kBinGrid, b->n);
  // the binning also lays the descriptors out in binned order (scratch), so
  // the group launches stream them instead of gathering them through perm
  BinDesc bd{b->d_off, b->stride, bin_desc_off(d_scratch, kBinGrid),
             bin_desc_len(d_scratch, kBinGrid, b->n)};
  hipError_t e = launch_bin(b->d_len, b->n, perm, d_scratch, s, kBinGrid, bd, bb, true);
  if (e != hipSuccess) return -EIO;
  RxKArgs a = batch_args(c, b);
  a.perm = perm;
  a.off = bd.boff;
  a.len = bd.blen;
  a.by_pos = 1;
  const uint32_t *tab = bin_table(d_scratch, kBinGrid);
  a.plan = tab + kGroups + 1;
  a.off0 = b->d_off;
  a.len0 = b->d_len;
  const uint32_t maxlen = b->max_len ? b->max_len : 65535u;
  const int fv = forced_variant(c);
  for (int g = 0; g < kGroups; ++g) {
    // the group holding max_len also takes every group above it (all empty
    // when the hint is right; a wrong hint costs speed, never results)
    const bool last = g == kGroups - 1 || bb.b[g] >= maxlen;
    if (!last && g > 0 && bb.b[g] == bb.b[g - 1]) continue;   // empty by its bounds
    int variant = fv >= 0 && fv != RX_L4 ? fv
                  : dflt || g == kGroups - 1 ? kGroupVariant[g]
                                             : pick_variant(bb.b[g] + 15);
    // (a launch may run the whole batch when it is not binned:
    // pptk_rx_autotune's choice for its shape applies, as in batch order)
    if (fv < 0 && c->tuned[1][variant] >= 0 && c->tuned[1][variant] != RX_L4)
      variant = c->tuned[1][variant];
    a.plan_group = (uint32_t)g;
    a.range_lo = tab + g;
    a.range_hi = tab + (last ? kGroups : g + 1);
    a.tune = pick_tune(c, variant, true);
    e = launch_rx(variant, a, grid_for(c, variant, b->n), s);
    if (e != hipSuccess) return -EIO;
    if (last) break;
  }
  return 0;
}

int pptk_rx_set_tuning(struct pptk_rx_ctx *c, int variant, int flags) {
  if (!c || variant < -1 || variant >= RX_NVARIANTS || flags < -1) return -EINVAL;
  if (flags >= 0 && ((uint32_t)flags & ~kTuneMask)) return -EINVAL;
  c->forced_variant = variant;
  // the rate limiter's bit is its own switch: flags that hold nothing else
  // leave the receive transform's memory policy automatic
  const int rx = flags < 0 ? -1 : flags & ~PPTK_RX_TUNE_PERMIT_PASSES;
  c->forced_flags = flags >= 0 && rx == 0 && (flags & PPTK_RX_TUNE_PERMIT_PASSES) ? -1 : rx;
  c->permit_passes = flags >= 0 && (flags & PPTK_RX_TUNE_PERMIT_PASSES);
  return 0;
}

// CU-mask bit i names CU i / nxcc of XCC i % nxcc, and CU k of an XCC sits
// in shader engine k % 4 (tools/cumask_map.py, profiles/r05 row aj): the
// top coll_cus bits are coll_cus / nxcc CUs of every XCC, the same number
// in each of its four SEs when that is a multiple of 4.  Each workgroup goes
// to an XCC and SE in turn, so a mask that leaves one SE short of another
// overfills it and the persistent grid runs a tail (-EINVAL below).
static constexpr int kSePerXcc = 4;

int pptk_rx_stream_split(struct pptk_rx_ctx *c, int coll_cus, void **rx_stream,
                         void **coll_stream) {
  if (!c || coll_cus < 0) return -EINVAL;
  if (coll_cus == 0) {   // the whole chip for the grids again; the streams stay the context's
    if (rx_stream) *rx_stream = nullptr;
    if (coll_stream) *coll_stream = nullptr;
    c->coll_cus = 0;
    return 0;
  }
  if (!rx_stream || !coll_stream) return -EINVAL;
  *rx_stream = *coll_stream = nullptr;
  if (c->split_coll && c->split_cus == coll_cus) {   // the pair the context holds
    *rx_stream = c->split_rx;
    *coll_stream = c->split_coll;
    c->coll_cus = coll_cus;
    return 0;
  }
  // A new pair: the communicator's channel cap (ncclConfig_t.maxCTAs, fixed
  // when it is created) follows the collective stream's CUs, so that stream
  // cannot change under a communicator -- or a creation in progress.
  if (ctx_comm_slot(c)->load(std::memory_order_acquire) != nullptr) return -EBUSY;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  int nxcc = 1;
  if (hipDeviceGetAttribute(&nxcc, hipDeviceAttributeNumberOfXccs, c->device) != hipSuccess ||
      nxcc < 1)
    nxcc = 1;
  if (coll_cus % (nxcc * kSePerXcc) || coll_cus >= c->ncu || c->ncu % nxcc) return -EINVAL;
  std::vector<uint32_t> rx((c->ncu + 31) / 32, 0), coll(rx.size(), 0);
  for (int i = 0; i < c->ncu; ++i) (i >= c->ncu - coll_cus ? coll : rx)[i / 32] |= 1u << (i % 32);
  hipStream_t a = nullptr, b = nullptr;
  if (hipExtStreamCreateWithCUMask(&a, (uint32_t)rx.size(), rx.data()) != hipSuccess) return -EIO;
  if (hipExtStreamCreateWithCUMask(&b, (uint32_t)coll.size(), coll.data()) != hipSuccess) {
    (void)hipStreamDestroy(a);
    return -EIO;
  }
  drop_split_streams(c);   // a pair of another CU count, no communicator since
  {
    std::lock_guard<std::mutex> g(g_split_mu);
    g_split_owned[a] = c;
    g_split_owned[b] = c;
    g_split_retired.erase(a);
    g_split_retired.erase(b);
  }
  c->split_rx = a;
  c->split_coll = b;
  c->split_cus = coll_cus;
  *rx_stream = a;
  *coll_stream = b;
  c->coll_cus = coll_cus;
  return 0;
}

int pptk_rx_stream_destroy(void *stream) {
  if (!stream) return -EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  {
    std::lock_guard<std::mutex> g(g_split_mu);
    if (g_split_owned.count(s)) return -EBUSY;   // its context destroys it
    if (g_split_retired.erase(s)) return 0;      // its context already did
  }
  return hip_err(hipStreamDestroy(s));
}

int pptk_rx_variant_count(void) { return RX_NVARIANTS; }

int pptk_rx_last_variant(const struct pptk_rx_ctx *c) { return c ? c->last_variant : -1; }

size_t pptk_rx_permit_scratch_bytes(uint64_t n, uint32_t hash_size) {
  if (hash_size == 0 || (hash_size & (hash_size - 1)) || n > 0xffffffffull) return 0;
  return permit_scratch_bytes(n, hash_size);
}

static int permit_common(struct pptk_rx_ctx *c, const struct pptk_rx_rec *d_recs,
                         const struct pptk_rx_rec32 *d_recs32, const uint32_t *d_keys,
                         uint64_t n, int family, const uint8_t *d_subject, uint32_t *d_tokens,
                         uint8_t *d_verdict, void *d_scratch, void *stream) {
  if (!c || (family != 4 && family != 6) || n > 0xffffffffull) return -EINVAL;
  if ((family == 4 && !c->opts.iphash_bits4) || (family == 6 && !c->opts.iphash_bits6))
    return -EINVAL;   // the records carry no bucket for that family
  const uint32_t hs = c->opts.iphash_size;
  if (hs == 0 || (hs & (hs - 1))) return -EINVAL;
  if (n == 0) return 0;
  if ((!d_recs && !d_recs32 && !d_keys) || !d_tokens || !d_verdict || !d_scratch) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  PermitArgs a{};
  a.recs = d_recs32 || d_keys ? nullptr : d_recs;
  a.recs32 = d_keys ? nullptr : d_recs32;
  a.keys_in = d_keys;
  a.n = n;
  a.subject = d_subject;
  a.tokens = d_tokens;
  a.verdict = d_verdict;
  a.hash_size = hs;
  a.family = family;
  // the fused kernel's workgroups must all be resident at once (grid
  // barriers): no more than the CUs a split leaves the batches' stream
  a.ncu = c->ncu - c->coll_cus;
  a.force_passes =
      c->permit_passes || (env_tune() >= 0 && (env_tune() & PPTK_RX_TUNE_PERMIT_PASSES)) ? 1 : 0;
  return hip_err(launch_permit(a, d_scratch, (hipStream_t)stream));
}

int pptk_rx_permit_status(struct pptk_rx_ctx *c, const void *d_scratch, void *stream) {
  if (!c || !d_scratch) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  return permit_status(d_scratch, (hipStream_t)stream);
}

int pptk_rx_permit_device(struct pptk_rx_ctx *c, const struct pptk_rx_rec *d_recs,
                          const struct pptk_rx_rec32 *d_recs32, uint64_t n, int family,
                          const uint8_t *d_subject, uint32_t *d_tokens, uint8_t *d_verdict,
                          void *d_scratch, void *stream) {
  if (!d_recs && !d_recs32) return -EINVAL;
  return permit_common(c, d_recs, d_recs32, nullptr, n, family, d_subject, d_tokens, d_verdict,
                       d_scratch, stream);
}

int pptk_rx_permit_keys_device(struct pptk_rx_ctx *c, const uint32_t *d_keys, uint64_t n,
                               int family, const uint8_t *d_subject, uint32_t *d_tokens,
                               uint8_t *d_verdict, void *d_scratch, void *stream) {
  if (!d_keys && n) return -EINVAL;
  return permit_common(c, nullptr, nullptr, d_keys, n, family, d_subject, d_tokens, d_verdict,
                       d_scratch, stream);
}

int pptk_rx_tokens_refill_device(struct pptk_rx_ctx *c, uint32_t *d_tokens, uint32_t start,
                                 uint32_t end, uint32_t add, uint32_t initial_tokens,
                                 void *stream) {
  if (!c || !d_tokens || start > end || end > c->opts.iphash_size) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  return hip_err(launch_refill(d_tokens, start, end, add, initial_tokens, (hipStream_t)stream));
}

size_t pptk_rx_bin_scratch_bytes(uint64_t n) { return bin_scratch_bytes(n, kBinGrid); }

int pptk_rx_bin_device(struct pptk_rx_ctx *c, const uint16_t *d_len, uint64_t n,
                       uint32_t *d_perm, void *d_scratch, void *stream) {
  if (!c || (n && (!d_len || !d_perm || !d_scratch))) return -EINVAL;
  if (n > 0xffffffffull) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  return hip_err(launch_bin(d_len, n, d_perm, d_scratch, (hipStream_t)stream, kBinGrid,
                            BinDesc{nullptr, 0, nullptr, nullptr}, bin_bounds(), false));
}

static int ensure_slot(pptk_rx_ctx *c, RxSlot &sl, size_t pkts, size_t bytes) {
  if (sl.stream && pkts <= sl.cap_pkts && bytes <= sl.cap_bytes) return 0;
  free_slot(sl);
  pkts = std::max(pkts, (size_t)c->opts.max_batch);
  bytes = std::max(bytes, (size_t)c->opts.max_batch * ((c->opts.max_frame + 15) & ~15u)) + 64;
  if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void **)&sl.h_frames, bytes, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&sl.h_off, pkts * 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&sl.h_len, pkts * 2, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&sl.h_recs, pkts * 64, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void **)&sl.d_frames, bytes) != hipSuccess ||
      hipMalloc((void **)&sl.d_off, pkts * 8) != hipSuccess ||
      hipMalloc((void **)&sl.d_len, pkts * 2) != hipSuccess ||
      hipMalloc((void **)&sl.d_recs, pkts * 64) != hipSuccess) {
    free_slot(sl);
    return -ENOMEM;
  }
  if (hipHostGetDevicePointer((void **)&sl.hd_frames, sl.h_frames, 0) != hipSuccess ||
      hipHostGetDevicePointer((void **)&sl.hd_off, sl.h_off, 0) != hipSuccess ||
      hipHostGetDevicePointer((void **)&sl.hd_len, sl.h_len, 0) != hipSuccess ||
      hipHostGetDevicePointer((void **)&sl.hd_recs, sl.h_recs, 0) != hipSuccess) {
    free_slot(sl);
    return -EIO;
  }
  sl.cap_pkts = pkts;
  sl.cap_bytes = bytes;
  sl.dev_cap = bytes;
  return 0;
}

// Room for a registered-ring span of `bytes` in the slot's device frame
// buffer (the slot is idle: its last chunk was retired).  Sparse rings
// (e.g. 2 KB netmap slots) have spans longer than max_batch * max_frame;
// grown up to 4x the staging size, once.
static bool fit_span(RxSlot &sl, size_t bytes) {
  if (bytes <= sl.dev_cap) return true;
  if (bytes > 4 * sl.cap_bytes) return false;
  uint8_t *p = nullptr;
  if (hipMalloc((void **)&p, bytes) != hipSuccess) return false;
  (void)hipFree(sl.d_frames);
  sl.d_frames = p;
  sl.dev_cap = bytes;
  return true;
}

// Chunks run "direct" -- the kernel reads the descriptors (and staged
// frames) from the pinned staging buffers and writes the records into
// pinned memory over PCIe: one kernel launch per chunk instead of three
// host-to-device copies, the launch and a device-to-host copy -- when the
// frames come from a registered ring (the kernel reads them over PCIe
// anyway) or the staged frame bytes are at most this many.  2 MiB: with
// four chunks in flight the DMA copy beats the kernel's PCIe reads from
// there on (1 M-frame C64 calls 375 -> 449 Mpkt/s staged, ring spans
// 325 -> 408; 4 096-frame C1500 calls 278 -> 238 us), while calls of up to
// ~1 400 1500-byte frames keep the single launch (DESIGN.md "End-to-end").
// PPTK_RX_DIRECT_MAX_BYTES overrides.
static size_t direct_max_bytes() {
  static const long v = env_long("PPTK_RX_DIRECT_MAX_BYTES", 2l << 20);
  return v < 0 ? 0 : (size_t)v;
}

// Bulky staged chunks go down by DMA, but their descriptors and records do
// not: the kernel reads the 10-byte descriptors from the pinned staging and
// writes the records into pinned memory over PCIe ("split" chunks), so the
// copy engine runs nothing but the frame copies back to back -- the two
// descriptor copies and the record copy cost ~0.18 ms of copy-engine time
// per 65 536-frame chunk beside its 2.2 ms frame copy (DESIGN.md
// "End-to-end").  PPTK_RX_SPLIT=0 restores the copies (A/B).
static bool split_chunks() {
  static const long v = EXP_KNOB("PPTK_RX_SPLIT", 1);
  return v != 0;
}

// A registered ring's chunk whose frames lie densely in the ring (frame
// bytes >= this fraction of the span they cover) and whose span is above
// the direct threshold is copied down by DMA as one span instead of being
// read in place by the kernel: a dense span moves ~48 GB/s of frames that
// way, the kernel's own reads of host memory ~37-38, so the break-even is
// near 80 % (1500-byte frames in 2 KB netmap slots, 73 %, measured 37 GB/s
// by DMA against 38 in place; DESIGN.md "End-to-end").
// PPTK_RX_RING_DMA_PCT (percent; 0 = always, > 100 = never) overrides.
static double ring_dma_density() {
  static const long v = env_long("PPTK_RX_RING_DMA_PCT", 80);
  return v / 100.0;
}

// Uniform chunks (every frame one length, ring frames at one stride) run as
// fixed-stride batches without descriptors (enqueue_chunk).  PPTK_RX_UNIFORM=0
// turns that off (A/B).
static bool uniform_chunks() {
  static const long v = EXP_KNOB("PPTK_RX_UNIFORM", 1);
  return v != 0;
}

// Copy one frame into 16-byte-aligned pinned staging with non-temporal
// stores: the lines go to memory without being read for ownership first
// and without staying dirty in the host caches, where the copy engine's
// reads of the staging would have to snoop them.  The bytes past the frame
// up to the next 16-byte boundary are zero (the kernel never uses them).
// PPTK_RX_NT_GATHER=0: plain memcpy (A/B).
static bool nt_gather() {
  static const long v = EXP_KNOB("PPTK_RX_NT_GATHER", 1);
  return v != 0;
}

static void stage_frame(uint8_t *dst, const uint8_t *src, size_t n) {
  size_t k = 0;
  for (; k + 16 <= n; k += 16)
    _mm_stream_si128((__m128i *)(dst + k), _mm_loadu_si128((const __m128i *)(src + k)));
  if (k < n) {
    alignas(16) uint8_t t[16] = {0};
    memcpy(t, src + k, n - k);
    _mm_stream_si128((__m128i *)(dst + k), _mm_load_si128((const __m128i *)t));
  }
}

// The context's worker pool (nullptr with gather_threads <= 1).  If the
// threads cannot be started the batch runs on the calling thread alone (and
// later batches try again): no exception leaves the C ABI.
static WorkerPool *pool_of(pptk_rx_ctx *c) {
  const size_t nth = std::max<size_t>(1, std::min<size_t>(c->opts.gather_threads, 64));
  if (nth > 1 && !c->pool) {
    try {
      c->pool = new WorkerPool(nth - 1);
    } catch (...) {
      c->pool = nullptr;
    }
  }
  return c->pool;
}

static size_t pool_size(const WorkerPool *pool) { return pool ? pool->size() : 1; }

// Copy n bytes, split over the pool when it pays (a few MB and up; 256 KB
// pieces measured slower than 1 MB ones on C64 chunks: the pool's per-item
// cost).
static void copy_out(WorkerPool *pool, void *dst, const void *src, size_t n) {
  constexpr size_t kPiece = 1u << 20;
#ifdef PPTK_RX_SERIAL_COPYOUT
  pool = nullptr;
#endif
  if (!pool || n < 2 * kPiece) {
    memcpy(dst, src, n);
    return;
  }
  const size_t parts = (n + kPiece - 1) / kPiece;
  pool->parallel_for(parts, [&](size_t i) {
    const size_t lo = i * kPiece, hi = std::min(n, lo + kPiece);
    memcpy((uint8_t *)dst + lo, (const uint8_t *)src + lo, hi - lo);
  });
}

// Wait for the slot's chunk and hand its records to the caller.
static int retire(RxSlot &sl, WorkerPool *pool) {
  if (!sl.busy) return 0;
  sl.busy = false;
  // (HIP spins before it blocks: polling hipEventQuery instead measured
  // equal on 32-frame chunks)
  if (hipEventSynchronize(sl.done) != hipSuccess) return -EIO;
  if (sl.out) copy_out(pool, sl.out, sl.h_recs, sl.count * sl.rec_bytes);
  return 0;
}

// The registered ring holding every frame of pkts[0, num), so that frame
// bytes can be read in place (the kernel reads whole 16-byte chunks, so each
// frame's chunk-rounded end must lie inside the ring too); NULL otherwise.
// The registered ring holding the call's first frame, the candidate for
// reading the frames in place; every chunk checks its own frames against it
// in its descriptor pass (enqueue_chunk) and is staged instead when one lies
// outside.  (A serial pass over all frames here, before the first chunk,
// had cost a 4 M-frame C64 call as much as its frame copies.)
static const RxRing *ring_of(const pptk_rx_ctx *c, const struct ldp_packet *pkts, int num) {
  if (c->rings.empty() || num <= 0) return nullptr;
  const uint8_t *p0 = (const uint8_t *)pkts[0].data;
  for (const RxRing &r : c->rings)
    if (p0 >= r.host && p0 < r.host + r.bytes) return &r;
  return nullptr;
}

// The registered region holding the caller's whole record array, so that
// the kernel writes the records there in place over PCIe (no record copy
// from the staging); NULL otherwise.
static const RxRing *records_region(const pptk_rx_ctx *c, const void *recs, size_t bytes) {
  const uint8_t *p = (const uint8_t *)recs;
  for (const RxRing &r : c->rings)
    if (p >= r.host && bytes <= r.bytes && (size_t)(p - r.host) <= r.bytes - bytes) return &r;
  return nullptr;
}

int pptk_rx_register_ring(struct pptk_rx_ctx *c, void *base, size_t bytes) {
  if (!c || !base || bytes == 0) return -EINVAL;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  if (hipHostRegister(base, bytes, hipHostRegisterMapped) != hipSuccess) return -EIO;
  void *dev = nullptr;
  if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
    (void)hipHostUnregister(base);
    return -EIO;
  }
  c->rings.push_back(RxRing{(uint8_t *)base, bytes, (const uint8_t *)dev});
  return 0;
}

int pptk_rx_unregister_ring(struct pptk_rx_ctx *c, void *base) {
  if (!c || !base) return -EINVAL;
  for (size_t i = 0; i < c->rings.size(); ++i) {
    if (c->rings[i].host == (uint8_t *)base) {
      DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
      for (RxSlot &sl : c->slot)   // no chunk may still read the ring
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
      (void)hipHostUnregister(base);
      c->rings.erase(c->rings.begin() + (long)i);
      return 0;
    }
  }
  return -EINVAL;
}

// A chunk that failed part-way: nothing it queued may still run (it may
// read the caller's frames or write the slot) when the error is returned.
static int chunk_failed(RxSlot &sl, int rc) {
  (void)hipStreamSynchronize(sl.stream);
  sl.busy = false;
  return rc;
}

// One chunk of a host batch (cnt <= opts.max_batch frames) into slot `sl`,
// idle and sized by ensure_slot: its descriptors and frames, then its
// copies, the launch and the record copy-back queued on the slot's stream,
// nothing waited for.  retire() waits for it and hands the records to `out`.
// In a registered ring the kernel reads the frames in place over PCIe (or
// the span goes down by DMA) and only the 10-byte descriptors are written.
static size_t chunk_bytes(const pptk_rx_ctx *c);

static int enqueue_chunk(pptk_rx_ctx *c, RxSlot &sl, const struct ldp_packet *cp, size_t cnt,
                         void *out, size_t rec_bytes, const RxRing *ring,
                         const RxRing *rreg, WorkerPool *pool) {
  const uint32_t maxf = c->opts.max_frame ? c->opts.max_frame : 65535u;
  // Descriptors, then the frame bytes.  On one thread (no pool, or a
  // small chunk) both in one pass.  With the pool, both in parallel over
  // parts of the chunk: a first pass writes the lengths (and a ring's
  // offsets) and sums each part's staging bytes, a serial prefix over the
  // parts gives each part its staging base, and a second pass writes the
  // staging offsets while it gathers the frames (a serial descriptor pass
  // had cost a 65 536-frame C64 chunk as much as the whole parallel
  // gather, DESIGN.md "End-to-end").
  const bool nt = nt_gather();
  auto stage = [&sl, cp, nt](size_t i) {
    if (nt) stage_frame(sl.h_frames + sl.h_off[i], (const uint8_t *)cp[i].data, sl.h_len[i]);
    else memcpy(sl.h_frames + sl.h_off[i], cp[i].data, sl.h_len[i]);
  };
  // one part: lengths (+ ring offsets / span) and, for staged chunks, the
  // staging bytes it needs; with `base` given, also the staging offsets
  // and the gather
  // (write = false: a ring chunk's first pass -- the span, the checks, the
  // uniformity -- with nothing written; a uniform ring chunk needs no more)
  auto describe = [&sl, cp, ring, maxf, nt, &stage](size_t i0, size_t i1, size_t base,
                                                    bool gather, PartDesc &d, bool write = true) {
    size_t pos = base;
    if (i1 > i0) {
      d.p0 = (const uint8_t *)cp[i0].data;
      d.sz0 = cp[i0].sz;
      d.stride = i1 - i0 > 1 ? (const uint8_t *)cp[i0 + 1].data - d.p0 : 0;
      d.same = d.p0 != nullptr && d.sz0 <= maxf;
      d.uni = d.same;
    }
    for (size_t i = i0; i < i1; ++i) {
      const struct ldp_packet &pk = cp[i];
      const bool ok = pk.data && pk.sz <= maxf;
      const uint32_t sz = ok ? pk.sz : 0u;
      d.same = d.same && ok && pk.sz == d.sz0;
      d.uni = d.uni && d.same && (const uint8_t *)pk.data == d.p0 + (int64_t)(i - i0) * d.stride;
      if (write) sl.h_len[i] = (uint16_t)sz;
      if (ring) {
        const uint8_t *pd = (const uint8_t *)pk.data;
        // (every frame's chunk-rounded end inside the registered region)
        d.outside = d.outside || (pd && (pd < ring->host ||
                                         (((size_t)(pd - ring->host) + pk.sz + 15) & ~(size_t)15) >
                                             ring->bytes));
        const uint64_t o = pd ? (uint64_t)(pd - ring->host) : 0u;
        if (write) sl.h_off[i] = o;
        d.lo = std::min<size_t>(d.lo, o);
        // (the frame's chunk-rounded END, clamped to the region: a span
        // copy must not read past the registered memory; the kernel's reads
        // past a frame's end stay inside the span's 16-byte slack)
        d.hi = std::max<size_t>(d.hi, std::min<size_t>((o + sz + 15) & ~(size_t)15, ring->bytes));
        d.fbytes += sz;
      } else if (gather) {
        sl.h_off[i] = pos;
        if (sz) stage(i);
      }
      pos += (sz + 15) & ~(size_t)15;
      d.maxlen = std::max(d.maxlen, sz);
    }
    d.bytes = pos - base;
    // this thread's streaming stores, before the copy is queued
    if (gather && nt) _mm_sfence();
  };
  // The pool only for big chunks: waking it costs ~20-40 µs, more than a
  // 256-frame or even a 1.5 MB gather saves (DESIGN.md "End-to-end").
  // Staged chunks: parts of ~1024 frames or ~256 KB of frame bytes
  // (estimated from the first frame), at most 8 per thread, in ONE pass
  // over the pool -- each
  // part sums its staging bytes, takes its base from the previous part's
  // published running total (parts are claimed in order, so that one is
  // done or in progress), publishes its own, then writes its offsets and
  // gathers.  Ring chunks (no gather): parts of ~2048 frames.
  const size_t est = cnt * (size_t)std::min<uint32_t>(cp[0].sz, maxf);
  const bool staged = !ring;
  size_t nparts = 1;
  if (pool && staged && (cnt >= 8192 || est >= (4u << 20)))
    nparts = std::max(cnt / 1024, est >> 18);
  else if (pool && !staged && cnt >= 16384)
    nparts = cnt / 2048;
  nparts = std::max<size_t>(1, std::min<size_t>(nparts, std::min<size_t>(8 * pool_size(pool), cnt)));
  std::vector<PartDesc> &parts = sl.parts;
  parts.assign(nparts, PartDesc{});
  if (!staged) {
    // first pass: nothing written; a frame outside the ring stages the
    // chunk, a uniform chunk needs no descriptors at all
    auto pass = [&](bool write) {
      if (nparts == 1)
        describe(0, cnt, 0, false, parts[0], write);
      else
        pool->parallel_for(nparts, [&](size_t t) {
          parts[t] = PartDesc{};
          describe(cnt * t / nparts, cnt * (t + 1) / nparts, 0, false, parts[t], write);
        });
    };
    pass(false);
    bool outside = false, uni = uniform_chunks() && cnt > 1;
    for (const PartDesc &d : parts) outside = outside || d.outside;
    if (outside) {   // staged instead (the slot is idle: size its staging)
      const int rc = ensure_slot(c, sl, std::max<size_t>(c->opts.max_batch, 1), chunk_bytes(c));
      return rc ? rc : enqueue_chunk(c, sl, cp, cnt, out, rec_bytes, nullptr, rreg, pool);
    }
    for (size_t t = 0; t < parts.size() && uni; ++t)
      uni = parts[t].uni && parts[t].sz0 == parts[0].sz0 && parts[t].stride == parts[0].stride &&
            parts[t].stride > 0 &&
            parts[t].p0 == parts[0].p0 + (int64_t)(cnt * t / parts.size()) * parts[0].stride;
    if (!uni) {
      for (PartDesc &d : parts) d = PartDesc{};
      pass(true);
    }
  } else if (nparts == 1) {
    describe(0, cnt, 0, staged, parts[0]);
  } else {
    if (sl.run_cap < nparts) {
      sl.run.reset(new std::atomic<size_t>[nparts]);
      sl.run_cap = nparts;
    }
    std::atomic<size_t> *run = sl.run.get();
    for (size_t t = 0; t < nparts; ++t) run[t].store(SIZE_MAX, std::memory_order_relaxed);
    pool->parallel_for(nparts, [&](size_t t) {
      const size_t i0 = cnt * t / nparts, i1 = cnt * (t + 1) / nparts;
      PartDesc &d = parts[t];
      describe(i0, i1, 0, false, d);            // lengths, this part's bytes
      size_t base = 0;
      if (t > 0)
        while ((base = run[t - 1].load(std::memory_order_acquire)) == SIZE_MAX) _mm_pause();
      run[t].store(base + d.bytes, std::memory_order_release);
      PartDesc d2{};
      describe(i0, i1, base, true, d2);         // offsets + gather
    });
  }
  size_t pos = 0, lo = SIZE_MAX, hi = 0, fbytes = 0;
  uint32_t maxlen = 0;
  for (const PartDesc &d : parts) {
    pos += d.bytes;
    lo = std::min(lo, d.lo);
    hi = std::max(hi, d.hi);
    fbytes += d.fbytes;
    maxlen = std::max(maxlen, d.maxlen);
  }
  // Uniform chunk: every frame the same length (and, for a registered ring,
  // at one fixed stride from the first): it runs as a fixed-stride batch --
  // no descriptor is read by the kernel (in a staged chunk the frames sit at
  // 16-byte-rounded offsets, i.e. at a fixed stride already), and frames of
  // at most 64 bytes take the lane kernel.  A C64 chunk then moves its frames
  // and its records over PCIe and nothing else.
  bool uni_len = !parts.empty(), uni_ptr = uni_len;
  int64_t stride = 0;
  {
    const PartDesc &f = parts[0];
    stride = f.stride;
    for (size_t t = 0; t < parts.size() && uni_len; ++t) {
      const PartDesc &d = parts[t];
      const size_t i0 = cnt * t / parts.size();
      uni_len = d.same && d.sz0 == f.sz0;
      // (each part's own stride, and its first frame where the first
      // part's stride puts it; one-frame parts have no stride of their own)
      uni_ptr = uni_ptr && uni_len && d.uni &&
                (d.stride == stride || cnt * (t + 1) / parts.size() - i0 == 1) &&
                d.p0 == f.p0 + (int64_t)i0 * stride;
    }
    if (cnt == 1) uni_ptr = false;
  }
  const uint32_t ulen = parts.empty() ? 0u : parts[0].sz0;
  // a dense ring chunk goes down as one span; the kernel sees the span's
  // buffer shifted down by `lo`, so the ring offsets stay as they are
  const bool ring_dma = ring && hi > lo && hi - lo > direct_max_bytes() &&
                        (double)fbytes >= ring_dma_density() * (double)(hi - lo) &&
                        fit_span(sl, hi - lo + 16);
  hipStream_t s = sl.stream;
  const bool direct =
      ring ? direct_max_bytes() > 0 && !ring_dma : pos <= direct_max_bytes();
  // descriptors and records over PCIe, frames by DMA
  const bool split = !direct && (ring_dma || !ring) && split_chunks();
  const bool pcie = direct || split;
  if ((!direct && !ring &&
       hipMemcpyAsync(sl.d_frames, sl.h_frames, std::max<size_t>(pos, 16),
                      hipMemcpyHostToDevice, s) != hipSuccess) ||
      (ring_dma && hipMemcpyAsync(sl.d_frames, ring->host + lo, hi - lo,
                                  hipMemcpyHostToDevice, s) != hipSuccess) ||
      (!pcie &&
       (hipMemcpyAsync(sl.d_off, sl.h_off, cnt * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(sl.d_len, sl.h_len, cnt * 2, hipMemcpyHostToDevice, s) != hipSuccess)))
    return chunk_failed(sl, -EIO);
  pptk_rx_dev_batch b;
  memset(&b, 0, sizeof(b));
  b.d_frames = ring && !ring_dma ? ring->dev
               : ring_dma           ? (const uint8_t *)((uintptr_t)sl.d_frames - lo)
               : direct             ? sl.hd_frames
                                    : sl.d_frames;
  b.d_off = pcie ? sl.hd_off : sl.d_off;
  b.d_len = pcie ? sl.hd_len : sl.d_len;
  b.max_len = maxlen;
  b.n = cnt;
  if (uniform_chunks() && cnt > 1 && uni_len && (!ring || (uni_ptr && stride > 0))) {
    // fixed stride: staged frames at i * round16(len); ring frames at the
    // first frame's place + i * stride
    b.d_off = nullptr;
    b.d_len = nullptr;
    b.fixed_len = ulen;
    if (ring) {
      b.d_frames += (size_t)(parts[0].p0 - ring->host);
      b.stride = (uint64_t)stride;
    } else {
      b.stride = (ulen + 15u) & ~15u;
      if (b.stride == 0) b.stride = 16;
    }
  }
  // records: into the caller's array itself when it is registered
  void *d_out = rreg ? (void *)(rreg->dev + ((const uint8_t *)out - rreg->host))
                : pcie ? (void *)sl.hd_recs
                       : (void *)sl.d_recs;
  if (rec_bytes == 32) b.d_recs32 = (pptk_rx_rec32 *)d_out;   // compact records
  else b.d_recs = (pptk_rx_rec *)d_out;
  const int rc = pptk_rx_batch_device(c, &b, s);
  if (rc != 0) return chunk_failed(sl, rc);
  if ((!pcie && !rreg &&
       hipMemcpyAsync(sl.h_recs, sl.d_recs, cnt * rec_bytes, hipMemcpyDeviceToHost, s) !=
           hipSuccess) ||
      hipEventRecord(sl.done, s) != hipSuccess)
    return chunk_failed(sl, -EIO);
  sl.out = rreg ? nullptr : out;   // (retire copies only staged records)
  sl.rec_bytes = rec_bytes;
  sl.count = cnt;
  sl.busy = true;
  return 0;
}

// Slots a synchronous pptk_rx_batch rotates over (chunks in flight; a slot
// is allocated when a call first has that many chunks): four measured
// +17-24 % on 1 M-frame C64 calls against two, C1500 +1-2 % (at the PCIe
// ceiling either way; DESIGN.md "End-to-end").  PPTK_RX_SYNC_SLOTS (2 ..
// PPTK_RX_MAX_INFLIGHT) overrides.
static size_t sync_slots() {
  static const long v = env_long("PPTK_RX_SYNC_SLOTS", PPTK_RX_MAX_INFLIGHT);
  return (size_t)std::min<long>(std::max<long>(v, 2), PPTK_RX_MAX_INFLIGHT);
}

// Staging bytes a slot needs for one chunk of this context's batches.
static size_t chunk_bytes(const pptk_rx_ctx *c) {
  const uint32_t maxf = c->opts.max_frame ? c->opts.max_frame : 65535u;
  return std::max<size_t>(c->opts.max_batch, 1) * ((maxf + 15) & ~15u);
}

static bool host_args_ok(const pptk_rx_ctx *c, const struct ldp_packet *pkts, int num,
                         const void *recs) {
  return c && num >= 0 && (num == 0 || (pkts && recs));
}

// pptk_rx_batch / pptk_rx_batch32: records of rec_bytes (64 or 32) each.
static int host_batch(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num, void *recs,
                      size_t rec_bytes) {
  if (!host_args_ok(c, pkts, num, recs)) return -EINVAL;
  if (num == 0) return 0;
  if (c->async_n) return -EBUSY;   // the submissions own the slots
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  WorkerPool *pool = pool_of(c);
  const RxRing *ring = ring_of(c, pkts, num);
  const RxRing *rreg = records_region(c, recs, (size_t)num * rec_bytes);
  const size_t chunk = std::max<size_t>(c->opts.max_batch, 1);
  int rc = 0;
  // Multi-buffered: while chunk k runs on one slot's stream (H2D, kernel,
  // D2H), the host gathers the next chunks into the other slots.
  const size_t nslots = sync_slots();
  size_t k = 0, cnt = 0;
  for (size_t first = 0; first < (size_t)num && rc == 0; first += cnt, ++k) {
    RxSlot &sl = c->slot[k % nslots];
    if ((rc = retire(sl, pool)) != 0) break;
    cnt = std::min(chunk, (size_t)num - first);
    if ((rc = ensure_slot(c, sl, chunk, ring ? 64 : chunk_bytes(c))) != 0) break;
    rc = enqueue_chunk(c, sl, pkts + first, cnt, (uint8_t *)recs + first * rec_bytes, rec_bytes,
                       ring, rreg, pool);
  }
  // drain (also on error: nothing may still read the caller's buffers)
  for (RxSlot &sl : c->slot) {
    const int r2 = retire(sl, pool);
    if (rc == 0) rc = r2;
  }
  return rc;
}

int pptk_rx_batch(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num,
                  struct pptk_rx_rec *recs) {
  return host_batch(c, pkts, num, recs, sizeof(pptk_rx_rec));
}

int pptk_rx_batch32(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num,
                    struct pptk_rx_rec32 *recs) {
  return host_batch(c, pkts, num, recs, sizeof(pptk_rx_rec32));
}

static int host_submit(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num, void *recs,
                       size_t rec_bytes) {
  if (!host_args_ok(c, pkts, num, recs)) return -EINVAL;
  if (num == 0) return 0;
  if ((size_t)num > std::max<size_t>(c->opts.max_batch, 1)) return -EINVAL;
  if (c->async_n >= PPTK_RX_MAX_INFLIGHT) return -EBUSY;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  const RxRing *ring = ring_of(c, pkts, num);
  const RxRing *rreg = records_region(c, recs, (size_t)num * rec_bytes);
  // the slots rotate in submission order (FIFO), so consecutive
  // submissions run on different streams and may overlap on the GPU
  RxSlot &sl = c->slot[(c->async_head + c->async_n) % PPTK_RX_MAX_INFLIGHT];
  int rc = ensure_slot(c, sl, std::max<size_t>(c->opts.max_batch, 1), ring ? 64 : chunk_bytes(c));
  if (rc == 0)
    rc = enqueue_chunk(c, sl, pkts, (size_t)num, recs, rec_bytes, ring, rreg, pool_of(c));
  if (rc != 0) return rc;
  ++c->async_n;
  return 0;
}

int pptk_rx_batch_submit(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num,
                         struct pptk_rx_rec *recs) {
  return host_submit(c, pkts, num, recs, sizeof(pptk_rx_rec));
}

int pptk_rx_batch_submit32(struct pptk_rx_ctx *c, const struct ldp_packet *pkts, int num,
                           struct pptk_rx_rec32 *recs) {
  return host_submit(c, pkts, num, recs, sizeof(pptk_rx_rec32));
}

int pptk_rx_batch_complete(struct pptk_rx_ctx *c) {
  if (!c) return -EINVAL;
  if (c->async_n == 0) return -ENOENT;
  DeviceScope dg(c->device);
  if (!dg.ok) return -EIO;
  RxSlot &sl = c->slot[c->async_head];
  const int cnt = (int)sl.count;
  const int rc = retire(sl, c->pool);
  // (dropped from the queue even on an error: its slot is idle again)
  c->async_head = (c->async_head + 1) % PPTK_RX_MAX_INFLIGHT;
  --c->async_n;
  return rc ? rc : cnt;
}

int pptk_rx_batch_pending(const struct pptk_rx_ctx *c) { return c ? c->async_n : -EINVAL; }

}  // extern "C"
