// rx_comm.hip -- multi-GPU part of the C-ABI (include/pptk_rx.h, "Multi-GPU").
//
// Packet batches shard embarrassingly: every GPU runs the
// receive transform on its own contiguous range of frames and the only
// exchange is one all-gather of the per-frame flow hashes, so that every
// GPU ends up with the flow hash of every frame of the batch.  That
// collective is RCCL's ncclAllGather over xGMI on a communicator owned by
// the context, enqueued on the caller's stream right behind the batch that
// produced the hashes (pptk_rx_dev_batch.d_hash), so it needs no host
// synchronisation and overlaps the next batch's kernel when the caller
// alternates streams.
//
// Two ways to build the communicator, matching the reference's two scaling
// models: one process per GPU (pptk_rx_comm_uid on one rank, the 128-byte id
// passed to every rank by the application, pptk_rx_comm_create on each), or
// one process driving every GPU with one rx thread per GPU, as LDP's
// multi-queue loops run one thread per queue (reference ldp/ldprecvmt.c:
// 174-182): pptk_rx_comm_create_all over one context per GPU.
//
// Failure containment.  The reference's queue threads share nothing, so one
// failing thread cannot stall the others; a collective can: a rank that
// never joins (or dies, or skips a gather) leaves every other rank waiting
// inside RCCL.  So every wait here is bounded by opts.comm_timeout_ms:
// creation (init plus a warm-up gather that makes RCCL connect the ring)
// runs on a helper thread the caller stops waiting for at the deadline
// (-ETIMEDOUT; bounded_init below says why RCCL's own non-blocking mode is
// not enough); pptk_rx_comm_sync waits for a stream with the same deadline,
// surfaces RCCL's asynchronous errors (-EIO) and aborts the communicator on
// either, which makes RCCL's kernels give up so the stream drains;
// pptk_rx_comm_abort (any thread) cancels a communicator that other threads
// may be waiting on (-ECANCELED from then on).
//
// RCCL is loaded on first use (dlopen): a single-GPU application never maps
// the 570 MB library, and a box without it gets -ENOSYS from these entry
// points only.
//
// Errors: 0 or -errno; contract violations -EINVAL before RCCL is called,
// RCCL argument errors -EINVAL, every other RCCL or HIP failure -EIO.
#include <dlfcn.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>
#include <vector>

#include <rccl/rccl.h>   // types and constants only: the functions are dlsym'd

#include "rx_internal.h"

using namespace pptk;

// Experiment builds: PPTK_RX_COMM_TRACE=1 traces the communicator calls.
#ifdef PPTK_RX_EXPERIMENTS
#include <stdio.h>
#define COMM_TRACE(...)                                              \
  do {                                                               \
    static const bool on_ = getenv("PPTK_RX_COMM_TRACE") != nullptr; \
    if (on_) {                                                       \
      fprintf(stderr, "[pptk comm] " __VA_ARGS__);                   \
      fputc('\n', stderr);                                           \
    }                                                                \
  } while (0)
#else
#define COMM_TRACE(...) \
  do {                  \
  } while (0)
#endif

namespace {

// The RCCL entry points used here, resolved once from librccl.so.1.
struct Rccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId *);
  ncclResult_t (*CommInitRankConfig)(ncclComm_t *, int, ncclUniqueId, int, ncclConfig_t *);
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t *);
  ncclResult_t (*CommFinalize)(ncclComm_t);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommAbort)(ncclComm_t);
  ncclResult_t (*GroupStart)(void);
  ncclResult_t (*GroupEnd)(void);
  ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t);
  bool ok;
};

const Rccl *rccl() {
  static Rccl r{};
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    // the RCCL this library was compiled against first (ncclConfig_t is
    // versioned), then whatever the process already maps
    for (const char *name : {"/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) return;
    bool all = true;
    auto sym = [&](auto &fp, const char *name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      all = all && fp != nullptr;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRankConfig, "ncclCommInitRankConfig");
    sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(r.CommFinalize, "ncclCommFinalize");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommAbort, "ncclCommAbort");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.AllGather, "ncclAllGather");
    r.ok = all;   // (the handle stays open for the life of the process)
  });
  return r.ok ? &r : nullptr;
}

int nccl_err(ncclResult_t r) {
  if (r == ncclSuccess) return 0;
  if (r == ncclInvalidArgument || r == ncclInvalidUsage) return -EINVAL;
  return -EIO;
}

using Clock = std::chrono::steady_clock;

struct Deadline {
  Clock::time_point t;
  explicit Deadline(uint32_t ms) : t(Clock::now() + std::chrono::milliseconds(ms)) {}
  bool passed() const { return Clock::now() >= t; }
};

// Poll back-off: tight for the first millisecond (a gather that is about
// to finish), then 100 us sleeps.
struct Backoff {
  Clock::time_point t0 = Clock::now();
  void pause() {
    if (Clock::now() - t0 < std::chrono::milliseconds(1)) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
};

struct InitJob;

// A context's communicator slot.  Besides a live (or aborted) communicator
// it holds, while pptk_rx_comm_create runs, the creation in progress (so an
// abort from another thread can cancel it), and, when an abort arrives at a
// context that has no communicator yet, that pending abort (its next
// pptk_rx_comm_create returns -ECANCELED at once).
enum class CommState { kCreating, kReady, kPendingAbort };

struct RxComm {
  std::mutex mu;          // guards comm and state against a concurrent abort
  CommState state = CommState::kReady;
  ncclComm_t comm = nullptr;
  int nranks = 0;
  int rank = 0;
  bool aborted = false;   // comm is gone (aborted); only the struct remains
  std::shared_ptr<InitJob> job;   // kCreating: the creation to cancel
};

// Slot reads that go on to lock an RxComm (abort) and slot clears that
// delete one (a failed or cancelled creation, a consumed pending abort,
// destroy) are serialised by this lock, so an abort from another thread
// never touches a deleted RxComm.
std::mutex g_slots;

RxComm *comm_of(const pptk_rx_ctx *c) {
  return (RxComm *)ctx_comm_slot((pptk_rx_ctx *)c)->load(std::memory_order_acquire);
}

// The context's communicator, if it has one (live or aborted): not a
// creation in progress, not a pending abort.
RxComm *live_comm_of(const pptk_rx_ctx *c) {
  RxComm *m = comm_of(c);
  return m && m->state == CommState::kReady ? m : nullptr;
}

void set_comm(pptk_rx_ctx *c, RxComm *m) {
  ctx_comm_slot(c)->store(m, std::memory_order_release);
}

// Wait while RCCL reports the communicator's last call in progress; the
// final state, or ncclInProgress if the deadline passed first.
ncclResult_t wait_ready(const Rccl *R, ncclComm_t comm, const Deadline &d) {
  Backoff b;
  for (;;) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t r = R->CommGetAsyncError(comm, &st);
    if (r != ncclSuccess) return r;
    if (st != ncclInProgress || d.passed()) return st;
    b.pause();
  }
}

// Abort under the lock, once.
void abort_locked(const Rccl *R, RxComm *m) {
  if (m->aborted) return;
  (void)R->CommAbort(m->comm);
  m->comm = nullptr;
  m->aborted = true;
}

// Orderly teardown of a healthy communicator: finalize (flushes what was
// enqueued), bounded wait, destroy; abort if the flush does not finish.
void teardown(const Rccl *R, RxComm *m, uint32_t timeout_ms) {
  std::lock_guard<std::mutex> g(m->mu);
  if (m->aborted) return;
  const Deadline d(timeout_ms);
  ncclResult_t r = R->CommFinalize(m->comm);
  if (r == ncclSuccess || r == ncclInProgress) r = wait_ready(R, m->comm, d);
  if (r == ncclSuccess) {
    (void)R->CommDestroy(m->comm);
    m->comm = nullptr;
    m->aborted = true;
  } else {
    abort_locked(R, m);
  }
}

// The communicator's configuration: non-blocking (every wait here is
// polled under a deadline), and, on a context whose CUs pptk_rx_stream_split
// divided, at most one RCCL block per CU left to the collective stream
// (maxCTAs = coll_cus).  RCCL's all-gather kernel takes a whole CU per block
// on gfx950, so with more channels than those CUs the
// collective's blocks could not all be resident beside the batches' grid and
// the gather would run in waves; the cap is a creation-time setting, which is
// why the split has to come first (pptk_rx_stream_split: -EBUSY once a
// communicator exists).  Uncapped (RCCL's own channel count) without a split.
ncclConfig_t comm_config(int coll_cus) {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  if (coll_cus > 0) cfg.maxCTAs = coll_cus;
#ifdef PPTK_RX_EXPERIMENTS
  if (getenv("PPTK_RX_COMM_BLOCKING")) cfg.blocking = 1;
#endif
  return cfg;
}

// Communicator creation, bounded whatever RCCL does.  The init runs on a
// helper thread and the caller waits for it until the deadline.  RCCL is
// meant to return from a non-blocking init at once (ncclConfig_t.blocking =
// 0, then poll ncclCommGetAsyncError; torch's bundled RCCL 2.26.6 does), but
// /opt/rocm's RCCL 2.27.7 runs the init synchronously inside
// ncclCommInitRankConfig, in a group or not (measured: with a rank that never
// joins the call did not return for 30 s).  So the helper does the whole
// init -- the call, then the polling of a non-blocking one -- and if the
// caller gives up first it marks the job abandoned and returns -ETIMEDOUT:
// the helper aborts whatever it built once RCCL lets it go (at once for a
// non-blocking init; for one stuck inside RCCL, when the missing rank
// appears or the process exits).  The job is shared, so either side may
// finish last.
struct InitJob {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false, abandoned = false;
  bool cancelled = false;   // pptk_rx_comm_abort on a context being created
  ncclResult_t r = ncclSuccess;
  std::vector<ncclComm_t> comms;
};

// Helper threads the caller gave up on (deadline or abort) that have not
// finished yet: one stuck inside RCCL's synchronous init stays until the
// missing rank appears or the process exits, so a caller retrying creation
// could pile them up; beyond kMaxAbandoned creation returns -EAGAIN.
constexpr int kMaxAbandoned = 4;
std::atomic<int> g_abandoned{0};

bool job_abandoned(const std::shared_ptr<InitJob> &job) {
  std::lock_guard<std::mutex> g(job->mu);
  return job->abandoned;
}

// Fault injection for the failure-containment tests (a rank that inits but
// never issues the warm-up gather cannot be staged on a one-GPU box):
// PPTK_RX_COMM_TEST_WARMUP_STALL_MS=t holds the warm-up stream behind a
// kernel that spins for t ms (bounded: at most 60 s) before the gather, as a
// peer that never arrives would.  Read at each creation; unset in production.
__global__ void warmup_stall_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// Compiled in only by the test library (PPTK_RX_TEST_HOOKS,
// tests/hooks/libpptkrx_hooks.so); the product library never reads it.
uint32_t warmup_stall_ms() {
#ifdef PPTK_RX_TEST_HOOKS
  const char *e = getenv("PPTK_RX_COMM_TEST_WARMUP_STALL_MS");
  const long v = e ? atol(e) : 0;
  return v <= 0 ? 0u : (uint32_t)std::min(v, 60000L);
#else
  return 0;
#endif
}

void init_run(const Rccl *R, std::shared_ptr<InitJob> job, ncclUniqueId id,
              std::vector<int> devs, std::vector<int> ranks, std::vector<int> caps, int nranks,
              uint32_t timeout_ms) {
  // the helper's own bound (the caller's deadline plus a margin): even if
  // nobody marks the job abandoned, no wait here is unbounded
  const Deadline until(timeout_ms + 1000);
  const size_t k = devs.size();
  std::vector<ncclComm_t> comms(k, nullptr);
  std::vector<ncclConfig_t> cfg(k);
  for (size_t i = 0; i < k; ++i) cfg[i] = comm_config(caps[i]);
  auto going = [](ncclResult_t x) { return x == ncclSuccess || x == ncclInProgress; };
  ncclResult_t r = k > 1 ? R->GroupStart() : ncclSuccess;   // (ncclCommInitAll's form)
  for (size_t i = 0; i < k && going(r); ++i) {
    if (hipSetDevice(devs[i]) != hipSuccess) r = ncclUnhandledCudaError;
    else r = R->CommInitRankConfig(&comms[i], nranks, id, ranks[i], &cfg[i]);
  }
  if (k > 1) {
    const ncclResult_t re = R->GroupEnd();
    if (going(r)) r = re;
  }
  COMM_TRACE("init job: init calls returned %d", (int)r);
  // a non-blocking init goes on in RCCL: poll until it is done, or until
  // the caller has given up
  Backoff b;
  for (size_t i = 0; i < k && going(r);) {
    ncclResult_t st = ncclInProgress;
    if (!comms[i] || R->CommGetAsyncError(comms[i], &st) != ncclSuccess) st = ncclInternalError;
    if (st != ncclInProgress) {
      r = st;
      ++i;
      continue;
    }
    if (job_abandoned(job) || until.passed()) {
      r = ncclInProgress;
      break;
    }
    b.pause();
  }
  // Warm-up gather of one element on every new communicator: RCCL sets
  // up its ring connections with the peers lazily, at the first collective,
  // and that setup can block inside ncclAllGather; doing it here puts it
  // under the same deadline, so the product's gathers only enqueue.
  if (r == ncclSuccess) {
    std::vector<hipStream_t> st(k, nullptr);
    std::vector<uint64_t *> buf(k, nullptr);
    const uint32_t stall = warmup_stall_ms();
    for (size_t i = 0; i < k && r == ncclSuccess; ++i)
      if (hipSetDevice(devs[i]) != hipSuccess ||
          hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking) != hipSuccess ||
          hipMalloc((void **)&buf[i], (size_t)nranks * 8) != hipSuccess ||
          hipMemsetAsync(buf[i], 0, (size_t)nranks * 8, st[i]) != hipSuccess)
        r = ncclUnhandledCudaError;
    for (size_t i = 0; i < k && r == ncclSuccess && stall; ++i) {
      (void)hipSetDevice(devs[i]);
      hipLaunchKernelGGL(warmup_stall_kernel, dim3(1), dim3(64), 0, st[i], (uint64_t)stall * 100000u);
    }
    if (r == ncclSuccess && k > 1) r = R->GroupStart();
    for (size_t i = 0; i < k && going(r); ++i) {
      (void)hipSetDevice(devs[i]);
      r = R->AllGather(buf[i] + ranks[i], buf[i], 1, ncclUint64, comms[i], st[i]);
    }
    if (k > 1 && going(r)) r = R->GroupEnd();
    // Enqueued; now let it finish -- polled, never a blocking wait: a peer
    // that inits but never issues its part of the gather would otherwise
    // keep this thread (and RCCL's kernel) waiting for ever.  Given up on
    // (abandoned by the caller, or this thread's own deadline), the new
    // communicators are aborted, so RCCL's kernels return and the streams
    // drain before the buffers are freed.
    bool quit = false;
    for (size_t i = 0; i < k && going(r) && !quit;) {
      ncclResult_t st2 = ncclInProgress;
      if (R->CommGetAsyncError(comms[i], &st2) != ncclSuccess) st2 = ncclInternalError;
      (void)hipSetDevice(devs[i]);
      const hipError_t q = hipStreamQuery(st[i]);
      if (st2 != ncclSuccess && st2 != ncclInProgress) {
        r = st2;
      } else if (q == hipSuccess && st2 == ncclSuccess) {
        ++i;
      } else if (q != hipSuccess && q != hipErrorNotReady) {
        r = ncclUnhandledCudaError;
      } else if (job_abandoned(job) || until.passed()) {
        quit = true;
        r = ncclInProgress;
      } else {
        b.pause();
      }
    }
    if (r != ncclSuccess) {
      for (size_t i = 0; i < k; ++i)
        if (comms[i] && hipSetDevice(devs[i]) == hipSuccess) (void)R->CommAbort(comms[i]);
      comms.assign(k, nullptr);
    }
    // (an aborted gather returns; a stream still busy after 10 s keeps its
    // buffer: leaked rather than freed under a running kernel)
    const Deadline drain(10000);
    Backoff b2;
    for (size_t i = 0; i < k; ++i) {
      (void)hipSetDevice(devs[i]);
      bool idle = !st[i];
      while (!idle) {
        const hipError_t q = hipStreamQuery(st[i]);
        idle = q != hipErrorNotReady;
        if (!idle && drain.passed()) break;
        if (!idle) b2.pause();
      }
      if (idle && buf[i]) (void)hipFree(buf[i]);
      if (idle && st[i]) (void)hipStreamDestroy(st[i]);
    }
    COMM_TRACE("init job: warm-up gather %d", (int)r);
  }
  bool abandoned;
  {
    std::lock_guard<std::mutex> g(job->mu);
    abandoned = job->abandoned;
    if (!abandoned) {
      job->r = r;
      job->comms = comms;
      job->done = true;
    }
  }
  if (abandoned) {   // the caller returned -ETIMEDOUT / -ECANCELED: nobody owns these
    COMM_TRACE("init job: abandoned, aborting");
    for (size_t i = 0; i < k; ++i)
      if (comms[i] && hipSetDevice(devs[i]) == hipSuccess) (void)R->CommAbort(comms[i]);
    g_abandoned.fetch_sub(1);
  } else {
    job->cv.notify_all();
  }
}

// Start the init of ranks[i] on devs[i] (i < devs.size()) of an
// nranks-rank communicator and wait for it, at most timeout_ms.  0 with
// comms filled, or -errno with nothing left behind for the caller.
// `job` is created by the caller (and published in the contexts' slots,
// so that pptk_rx_comm_abort can cancel it: -ECANCELED).  -EAGAIN when too
// many earlier helpers are still stuck (kMaxAbandoned).
int bounded_init(const Rccl *R, const std::shared_ptr<InitJob> &job, const ncclUniqueId &id,
                 const std::vector<int> &devs, const std::vector<int> &ranks,
                 const std::vector<int> &caps, int nranks, uint32_t timeout_ms,
                 std::vector<ncclComm_t> &comms) {
  if (g_abandoned.load() >= kMaxAbandoned) return -EAGAIN;
  try {
    std::thread(init_run, R, job, id, devs, ranks, caps, nranks, timeout_ms).detach();
  } catch (...) {
    return -EAGAIN;
  }
  const auto until = Clock::now() + std::chrono::milliseconds(timeout_ms);
  std::unique_lock<std::mutex> g(job->mu);
  const bool done = job->cv.wait_until(g, until, [&] { return job->done || job->cancelled; });
  if (!job->done) {
    job->abandoned = true;   // the helper aborts what it builds and counts itself out
    g_abandoned.fetch_add(1);
    COMM_TRACE("create: %s, init abandoned", done ? "cancelled" : "deadline passed");
    return done ? -ECANCELED : -ETIMEDOUT;
  }
  const ncclResult_t r = job->r;
  const bool cancelled = job->cancelled;
  comms = job->comms;
  g.unlock();
  if (r == ncclSuccess && !cancelled) return 0;
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (size_t i = 0; i < comms.size(); ++i)
    if (comms[i] && hipSetDevice(devs[i]) == hipSuccess) (void)R->CommAbort(comms[i]);
  if (prev >= 0) (void)hipSetDevice(prev);
  comms.clear();
  if (cancelled) return -ECANCELED;
  return r == ncclInProgress ? -ETIMEDOUT : nccl_err(r);
}

// Publish a creation in progress in each context's slot.  -ECANCELED (and
// the pending aborts consumed) if an abort is pending on any of them,
// -EINVAL if one already has a communicator or a creation in progress.
int begin_create(pptk_rx_ctx *const *ctxs, int n, const std::shared_ptr<InitJob> &job,
                 std::vector<RxComm *> &ms) {
  std::lock_guard<std::mutex> g(g_slots);
  bool pending = false;
  for (int i = 0; i < n; ++i) {
    RxComm *m = comm_of(ctxs[i]);
    if (m && m->state != CommState::kPendingAbort) return -EINVAL;
    pending = pending || m != nullptr;
  }
  if (pending) {
    for (int i = 0; i < n; ++i)
      if (RxComm *m = comm_of(ctxs[i])) {
        set_comm(ctxs[i], nullptr);
        delete m;
      }
    return -ECANCELED;
  }
  ms.assign((size_t)n, nullptr);
  for (int i = 0; i < n; ++i) {
    RxComm *m = new (std::nothrow) RxComm();
    if (!m) {
      for (int k = 0; k < i; ++k) {
        set_comm(ctxs[k], nullptr);
        delete ms[(size_t)k];
      }
      return -ENOMEM;
    }
    m->state = CommState::kCreating;
    m->job = job;
    ms[(size_t)i] = m;
    set_comm(ctxs[i], m);
  }
  return 0;
}

// End a creation: on success the contexts' communicators go live (unless an
// abort arrived after the init finished: then they are aborted and the
// call fails with -ECANCELED); on failure the slots are cleared.
int end_create(const Rccl *R, pptk_rx_ctx *const *ctxs, int n, std::vector<RxComm *> &ms,
               const std::vector<ncclComm_t> &comms, int rc) {
  std::lock_guard<std::mutex> g(g_slots);
  if (rc == 0) {
    bool cancelled = false;
    for (int i = 0; i < n; ++i) {
      std::lock_guard<std::mutex> gm(ms[(size_t)i]->mu);
      std::lock_guard<std::mutex> gj(ms[(size_t)i]->job->mu);
      cancelled = cancelled || ms[(size_t)i]->job->cancelled;
    }
    if (!cancelled) {
      for (int i = 0; i < n; ++i) {
        RxComm *m = ms[(size_t)i];
        std::lock_guard<std::mutex> gm(m->mu);
        m->comm = comms[(size_t)i];
        m->state = CommState::kReady;
        m->job.reset();
      }
      return 0;
    }
    for (int i = 0; i < n; ++i) {
      DeviceScope ds(ctx_device(ctxs[i]));
      (void)R->CommAbort(comms[(size_t)i]);
    }
    rc = -ECANCELED;
  }
  for (int i = 0; i < n; ++i) {
    set_comm(ctxs[i], nullptr);
    delete ms[(size_t)i];
  }
  return rc;
}

}  // namespace

namespace pptk {

void comm_release(pptk_rx_ctx *c) {
  RxComm *m = comm_of(c);
  if (!m) return;
  if (m->state == CommState::kReady)
    if (const Rccl *R = rccl()) teardown(R, m, ctx_comm_timeout_ms(c));
  std::lock_guard<std::mutex> g(g_slots);
  set_comm(c, nullptr);
  { std::lock_guard<std::mutex> gm(m->mu); }   // (an abort still inside RCCL ends first)
  delete m;
}

}  // namespace pptk

extern "C" {

#ifdef PPTK_RX_TEST_HOOKS
// The test library's view of the communicator configuration a context with
// `coll_cus` split CUs creates (tests/test_capi.py, no GPU needed).
int pptk_rx_test_comm_config(int coll_cus, int *blocking, int *min_ctas, int *max_ctas) {
  const ncclConfig_t cfg = comm_config(coll_cus);
  if (blocking) *blocking = cfg.blocking;
  if (min_ctas) *min_ctas = cfg.minCTAs;
  if (max_ctas) *max_ctas = cfg.maxCTAs;
  return 0;
}
#endif

int pptk_rx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -EIO;
  return n;
}

int pptk_rx_comm_uid(uint8_t uid[PPTK_RX_COMM_UID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == PPTK_RX_COMM_UID_BYTES, "RCCL unique id size");
  if (!uid) return -EINVAL;
  const Rccl *R = rccl();
  if (!R) return -ENOSYS;
  ncclUniqueId id;
  const int rc = nccl_err(R->GetUniqueId(&id));
  if (rc == 0) memcpy(uid, &id, sizeof(id));
  return rc;
}

int pptk_rx_comm_create(struct pptk_rx_ctx *c, int nranks, int rank,
                        const uint8_t uid[PPTK_RX_COMM_UID_BYTES]) {
  if (!c || !uid || nranks < 1 || rank < 0 || rank >= nranks) return -EINVAL;
  const Rccl *R = rccl();
  if (!R) return -ENOSYS;
  std::shared_ptr<InitJob> job;
  try {
    job = std::make_shared<InitJob>();
  } catch (...) {
    return -ENOMEM;
  }
  std::vector<RxComm *> ms;
  int rc = begin_create(&c, 1, job, ms);
  if (rc != 0) return rc;
  ms[0]->nranks = nranks;
  ms[0]->rank = rank;
  ncclUniqueId id;
  memcpy(&id, uid, sizeof(id));
  COMM_TRACE("create: init rank %d of %d", rank, nranks);
  std::vector<ncclComm_t> comms;
  rc = bounded_init(R, job, id, {ctx_device(c)}, {rank}, {ctx_coll_cap(c)}, nranks,
                    ctx_comm_timeout_ms(c), comms);
  COMM_TRACE("create: %d", rc);
  return end_create(R, &c, 1, ms, comms, rc);
}

int pptk_rx_comm_create_all(struct pptk_rx_ctx *const *ctxs, int n) {
  if (!ctxs || n < 1) return -EINVAL;
  std::vector<int> devs((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return -EINVAL;
    devs[(size_t)i] = ctx_device(ctxs[i]);
    for (int k = 0; k < i; ++k)   // one rank per GPU
      if (devs[(size_t)k] == devs[(size_t)i] || ctxs[k] == ctxs[i]) return -EINVAL;
  }
  const Rccl *R = rccl();
  if (!R) return -ENOSYS;
  ncclUniqueId id;
  int rc = nccl_err(R->GetUniqueId(&id));
  if (rc != 0) return rc;
  std::shared_ptr<InitJob> job;
  try {
    job = std::make_shared<InitJob>();
  } catch (...) {
    return -ENOMEM;
  }
  std::vector<RxComm *> ms;
  if ((rc = begin_create(ctxs, n, job, ms)) != 0) return rc;
  for (int i = 0; i < n; ++i) {
    ms[(size_t)i]->nranks = n;
    ms[(size_t)i]->rank = i;
  }
  // one group of per-device inits (what ncclCommInitAll does), bounded
  std::vector<int> ranks((size_t)n), caps((size_t)n);
  for (int i = 0; i < n; ++i) {
    ranks[(size_t)i] = i;
    caps[(size_t)i] = ctx_coll_cap(ctxs[i]);
  }
  std::vector<ncclComm_t> comms;
  rc = bounded_init(R, job, id, devs, ranks, caps, n, ctx_comm_timeout_ms(ctxs[0]), comms);
  return end_create(R, ctxs, n, ms, comms, rc);
}

int pptk_rx_comm_destroy(struct pptk_rx_ctx *c) {
  if (!c) return -EINVAL;
  RxComm *m = comm_of(c);
  if (m && m->state == CommState::kCreating) return -EBUSY;
  DeviceScope ds(ctx_device(c));
  comm_release(c);   // (also drops a pending abort)
  return 0;
}

int pptk_rx_comm_abort(struct pptk_rx_ctx *c) {
  if (!c) return -EINVAL;
  std::unique_lock<std::mutex> g(g_slots);
  RxComm *m = comm_of(c);
  if (!m) {   // nothing to cancel yet: the context's next creation is
    m = new (std::nothrow) RxComm();
    if (!m) return -ENOMEM;
    m->state = CommState::kPendingAbort;
    set_comm(c, m);
    return 0;
  }
  std::unique_lock<std::mutex> gm(m->mu);
  if (m->state == CommState::kPendingAbort) return 0;
  if (m->state == CommState::kCreating) {
    {
      std::lock_guard<std::mutex> gj(m->job->mu);
      m->job->cancelled = true;
    }
    m->job->cv.notify_all();
    return 0;
  }
  // A live communicator: RCCL's abort can block while its kernels drain, so
  // it runs under the communicator's own lock only -- every other context's
  // create, destroy and abort go on meanwhile.  Nothing frees this RxComm
  // while its lock is held: a live slot is deleted only by
  // pptk_rx_comm_destroy / pptk_rx_ctx_destroy of this context (which must
  // not race with this call, pptk_rx.h) after taking the same lock.
  g.unlock();
  const Rccl *R = rccl();
  if (!R) return -ENOSYS;
  DeviceScope ds(ctx_device(c));
  abort_locked(R, m);
  return 0;
}

int pptk_rx_comm_info(const struct pptk_rx_ctx *c, int *nranks, int *rank) {
  if (!c) return -EINVAL;
  const RxComm *m = live_comm_of(c);
  if (!m) return -EINVAL;
  if (nranks) *nranks = m->nranks;
  if (rank) *rank = m->rank;
  return 0;
}

void pptk_rx_shard_range(uint64_t n, int nranks, int rank, uint64_t *first, uint64_t *count,
                         uint64_t *per_rank) {
  uint64_t per = 0, lo = 0, cnt = 0;
  if (nranks >= 1 && rank >= 0 && rank < nranks) {
    per = (n + (uint64_t)nranks - 1) / (uint64_t)nranks;
    lo = (uint64_t)rank * per;
    if (lo > n) lo = n;
    cnt = n - lo < per ? n - lo : per;
  }
  if (first) *first = lo;
  if (count) *count = cnt;
  if (per_rank) *per_rank = per;
}

int pptk_rx_allgather_hash(struct pptk_rx_ctx *c, const uint64_t *d_hash, uint64_t n,
                           uint64_t *d_out, void *stream) {
  if (!c) return -EINVAL;
  RxComm *m = live_comm_of(c);
  if (!m) return -EINVAL;
  if (n == 0) return 0;
  if (!d_hash || !d_out) return -EINVAL;
  const Rccl *R = rccl();
  if (!R) return -ENOSYS;
  DeviceScope ds(ctx_device(c));
  if (!ds.ok) return -EIO;
  const Deadline d(ctx_comm_timeout_ms(c));
  Backoff b;
  std::unique_lock<std::mutex> g(m->mu);
  if (m->aborted) return -ECANCELED;
  ncclResult_t st = ncclSuccess;
  if (R->CommGetAsyncError(m->comm, &st) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress))
    return -EIO;   // an earlier collective failed: sync/abort, then a new communicator
  ncclResult_t r = R->AllGather(d_hash, d_out, (size_t)n, ncclUint64, m->comm, (hipStream_t)stream);
  // A non-blocking communicator may return while the enqueue (e.g. RCCL's
  // lazy connection setup with the peers at the first collective) goes on;
  // the call is complete once the state leaves ncclInProgress.  The lock is
  // dropped between polls so pptk_rx_comm_abort can cancel the wait.
  while (r == ncclInProgress) {
    ncclResult_t now = ncclInProgress;
    if (R->CommGetAsyncError(m->comm, &now) != ncclSuccess) return -EIO;
    r = now;
    if (r != ncclInProgress) break;
    if (d.passed()) {
      abort_locked(R, m);
      return -ETIMEDOUT;
    }
    g.unlock();
    b.pause();
    g.lock();
    if (m->aborted) return -ECANCELED;
  }
  return nccl_err(r);
}

int pptk_rx_comm_sync(struct pptk_rx_ctx *c, void *stream, uint32_t timeout_ms) {
  if (!c) return -EINVAL;
  RxComm *m = live_comm_of(c);
  const Rccl *R = m ? rccl() : nullptr;
  DeviceScope ds(ctx_device(c));
  if (!ds.ok) return -EIO;
  const hipStream_t s = (hipStream_t)stream;
  const Deadline d(timeout_ms ? timeout_ms : ctx_comm_timeout_ms(c));
  Backoff b;
  int rc = 0;
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) return -EIO;
    if (m && R) {
      std::lock_guard<std::mutex> g(m->mu);
      if (m->aborted) {
        rc = -ECANCELED;
        break;
      }
      ncclResult_t st = ncclSuccess;
      if (R->CommGetAsyncError(m->comm, &st) != ncclSuccess ||
          (st != ncclSuccess && st != ncclInProgress)) {
        abort_locked(R, m);
        rc = -EIO;
        break;
      }
      if (d.passed()) {
        abort_locked(R, m);
        rc = -ETIMEDOUT;
        break;
      }
    } else if (d.passed()) {
      return -ETIMEDOUT;   // no communicator to cancel: the stream is just slow
    }
    b.pause();
  }
  if (rc == 0) {
    if (m && R) {   // an error reported after the last kernel finished
      std::lock_guard<std::mutex> g(m->mu);
      ncclResult_t st = ncclSuccess;
      if (!m->aborted && (R->CommGetAsyncError(m->comm, &st) != ncclSuccess ||
                          (st != ncclSuccess && st != ncclInProgress))) {
        abort_locked(R, m);
        return -EIO;
      }
    }
    return 0;
  }
  // Aborted: RCCL's kernels see the abort flag and return, so the stream
  // drains; wait for that (bounded: this call must not become the hang).
  const Deadline drain(10000);
  Backoff b2;
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q != hipErrorNotReady || drain.passed()) break;
    b2.pause();
  }
  return rc;
}

}  // extern "C"
