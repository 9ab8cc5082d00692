/*
 * rx_multigpu.c -- one process driving every GPU of the node: one rx thread
 * and one pptk_rx_ctx per GPU, one RCCL communicator over all of them, the
 * batch sharded by pptk_rx_shard_range, and the flow hashes all-gathered so
 * every GPU holds the hash of every frame (the C8G configuration of
 * BASELINE.json, single-process form; bench.py runs the one-process-per-GPU
 * form).
 *
 * Each thread, like an ldp/ldprecvmt.c:16-67 queue thread: takes its device
 * frame and record rings from pptk_rx_ring_alloc and its two gather buffers
 * from pptk_rx_gather_alloc (both placed by the library's probe: what the
 * record, hash and gather writes cost beside the frame stream depends on
 * where the buffers sit, DESIGN.md sections 7-8; each rank prints the
 * placement it got), copies its shard of the frame set into the frame ring,
 * runs pptk_rx_batch_device with d_hash aimed at its own slice of gather
 * buffer r % 2, then pptk_rx_allgather_hash in place on the same stream, and
 * checks its records and the whole gathered hash array against the expected
 * records of the set file.
 *
 * Failure containment.  The reference's queue threads share nothing
 * (ldp/ldprecvmt.c:174-182), so one failing thread cannot stall the others;
 * here the gather ties them together, so a thread that fails anywhere calls
 * fail_all(), which aborts every context's communicator
 * (pptk_rx_comm_abort): siblings waiting for a gather it will never join
 * get -ECANCELED from pptk_rx_comm_sync (never hipStreamSynchronize on a
 * gather stream), siblings still inside (or not yet in) pptk_rx_comm_create
 * get -ECANCELED from it at once, and the process exits non-zero instead of
 * hanging.  A rank that never joins without failing makes the others'
 * pptk_rx_comm_create return -ETIMEDOUT after opts.comm_timeout_ms.
 *
 *   gcc -O2 -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude \
 *       examples/rx_multigpu.c -Lpptk_amd -lpptkrx -L/opt/rocm/lib -lamdhip64 -o rx_multigpu
 *   ./rx_multigpu frames.rxq [ranks [rounds [split_cus]]]
 *
 * ranks defaults to the visible GPUs; rank r runs on GPU r % visible.
 * split_cus > 0 overlaps each gather with the next batch: the batches on one
 * stream, the gathers on another, the chip's CUs split between them with
 * pptk_rx_stream_split (split_cus CUs for the gathers; RCCL's kernel needs
 * whole CUs), batch r waiting for gather r - 2 (same buffer).
 * The split is made in main, before the communicator: the library then caps
 * the communicator's channels at split_cus (one RCCL block per CU left to
 * the gathers), and the two streams belong to the context, which destroys
 * them after its communicator.
 * Environment (tests, drills):
 *   RX_MULTIGPU_JOIN=threads   every thread joins with pptk_rx_comm_create on
 *                              a uid made by main (the per-process form, in
 *                              threads) instead of pptk_rx_comm_create_all
 *   RX_MULTIGPU_FAIL=r         rank r's thread fails: before joining (JOIN=
 *                              threads) or before its first gather
 *   RX_MULTIGPU_TIMEOUT_MS=t   opts.comm_timeout_ms
 *   RX_MULTIGPU_TRACE=1        progress lines on stderr
 */
#include <errno.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "pptk_rx.h"
#include "rxq_file.h"

#define MAXR 64

static struct pptk_rx_ctx *g_ctx[MAXR];
static int g_nranks;
static atomic_int g_failed;
static int g_join_threads, g_fail_rank = -1;
static int g_split;   /* split_cus */
static uint8_t g_uid[PPTK_RX_COMM_UID_BYTES];
static int g_trace;

static void trace(const char *fmt, ...)
{
  struct timespec ts;
  va_list ap;
  if (!g_trace)
    return;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  fprintf(stderr, "[%ld.%03ld] ", (long)ts.tv_sec, ts.tv_nsec / 1000000);
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}

/* Cancel every communicator once: no sibling keeps waiting for a gather
 * the failed thread will not issue. */
static void fail_all(void)
{
  if (atomic_exchange(&g_failed, 1))
    return;
  for (int i = 0; i < g_nranks; i++) {
    int rc = pptk_rx_comm_abort(g_ctx[i]);   /* also cancels a creation in progress or to come */
    trace("fail_all: abort rank %d: %d", i, rc);
  }
}

struct gpu_thread {
  int rank, nranks, rounds, device;
  struct pptk_rx_ctx *ctx;
  const struct rxq_set *set;
  unsigned long rec_mismatches, hash_mismatches;
  int rc;
  /* split_cus > 0: the context's split streams (pptk_rx_stream_split in
   * main, before the communicator; the context owns and destroys them) */
  hipStream_t split_st, split_cs;
};

#define CHECK_HIP(x)                 \
  do {                               \
    if ((x) != hipSuccess) {         \
      t->rc = -EIO;                  \
      goto out;                      \
    }                                \
  } while (0)

static void *thrfn(void *arg)
{
  struct gpu_thread *t = arg;
  const struct rxq_set *s = t->set;
  const uint64_t n = s->h.n;
  uint64_t first, count, per;
  uint64_t *d_off = NULL, *d_out = NULL, *h_off = NULL, *h_out = NULL;
  uint16_t *d_len = NULL;
  struct pptk_rx_rec *h_recs = NULL;
  hipStream_t st = NULL, cs = NULL;   /* batches; gathers (split_cus > 0) */
  hipEvent_t kdone[2] = {NULL, NULL}, gdone[2] = {NULL, NULL};
  uint64_t lo = 0, hi = 0;
  struct pptk_rx_dev_batch b;
  struct pptk_rx_ring ring;
  struct pptk_rx_ring_spec rs;
  struct pptk_rx_gather gat;
  struct pptk_rx_gather_spec gs;

  memset(&ring, 0, sizeof(ring));
  memset(&gat, 0, sizeof(gat));

  if (g_join_threads) {   /* collective: every rank's thread joins */
    if (t->rank == g_fail_rank) {
      t->rc = -ECANCELED;   /* drill: this rank never joins */
      goto out;
    }
    trace("rank %d: joining", t->rank);
    t->rc = pptk_rx_comm_create(t->ctx, t->nranks, t->rank, g_uid);
    trace("rank %d: pptk_rx_comm_create %d", t->rank, t->rc);
    if (t->rc != 0)
      goto out;
  }
  pptk_rx_shard_range(n, t->nranks, t->rank, &first, &count, &per);
  if (count) {   /* the shard's bytes, offsets rebased to its first frame */
    lo = s->off[first];
    for (uint64_t i = first; i < first + count; i++) {
      uint64_t e = s->off[i] + s->len[i];
      if (s->off[i] < lo)
        lo = s->off[i];
      if (e > hi)
        hi = e;
    }
  }
  CHECK_HIP(hipSetDevice(t->device));
  if (t->split_cs) {
    /* the rings' and gather buffers' probes run on the batches' stream, with
     * the grid the split leaves it */
    st = t->split_st;
    cs = t->split_cs;
    for (int k = 0; k < 2; k++) {
      CHECK_HIP(hipEventCreateWithFlags(&kdone[k], hipEventDisableTiming));
      CHECK_HIP(hipEventCreateWithFlags(&gdone[k], hipEventDisableTiming));
    }
  } else {
    CHECK_HIP(hipStreamCreate(&st));
  }
  /* the frame and record rings of this queue, placed by the library */
  memset(&rs, 0, sizeof(rs));
  rs.frame_bytes = hi - lo + 64;
  rs.nrec = count ? count : 1;
  rs.rec_bytes = sizeof(struct pptk_rx_rec);
  rs.probe_len = rs.frame_bytes >= 1500 ? 0 : (uint32_t)rs.frame_bytes;
  /* the gather probe below runs after the scrub; the ring probe writes the
   * dense hashes too, as this queue's batches do */
  rs.flags = PPTK_RX_RING_SETTLE | PPTK_RX_RING_PROBE_HASH;
  if ((t->rc = pptk_rx_ring_alloc(t->ctx, &rs, &ring, st)) != 0)
    goto out;
  CHECK_HIP(hipMalloc((void **)&d_off, count * 8 + 8));
  CHECK_HIP(hipMalloc((void **)&d_len, count * 2 + 2));
  h_off = malloc(count * 8 + 8);
  h_out = malloc(per * (uint64_t)t->nranks * 8 + 8);
  h_recs = malloc(count * sizeof(struct pptk_rx_rec) + 64);
  if (!h_off || !h_out || !h_recs) {
    t->rc = -ENOMEM;
    goto out;
  }
  for (uint64_t i = 0; i < count; i++)
    h_off[i] = s->off[first + i] - lo;
  CHECK_HIP(hipMemcpy(ring.d_frames, s->buf + lo, hi - lo + 16, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_off, h_off, count * 8, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_len, s->len + first, count * 2, hipMemcpyHostToDevice));
  if (!g_join_threads && t->rank == g_fail_rank) {
    t->rc = -ECANCELED;   /* drill: fail before the first gather */
    goto out;
  }

  memset(&b, 0, sizeof(b));
  b.d_frames = ring.d_frames;
  b.d_off = d_off;
  b.d_len = d_len;
  b.max_len = 65535;
  b.n = count;
  b.d_recs = ring.d_recs;
  /* the two gather buffers, placed by the library with this batch */
  memset(&gs, 0, sizeof(gs));
  gs.per_rank = per;
  gs.nranks = t->nranks;
  gs.rank = t->rank;
  if ((t->rc = pptk_rx_gather_alloc(t->ctx, &b, &gs, &gat, st)) != 0)
    goto out;
  printf("rank %d: rings placed: pair (%d, %d) of %u x %u candidates, probe %.4f ms "
         "(plain allocation %.4f ms); gather region %d of %u, probe %.4f ms (plain %.4f ms)\n",
         t->rank, ring.chosen_frames, ring.chosen_recs, ring.frame_cands, ring.rec_cands,
         ring.chosen_ms, ring.first_ms, gat.chosen, gat.cands, gat.chosen_ms, gat.first_ms);
  for (int r = 0; r < t->rounds && t->rc == 0; r++) {
    d_out = gat.d_out[r & 1];   /* double-buffered, as an rx loop overlapping gathers does */
    b.d_hash = d_out + (uint64_t)t->rank * per;   /* this rank's slice: gather in place */
    if (cs && r >= 2)   /* the gather of round r - 2 has read this buffer */
      CHECK_HIP(hipStreamWaitEvent(st, gdone[r & 1], 0));
    if ((t->rc = pptk_rx_batch_device(t->ctx, &b, st)) != 0)
      break;
    if (cs) {   /* the gather beside the next batch, on the CUs left to it */
      CHECK_HIP(hipEventRecord(kdone[r & 1], st));
      CHECK_HIP(hipStreamWaitEvent(cs, kdone[r & 1], 0));
      if ((t->rc = pptk_rx_allgather_hash(t->ctx, b.d_hash, per, d_out, cs)) != 0)
        break;
      CHECK_HIP(hipEventRecord(gdone[r & 1], cs));
      continue;
    }
    if ((t->rc = pptk_rx_allgather_hash(t->ctx, b.d_hash, per, d_out, st)) != 0)
      break;
    /* bounded wait with RCCL error checks: -ECANCELED once a sibling failed */
    t->rc = pptk_rx_comm_sync(t->ctx, st, 0);
  }
  if (cs && t->rc == 0 && (t->rc = pptk_rx_comm_sync(t->ctx, cs, 0)) == 0)
    t->rc = pptk_rx_comm_sync(t->ctx, st, 0);
  if (t->rc)
    goto out;
  CHECK_HIP(hipMemcpy(h_recs, ring.d_recs, count * sizeof(struct pptk_rx_rec), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(h_out, d_out, per * (uint64_t)t->nranks * 8, hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < count; i++)
    if (memcmp(&h_recs[i], &s->want[first + i], sizeof(h_recs[i])) != 0)
      t->rec_mismatches++;
  for (uint64_t i = 0; i < n; i++)   /* global frame i sits at index i */
    if (h_out[i] != s->want[i].flow_hash)
      t->hash_mismatches++;
out:
  trace("rank %d: done, rc %d", t->rank, t->rc);
  if (t->rc)
    fail_all();
  if (cs)
    (void)pptk_rx_comm_sync(t->ctx, cs, 0);
  if (st)   /* drained: aborted gathers return, pptk_rx_comm_sync waited */
    (void)pptk_rx_comm_sync(t->ctx, st, 0);
  for (int k = 0; k < 2; k++) {   /* (drained above) */
    if (kdone[k])
      (void)hipEventDestroy(kdone[k]);
    if (gdone[k])
      (void)hipEventDestroy(gdone[k]);
  }
  if (st && !cs)   /* our own stream; the split ones are the context's */
    (void)hipStreamDestroy(st);
  (void)pptk_rx_ring_free(&ring);
  trace("rank %d: ring freed", t->rank);
  (void)pptk_rx_gather_free(&gat);
  (void)hipFree(d_off);
  (void)hipFree(d_len);
  free(h_off);
  free(h_out);
  free(h_recs);
  trace("rank %d: exit", t->rank);
  return NULL;
}

int main(int argc, char **argv)
{
  struct rxq_set set;
  int ndev = pptk_rx_device_count();
  int nr = argc > 2 ? atoi(argv[2]) : ndev, rounds = argc > 3 ? atoi(argv[3]) : 3;
  int split = argc > 4 ? atoi(argv[4]) : 0;
  const char *e;
  uint32_t timeout_ms = 0;
  struct gpu_thread thr[MAXR];
  pthread_t pth[MAXR];
  unsigned long bad = 0;
  int i, rc, failed = 0;

  setvbuf(stdout, NULL, _IOLBF, 0);   /* every line out before anything can go wrong */
  if (argc < 2 || rxq_load(argv[1], &set) != 0) {
    fprintf(stderr, "usage: rx_multigpu frames.rxq [ranks [rounds [split_cus]]]\n");
    return 1;
  }
  if (ndev < 1 || nr < 1 || nr > MAXR) {
    fprintf(stderr, "%d ranks requested, %d GPUs visible\n", nr, ndev);
    return 1;
  }
  g_join_threads = (e = getenv("RX_MULTIGPU_JOIN")) && !strcmp(e, "threads");
  g_split = split;
  if ((e = getenv("RX_MULTIGPU_FAIL")))
    g_fail_rank = atoi(e);
  g_trace = (e = getenv("RX_MULTIGPU_TRACE")) && *e == '1';
  if ((e = getenv("RX_MULTIGPU_TIMEOUT_MS")))
    timeout_ms = (uint32_t)strtoul(e, NULL, 10);
  g_nranks = nr;
  for (i = 0; i < nr; i++) {
    struct pptk_rx_opts o;
    pptk_rx_opts_default(&o);
    o.device = i % ndev;
    memcpy(o.key, set.h.key, 16);
    o.iphash_bits4 = 24;
    o.iphash_bits6 = 48;
    o.iphash_size = 4096;
    if (timeout_ms)
      o.comm_timeout_ms = timeout_ms;
    if ((rc = pptk_rx_ctx_create(&g_ctx[i], &o)) != 0) {
      fprintf(stderr, "pptk_rx_ctx_create(%d): %d\n", i, rc);
      return 1;
    }
    thr[i] = (struct gpu_thread){.rank = i, .nranks = nr, .rounds = rounds, .device = i % ndev,
                                 .ctx = g_ctx[i], .set = &set};
    if (g_split) {   /* before the communicator: it caps its channels at g_split */
      void *rx_s = NULL, *coll_s = NULL;
      if ((rc = pptk_rx_stream_split(g_ctx[i], g_split, &rx_s, &coll_s)) != 0) {
        fprintf(stderr, "pptk_rx_stream_split(%d, %d): %d\n", i, g_split, rc);
        return 1;
      }
      thr[i].split_st = rx_s;
      thr[i].split_cs = coll_s;
    }
  }
  if (g_join_threads)
    rc = pptk_rx_comm_uid(g_uid);
  else
    rc = pptk_rx_comm_create_all(g_ctx, nr);
  if (rc != 0) {
    fprintf(stderr, "%s: %d\n", g_join_threads ? "pptk_rx_comm_uid" : "pptk_rx_comm_create_all",
            rc);
    return 1;
  }
  for (i = 0; i < nr; i++) {
    if (pthread_create(&pth[i], NULL, thrfn, &thr[i]) != 0) {
      fail_all();
      nr = i;   /* join the ones started */
      failed = 1;
      break;
    }
  }
  for (i = 0; i < nr; i++) {
    int cr = 0, r = -1;
    pthread_join(pth[i], NULL);
    pptk_rx_comm_info(g_ctx[i], &cr, &r);
    printf("rank %d (GPU %d; communicator rank %d of %d): %lu record mismatches, "
           "%lu gathered-hash mismatches, rc %d\n",
           i, thr[i].device, r, cr, thr[i].rec_mismatches, thr[i].hash_mismatches, thr[i].rc);
    failed |= thr[i].rc != 0;
    bad += thr[i].rec_mismatches + thr[i].hash_mismatches;
  }
  for (i = 0; i < g_nranks; i++) {
    if (thr[i].split_cs) {   /* the context's streams: not the caller's to destroy */
      rc = pptk_rx_stream_destroy(thr[i].split_cs);
      printf("rank %d: pptk_rx_stream_destroy(gather stream) before the context: %d%s\n", i, rc,
             rc == -EBUSY ? " (EBUSY: the context owns it)" : "");
      if (rc != -EBUSY)
        failed = 1;
    }
    trace("destroying context %d", i);
    pptk_rx_ctx_destroy(g_ctx[i]);   /* its communicator, then its split streams */
  }
  trace("contexts destroyed");
  printf("rx_multigpu: %d ranks on %d GPUs, %u frames, %lu mismatches%s\n", g_nranks,
         g_nranks < ndev ? g_nranks : ndev, set.h.n, bad, failed ? ", FAILED" : "");
  rxq_free(&set);
  /* An RCCL init that a deadline or an abort made pptk_rx_comm_create give
   * up on may still be running in the library's helper thread (RCCL 2.27's
   * init does not return while a rank is missing).  exit() would run the
   * HIP and RCCL library destructors under it; leave without them. */
  fflush(stdout);
  fflush(stderr);
  _exit(failed ? 1 : bad ? 2 : 0);
}
