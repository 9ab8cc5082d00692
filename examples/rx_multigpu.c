/*
 * rx_multigpu.c -- one process driving every GPU of the node: one rx thread
 * and one pptk_rx_ctx per GPU, one RCCL communicator over all of them
 * (pptk_rx_comm_create_all), the batch sharded by pptk_rx_shard_range, and
 * the flow hashes all-gathered so every GPU holds the hash of every frame
 * (the C8G configuration of BASELINE.json, single-process form; bench.py
 * runs the one-process-per-GPU form).
 *
 * Each thread, like an ldp/ldprecvmt.c:16-67 queue thread: copies its shard
 * of the frame set to its GPU, runs pptk_rx_batch_device with d_hash aimed
 * at its own slice of the gather buffer, then pptk_rx_allgather_hash in
 * place on the same stream, and checks its records and the whole gathered
 * hash array against the expected records of the set file.
 *
 *   gcc -O2 -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude \
 *       examples/rx_multigpu.c -Lpptk_amd -lpptkrx -L/opt/rocm/lib -lamdhip64 -o rx_multigpu
 *   ./rx_multigpu frames.rxq [gpus [rounds]]
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "pptk_rx.h"
#include "rxq_file.h"

struct gpu_thread {
  int rank, nranks, rounds;
  struct pptk_rx_ctx *ctx;
  const struct rxq_set *set;
  unsigned long rec_mismatches, hash_mismatches;
  int rc;
};

#define CHECK_HIP(x)                 \
  do {                               \
    if ((x) != hipSuccess) {         \
      t->rc = -5;                    \
      goto out;                      \
    }                                \
  } while (0)

static void *thrfn(void *arg)
{
  struct gpu_thread *t = arg;
  const struct rxq_set *s = t->set;
  const uint64_t n = s->h.n;
  uint64_t first, count, per;
  uint8_t *d_frames = NULL;
  uint64_t *d_off = NULL, *d_out = NULL, *h_off = NULL, *h_out = NULL;
  uint16_t *d_len = NULL;
  struct pptk_rx_rec *d_recs = NULL, *h_recs = NULL;
  hipStream_t st = NULL;
  uint64_t lo = 0, hi = 0;
  struct pptk_rx_dev_batch b;

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
  CHECK_HIP(hipSetDevice(t->rank));   /* rank i = ctxs[i] = device i */
  CHECK_HIP(hipStreamCreate(&st));
  CHECK_HIP(hipMalloc((void **)&d_frames, hi - lo + 64));
  CHECK_HIP(hipMalloc((void **)&d_off, count * 8 + 8));
  CHECK_HIP(hipMalloc((void **)&d_len, count * 2 + 2));
  CHECK_HIP(hipMalloc((void **)&d_recs, count * sizeof(struct pptk_rx_rec) + 64));
  CHECK_HIP(hipMalloc((void **)&d_out, per * (uint64_t)t->nranks * 8 + 8));
  CHECK_HIP(hipMemset(d_out, 0, per * (uint64_t)t->nranks * 8 + 8));
  h_off = malloc(count * 8 + 8);
  h_out = malloc(per * (uint64_t)t->nranks * 8 + 8);
  h_recs = malloc(count * sizeof(struct pptk_rx_rec) + 64);
  if (!h_off || !h_out || !h_recs) {
    t->rc = -12;
    goto out;
  }
  for (uint64_t i = 0; i < count; i++)
    h_off[i] = s->off[first + i] - lo;
  CHECK_HIP(hipMemcpy(d_frames, s->buf + lo, hi - lo + 16, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_off, h_off, count * 8, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_len, s->len + first, count * 2, hipMemcpyHostToDevice));

  memset(&b, 0, sizeof(b));
  b.d_frames = d_frames;
  b.d_off = d_off;
  b.d_len = d_len;
  b.max_len = 65535;
  b.n = count;
  b.d_recs = d_recs;
  b.d_hash = d_out + (uint64_t)t->rank * per;   /* this rank's slice: gather in place */
  for (int r = 0; r < t->rounds && t->rc == 0; r++) {
    if ((t->rc = pptk_rx_batch_device(t->ctx, &b, st)) != 0)
      break;
    t->rc = pptk_rx_allgather_hash(t->ctx, b.d_hash, per, d_out, st);
  }
  if (t->rc)
    goto out;
  CHECK_HIP(hipStreamSynchronize(st));
  CHECK_HIP(hipMemcpy(h_recs, d_recs, count * sizeof(struct pptk_rx_rec), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(h_out, d_out, per * (uint64_t)t->nranks * 8, hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < count; i++)
    if (memcmp(&h_recs[i], &s->want[first + i], sizeof(h_recs[i])) != 0)
      t->rec_mismatches++;
  for (uint64_t i = 0; i < n; i++)   /* global frame i sits at index i */
    if (h_out[i] != s->want[i].flow_hash)
      t->hash_mismatches++;
out:
  if (st)
    (void)hipStreamDestroy(st);
  (void)hipFree(d_frames);
  (void)hipFree(d_off);
  (void)hipFree(d_len);
  (void)hipFree(d_recs);
  (void)hipFree(d_out);
  free(h_off);
  free(h_out);
  free(h_recs);
  return NULL;
}

int main(int argc, char **argv)
{
  struct rxq_set set;
  int ndev = pptk_rx_device_count();
  int ngpu = argc > 2 ? atoi(argv[2]) : ndev, rounds = argc > 3 ? atoi(argv[3]) : 3;
  struct pptk_rx_ctx *ctxs[64];
  struct gpu_thread thr[64];
  pthread_t pth[64];
  unsigned long bad = 0;
  int i, rc, failed = 0;

  if (argc < 2 || rxq_load(argv[1], &set) != 0) {
    fprintf(stderr, "usage: rx_multigpu frames.rxq [gpus [rounds]]\n");
    return 1;
  }
  if (ngpu < 1 || ngpu > ndev || ngpu > 64) {
    fprintf(stderr, "%d GPUs requested, %d visible\n", ngpu, ndev);
    return 1;
  }
  for (i = 0; i < ngpu; i++) {
    struct pptk_rx_opts o;
    pptk_rx_opts_default(&o);
    o.device = i;
    memcpy(o.key, set.h.key, 16);
    o.iphash_bits4 = 24;
    o.iphash_bits6 = 48;
    o.iphash_size = 4096;
    if ((rc = pptk_rx_ctx_create(&ctxs[i], &o)) != 0) {
      fprintf(stderr, "pptk_rx_ctx_create(%d): %d\n", i, rc);
      return 1;
    }
  }
  if ((rc = pptk_rx_comm_create_all(ctxs, ngpu)) != 0) {
    fprintf(stderr, "pptk_rx_comm_create_all: %d\n", rc);
    return 1;
  }
  for (i = 0; i < ngpu; i++) {
    thr[i] = (struct gpu_thread){.rank = i, .nranks = ngpu, .rounds = rounds, .ctx = ctxs[i],
                                 .set = &set};
    pthread_create(&pth[i], NULL, thrfn, &thr[i]);
  }
  for (i = 0; i < ngpu; i++) {
    int nr = 0, r = -1;
    pthread_join(pth[i], NULL);
    pptk_rx_comm_info(ctxs[i], &nr, &r);
    printf("GPU %d (rank %d of %d): %lu record mismatches, %lu gathered-hash mismatches, rc %d\n",
           i, r, nr, thr[i].rec_mismatches, thr[i].hash_mismatches, thr[i].rc);
    failed |= thr[i].rc != 0;
    bad += thr[i].rec_mismatches + thr[i].hash_mismatches;
  }
  for (i = 0; i < ngpu; i++)
    pptk_rx_ctx_destroy(ctxs[i]);   /* destroys the communicator too */
  printf("rx_multigpu: %d GPUs, %u frames, %lu mismatches\n", ngpu, set.h.n, bad);
  rxq_free(&set);
  return failed ? 1 : bad ? 2 : 0;
}
