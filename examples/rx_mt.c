/*
 * rx_mt.c -- multi-queue rx with one thread and one pptk_rx_ctx per queue.
 *
 * The reference's multi-queue receiver (ldp/ldprecvmt.c:16-67, threads
 * started at :174-182) runs one thread per rx queue, each looping
 * ldp_in_nextpkts -> (per-packet work) -> ldp_in_deallocate_some on its own
 * queue.  Here every thread owns its queue (a contiguous share of the frame
 * set, as RSS would spread flows) and its own context (own streams, own
 * pinned staging; contexts spread over the visible GPUs), and the
 * per-packet work is one pptk_rx_batch() per burst of up to BURST frames.
 * Every record is compared with the expected one from the set file, on
 * every lap.
 *
 *   gcc -O2 -pthread -Iinclude examples/rx_mt.c -Lpptk_amd -lpptkrx -o rx_mt
 *   ./rx_mt frames.rxq [threads [laps]]
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "pptk_rx.h"
#include "rxq_file.h"

#define BURST 1000 /* ldp/ldprecvmt.c:23: struct ldp_packet pkt_tbl[1000] */

struct rxq_thread {
  int id, device, laps;
  const struct rxq_set *set;
  uint32_t first, count;   /* this thread's queue */
  unsigned long pkts, mismatches;
  int rc;
};

static double now(void)
{
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec + tv.tv_usec * 1e-6;
}

static void *thrfn(void *arg)
{
  struct rxq_thread *t = arg;
  const struct rxq_set *s = t->set;
  static __thread struct ldp_packet pkt_tbl[BURST];
  static __thread struct pptk_rx_rec recs[BURST];
  struct pptk_rx_opts o;
  struct pptk_rx_ctx *ctx;
  pptk_rx_opts_default(&o);
  o.device = t->device;
  memcpy(o.key, s->h.key, 16);
  o.iphash_bits4 = 24;           /* the golden sets' ip_hash parameters */
  o.iphash_bits6 = 48;
  o.iphash_size = 4096;
  o.max_batch = 256;
  o.max_frame = 65535;
  if ((t->rc = pptk_rx_ctx_create(&ctx, &o)) != 0)
    return NULL;
  for (int lap = 0; lap < t->laps && t->rc == 0; lap++) {
    uint32_t head = 0;
    while (head < t->count) {
      /* num = ldp_in_nextpkts(intf->inq[id], pkt_tbl, BURST); */
      int num = t->count - head < BURST ? (int)(t->count - head) : BURST;
      for (int i = 0; i < num; i++) {
        uint32_t k = t->first + head + (uint32_t)i;
        pkt_tbl[i].data = s->buf + s->off[k];
        pkt_tbl[i].sz = s->len[k];
        pkt_tbl[i].ancillary = k;
      }
      if ((t->rc = pptk_rx_batch(ctx, pkt_tbl, num, recs)) != 0)
        break;
      for (int i = 0; i < num; i++)
        if (memcmp(&recs[i], &s->want[t->first + head + (uint32_t)i], sizeof(recs[i])) != 0)
          t->mismatches++;
      t->pkts += (unsigned long)num;
      /* ldp_in_deallocate_some(intf->inq[id], pkt_tbl, num); */
      head += (uint32_t)num;
    }
  }
  pptk_rx_ctx_destroy(ctx);
  return NULL;
}

int main(int argc, char **argv)
{
  struct rxq_set set;
  int nthr = argc > 2 ? atoi(argv[2]) : 4, laps = argc > 3 ? atoi(argv[3]) : 3;
  int ndev = pptk_rx_device_count();
  unsigned long pkts = 0, bad = 0;
  pthread_t pth[64];
  struct rxq_thread thr[64];
  double t0;
  int i, failed = 0;

  if (argc < 2 || rxq_load(argv[1], &set) != 0) {
    fprintf(stderr, "usage: rx_mt frames.rxq [threads [laps]]\n");
    return 1;
  }
  if (nthr < 1 || nthr > 64 || ndev < 1) {
    fprintf(stderr, "bad thread count %d or no GPU (%d)\n", nthr, ndev);
    return 1;
  }
  t0 = now();
  for (i = 0; i < nthr; i++) {
    thr[i] = (struct rxq_thread){.id = i, .device = i % ndev, .laps = laps, .set = &set};
    thr[i].first = (uint32_t)((uint64_t)set.h.n * (uint64_t)i / (uint64_t)nthr);
    thr[i].count = (uint32_t)((uint64_t)set.h.n * (uint64_t)(i + 1) / (uint64_t)nthr) - thr[i].first;
    pthread_create(&pth[i], NULL, thrfn, &thr[i]);
  }
  for (i = 0; i < nthr; i++) {
    pthread_join(pth[i], NULL);
    if (thr[i].rc != 0) {
      fprintf(stderr, "thread %d: error %d\n", i, thr[i].rc);
      failed = 1;
    }
    printf("thread %d (GPU %d): %lu frames, %lu mismatches\n", i, thr[i].device, thr[i].pkts,
           thr[i].mismatches);
    pkts += thr[i].pkts;
    bad += thr[i].mismatches;
  }
  printf("rx_mt: %d threads, %lu frames, %.3f MPPS, %lu mismatches\n", nthr, pkts,
         pkts / (now() - t0) / 1e6, bad);
  rxq_free(&set);
  return failed ? 1 : bad ? 2 : 0;
}
