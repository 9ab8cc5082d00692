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
 * every lap.  With "pipe", each thread keeps two bursts in flight
 * (pptk_rx_batch_submit, then pptk_rx_batch_complete of the previous burst
 * before its deallocate_some).  With "rec32" / "pipe32" the same with the
 * 32-byte compact records (pptk_rx_batch32 / pptk_rx_batch_submit32),
 * compared with the compact form of the expected records.
 *
 *   gcc -O2 -pthread -Iinclude examples/rx_mt.c -Lpptk_amd -lpptkrx -o rx_mt
 *   ./rx_mt frames.rxq [threads [laps [pipe|rec32|pipe32]]]
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
  int id, device, laps, pipe, rec32;
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

/* The compact record of a full one (include/pptk_rx.h: the same values, the
 * IPv6 addresses left out). */
static void to_rec32(const struct pptk_rx_rec *r, struct pptk_rx_rec32 *o)
{
  memset(o, 0, sizeof(*o));
  o->flow_hash = r->flow_hash;
  if (!(r->flags & PPTK_RX_F_IPV6)) {
    memcpy(&o->src4, r->src, 4);
    memcpy(&o->dst4, r->dst, 4);
  }
  o->sport = r->sport;
  o->dport = r->dport;
  o->flags = r->flags;
  o->proto = r->proto;
  o->l3_off = r->l3_off;
  o->l4_off = r->l4_off;
  o->l4_len = r->l4_len;
  o->src_bucket = r->src_bucket;
}

/* records of the burst starting at queue position `head` against the set
 * (recs: struct pptk_rx_rec[], or struct pptk_rx_rec32[] with rec32) */
static void check(struct rxq_thread *t, const void *recs, uint32_t head, int num)
{
  for (int i = 0; i < num; i++) {
    const struct pptk_rx_rec *w = &t->set->want[t->first + head + (uint32_t)i];
    if (t->rec32) {
      struct pptk_rx_rec32 w32;
      to_rec32(w, &w32);
      if (memcmp((const struct pptk_rx_rec32 *)recs + i, &w32, sizeof(w32)) != 0)
        t->mismatches++;
    } else if (memcmp((const struct pptk_rx_rec *)recs + i, w, sizeof(*w)) != 0) {
      t->mismatches++;
    }
  }
  t->pkts += (unsigned long)num;
}

static void *thrfn(void *arg)
{
  struct rxq_thread *t = arg;
  const struct rxq_set *s = t->set;
  /* two bursts: one in hand while the other is with the GPU (pipe) */
  static __thread struct ldp_packet pkt_tbl[2][BURST];
  static __thread struct pptk_rx_rec recs[2][BURST];
  uint32_t burst_head[2] = {0, 0};
  int burst_num[2] = {0, 0};
  struct pptk_rx_opts o;
  struct pptk_rx_ctx *ctx;
  pptk_rx_opts_default(&o);
  o.device = t->device;
  memcpy(o.key, s->h.key, 16);
  o.iphash_bits4 = 24;           /* the golden sets' ip_hash parameters */
  o.iphash_bits6 = 48;
  o.iphash_size = 4096;
  o.max_batch = t->pipe ? BURST : 256;   /* a submission is one chunk */
  o.max_frame = 65535;
  if ((t->rc = pptk_rx_ctx_create(&ctx, &o)) != 0)
    return NULL;
  int b = 0;   /* which of the two bursts is in hand */
  for (int lap = 0; lap < t->laps && t->rc == 0; lap++) {
    uint32_t head = 0;
    while (head < t->count) {
      /* num = ldp_in_nextpkts(intf->inq[id], pkt_tbl, BURST); */
      int num = t->count - head < BURST ? (int)(t->count - head) : BURST;
      for (int i = 0; i < num; i++) {
        uint32_t k = t->first + head + (uint32_t)i;
        pkt_tbl[b][i].data = s->buf + s->off[k];
        pkt_tbl[b][i].sz = s->len[k];
        pkt_tbl[b][i].ancillary = k;
      }
      if (!t->pipe) {
        t->rc = t->rec32 ? pptk_rx_batch32(ctx, pkt_tbl[b], num, (struct pptk_rx_rec32 *)recs[b])
                         : pptk_rx_batch(ctx, pkt_tbl[b], num, recs[b]);
        if (t->rc != 0)
          break;
        check(t, recs[b], head, num);
        /* ldp_in_deallocate_some(intf->inq[id], pkt_tbl, num); */
      } else {
        t->rc = t->rec32 ? pptk_rx_batch_submit32(ctx, pkt_tbl[b], num,
                                                  (struct pptk_rx_rec32 *)recs[b])
                         : pptk_rx_batch_submit(ctx, pkt_tbl[b], num, recs[b]);
        if (t->rc != 0)
          break;
        burst_head[b] = head;
        burst_num[b] = num;
        if (pptk_rx_batch_pending(ctx) == 2) {        /* two bursts in flight */
          int rc = pptk_rx_batch_complete(ctx);           /* the other burst */
          if (rc != burst_num[b ^ 1]) {
            t->rc = rc < 0 ? rc : -1;
            break;
          }
          check(t, recs[b ^ 1], burst_head[b ^ 1], burst_num[b ^ 1]);
          /* ldp_in_deallocate_some(intf->inq[id], pkt_tbl[b ^ 1], num); */
        }
        b ^= 1;
      }
      head += (uint32_t)num;
    }
  }
  while (t->rc == 0 && pptk_rx_batch_pending(ctx) > 0) {   /* the last burst */
    int rc = pptk_rx_batch_complete(ctx);
    if (rc != burst_num[b ^ 1]) {
      t->rc = rc < 0 ? rc : -1;
      break;
    }
    check(t, recs[b ^ 1], burst_head[b ^ 1], burst_num[b ^ 1]);
    b ^= 1;
  }
  pptk_rx_ctx_destroy(ctx);
  return NULL;
}

int main(int argc, char **argv)
{
  struct rxq_set set;
  int nthr = argc > 2 ? atoi(argv[2]) : 4, laps = argc > 3 ? atoi(argv[3]) : 3;
  const char *mode = argc > 4 ? argv[4] : "";
  int pipe = !strcmp(mode, "pipe") || !strcmp(mode, "pipe32");
  int rec32 = !strcmp(mode, "rec32") || !strcmp(mode, "pipe32");
  int ndev = pptk_rx_device_count();
  unsigned long pkts = 0, bad = 0;
  pthread_t pth[64];
  struct rxq_thread thr[64];
  double t0;
  int i, failed = 0;

  if (argc < 2 || rxq_load(argv[1], &set) != 0) {
    fprintf(stderr, "usage: rx_mt frames.rxq [threads [laps [pipe|rec32|pipe32]]]\n");
    return 1;
  }
  if (nthr < 1 || nthr > 64 || ndev < 1) {
    fprintf(stderr, "bad thread count %d or no GPU (%d)\n", nthr, ndev);
    return 1;
  }
  t0 = now();
  for (i = 0; i < nthr; i++) {
    thr[i] = (struct rxq_thread){.id = i, .device = i % ndev, .laps = laps, .pipe = pipe,
                                  .rec32 = rec32, .set = &set};
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
  printf("rx_mt: %d threads%s%s, %lu frames, %.3f MPPS, %lu mismatches\n", nthr,
         pipe ? " (pipelined)" : "", rec32 ? " (32-byte records)" : "", pkts,
         pkts / (now() - t0) / 1e6, bad);
  rxq_free(&set);
  return failed ? 1 : bad ? 2 : 0;
}
