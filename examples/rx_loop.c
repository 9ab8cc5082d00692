/*
 * rx_loop.c -- an LDP-style rx loop using the GPU batch transform.
 *
 * Mirrors the structure of the reference's ldp/ldprecv.c:32-71: a ring of
 * frames is handed out as struct ldp_packet batches (here by a synthetic
 * stand-in for ldp_in_nextpkts(), built with the reference's frame recipe
 * ldp/ldpsend.c:141-168), each batch goes through pptk_rx_batch() between
 * "nextpkts" and "deallocate_some", and the loop reports MPPS and the
 * checksum verdicts.  The ring is registered once for zero-copy reads.
 * With "pipe", DEPTH batches are in flight: batch k is fetched and
 * submitted (pptk_rx_batch_submit) before batch k-DEPTH+1 is completed and
 * released (pptk_rx_batch_complete, then deallocate_some), so the batches'
 * GPU round trips overlap the host work of the ones after them.
 *
 *   gcc -O2 -Iinclude examples/rx_loop.c -Lpptk_amd -lpptkrx -o rx_loop
 *   ./rx_loop [batches] [pipe]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "hashseed.h"
#include "ipcksum.h"
#include "iphdr.h"
#include "pptk_rx.h"

#define RING_SLOTS 4096
#define SLOT_BYTES 2048       /* netmap-style fixed buffers */
#define BATCH 1000            /* ldp/ldprecv.c:14 uses 1000 */
#define PAYLOAD 1458          /* 14 + 20 + 8 + 1458 = 1500-byte frames */
#define DEPTH 4               /* pipelined: batches in flight (<= PPTK_RX_MAX_INFLIGHT) */

static void put16(unsigned char *p, uint16_t v) { p[0] = (unsigned char)(v >> 8); p[1] = (unsigned char)v; }

/* Eth + IPv4 (DF, TTL 64) + UDP, checksums filled with the kept host API. */
static void construct_packet(unsigned char *f, uint32_t src, uint32_t dst, uint16_t sp,
                             uint16_t dp, unsigned seed)
{
  unsigned char *ip = f + 14, *udp = ip + 20;
  size_t i;
  memset(f, 0, 14 + 20 + 8);
  memset(f, 0x02, 12);
  put16(f + 12, ETHER_TYPE_IP);
  ip[0] = 0x45;
  put16(ip + 2, 20 + 8 + PAYLOAD);
  put16(ip + 6, 0x4000);
  ip[8] = 64;
  ip[9] = 17;
  hdr_set32n(ip + 12, src);
  hdr_set32n(ip + 16, dst);
  hdr_set16n(ip + 10, ip_hdr_cksum_calc(ip, 20));   /* field is 0 while summing */
  put16(udp, sp);
  put16(udp + 2, dp);
  put16(udp + 4, 8 + PAYLOAD);
  for (i = 0; i < PAYLOAD; i++)
    udp[8 + i] = (unsigned char)(seed * 131u + i * 7u);
  hdr_set16n(udp + 6, udp_cksum_calc(ip, 20, udp, 8 + PAYLOAD));
}

static unsigned long ok, bad;

static void tally(const struct pptk_rx_rec *recs, int num)
{
  int i;
  for (i = 0; i < num; i++) {
    if ((recs[i].flags & (PPTK_RX_F_IP_OK | PPTK_RX_F_L4_OK)) ==
        (PPTK_RX_F_IP_OK | PPTK_RX_F_L4_OK))
      ok++;
    else
      bad++;
  }
}

/* num = ldp_in_nextpkts(inq, pkt_tbl, BATCH): the next BATCH ring slots */
static void nextpkts(struct ldp_packet *pkt_tbl, unsigned char *ring, unsigned head)
{
  int i;
  for (i = 0; i < BATCH; i++) {
    unsigned slot = (head + (unsigned)i) % RING_SLOTS;
    pkt_tbl[i].data = ring + (size_t)slot * SLOT_BYTES;
    pkt_tbl[i].sz = 14 + 20 + 8 + PAYLOAD;
    pkt_tbl[i].ancillary = slot;                   /* netmap buf_idx stand-in */
  }
}

static double now(void)
{
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec + tv.tv_usec * 1e-6;
}

int main(int argc, char **argv)
{
  int batches = argc > 1 ? atoi(argv[1]) : 2000;
  int pipe = argc > 2 && strcmp(argv[2], "pipe") == 0;
  unsigned char *ring = aligned_alloc(4096, (size_t)RING_SLOTS * SLOT_BYTES);
  /* a packet table and record array per batch in flight (pipelined mode) */
  static struct ldp_packet pkt_tbl[DEPTH][BATCH];
  static struct pptk_rx_rec recs[DEPTH][BATCH];
  struct pptk_rx_opts o;
  struct pptk_rx_ctx *ctx;
  unsigned head = 0;
  unsigned long pkts = 0;
  double t0;
  int b, i, rc;

  for (i = 0; i < RING_SLOTS; i++)
    construct_packet(ring + (size_t)i * SLOT_BYTES, 0x0a000001u + (uint32_t)i, 0xc0a80001u,
                     (uint16_t)(1024 + i), 53, (unsigned)i);
  ring[(size_t)7 * SLOT_BYTES + 100] ^= 0xff;        /* one corrupted frame */

  hash_seed_init();
  pptk_rx_opts_default(&o);                          /* key = hash_seed */
  o.max_batch = BATCH;
  o.max_frame = 1518;
  if ((rc = pptk_rx_ctx_create(&ctx, &o)) != 0) {
    fprintf(stderr, "pptk_rx_ctx_create: %d\n", rc);
    return 1;
  }
  if ((rc = pptk_rx_register_ring(ctx, ring, (size_t)RING_SLOTS * SLOT_BYTES)) != 0)
    fprintf(stderr, "ring not registered (%d): staged copies instead\n", rc);
  /* the record array too: the records land in it directly, nothing is
     copied back per batch */
  if ((rc = pptk_rx_register_ring(ctx, recs, sizeof(recs))) != 0)
    fprintf(stderr, "record array not registered (%d): copied back instead\n", rc);

  t0 = now();
  for (b = 0; b < batches; b++) {
    const int k = pipe ? b % DEPTH : 0;
    nextpkts(pkt_tbl[k], ring, head);
    head = (head + BATCH) % RING_SLOTS;
    pkts += BATCH;
    if (!pipe) {
      if ((rc = pptk_rx_batch(ctx, pkt_tbl[0], BATCH, recs[0])) != 0) {
        fprintf(stderr, "pptk_rx_batch: %d\n", rc);
        return 1;
      }
      tally(recs[0], BATCH);
      /* ldp_in_deallocate_some(inq, pkt_tbl, num); */
      continue;
    }
    /* pipelined: batch b goes to the GPU, then batch b-DEPTH+1 comes back */
    if ((rc = pptk_rx_batch_submit(ctx, pkt_tbl[k], BATCH, recs[k])) != 0) {
      fprintf(stderr, "pptk_rx_batch_submit: %d\n", rc);
      return 1;
    }
    if (pptk_rx_batch_pending(ctx) == DEPTH) {
      if ((rc = pptk_rx_batch_complete(ctx)) != BATCH) {
        fprintf(stderr, "pptk_rx_batch_complete: %d\n", rc);
        return 1;
      }
      tally(recs[(b + 1) % DEPTH], BATCH);       /* batch b-DEPTH+1 */
      /* ldp_in_deallocate_some(inq, pkt_tbl[(b + 1) % DEPTH], num); */
    }
  }
  for (b -= pptk_rx_batch_pending(ctx); b < batches; b++) {   /* drain, oldest first */
    if ((rc = pptk_rx_batch_complete(ctx)) != BATCH) {
      fprintf(stderr, "pptk_rx_batch_complete: %d\n", rc);
      return 1;
    }
    tally(recs[b % DEPTH], BATCH);
  }
  printf("%lu frames, %.3f MPPS, %lu verified, %lu failed\n", pkts, pkts / (now() - t0) / 1e6,
         ok, bad);
  pptk_rx_unregister_ring(ctx, recs);
  pptk_rx_unregister_ring(ctx, ring);
  pptk_rx_ctx_destroy(ctx);
  free(ring);
  /* exactly the corrupted slot fails, once per lap of the ring */
  return bad == (pkts + RING_SLOTS - 1 - 7) / RING_SLOTS ? 0 : 2;
}
