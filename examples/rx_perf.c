/*
 * rx_perf.c -- device-resident throughput of the receive transform, timed
 * from a plain C host: the GPU counterpart of the reference's ipcksumperf
 * (iphdr/ipcksumperf.c:21-32, one 1500-byte buffer through ip_cksum_feed a
 * million times on one core).  Here `frames` frames of `bytes` bytes each
 * (IPv4/TCP, or IPv4/UDP below 54 bytes) sit in HBM at a fixed stride and
 * every launch verifies both checksums, parses the headers and hashes the
 * 5-tuple of all of them into 64-byte records (pptk_rx_batch_device).
 *
 * The frames are 4 096 distinct ones built with the kept PPTK C APIs
 * (ip_set_hdr_cksum_calc, tcp/udp_set_cksum_calc of ipcksum.h), repeated
 * over the batch.  After timing, the first 4 096 records are checked against
 * the same frames through the kept per-packet APIs on the host
 * (ip_hdr_cksum_calc, tcp/udp_cksum_calc, the iphdr.h getters and
 * siphash_buf over the record's 40-byte tuple), and the last 4 096 records
 * against the first.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude examples/rx_perf.c \
 *       -Lpptk_amd -lpptkrx -L/opt/rocm/lib -lamdhip64 -o rx_perf
 *   ./rx_perf [frames [bytes [reps [device]]]]     (16777216 1500 20 0)
 *
 * The device rings come from the library (pptk_rx_ring_alloc: placed by a
 * probe at allocation, the product default);
 * RX_PERF_RING=0 uses plain hipMalloc buffers instead.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "ipcksum.h"
#include "iphdr.h"
#include "pptk_rx.h"
#include "siphash.h"

#define POOL 4096u

static uint64_t rng = 0x5eed1500u;

static uint32_t next32(void)
{
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}

static void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* Eth + IPv4 (IHL 5, DF, TTL 64) + TCP (doff 5) or UDP, random addresses,
 * ports and payload, valid checksums (ldp/ldpsend.c:141-168 is the
 * reference's own recipe for a valid frame). */
static void make_frame(uint8_t *f, uint32_t bytes)
{
  const int udp = bytes < 54;
  uint8_t *ip = f + 14, *l4 = ip + 20;
  const uint16_t tl = (uint16_t)(bytes - 14);
  uint32_t i;
  memset(f, 0, bytes);
  for (i = 0; i < 12; i++) f[i] = (uint8_t)next32();
  put16(f + 12, 0x0800);
  ip[0] = 0x45;
  put16(ip + 2, tl);
  put16(ip + 4, (uint16_t)next32());
  put16(ip + 6, 0x4000);
  ip[8] = 64;
  ip[9] = udp ? 17 : 6;
  for (i = 12; i < 20; i++) ip[i] = (uint8_t)next32();
  for (i = 0; i < (uint32_t)tl - 20; i++) l4[i] = (uint8_t)next32();
  if (udp) {
    put16(l4 + 4, (uint16_t)(tl - 20));
    udp_set_cksum_calc(ip, 20, l4, (uint16_t)(tl - 20));
  } else {
    l4[12] = 0x50;
    tcp_set_cksum_calc(ip, 20, l4, (uint16_t)(tl - 20));
  }
  ip_set_hdr_cksum_calc(ip, 20);
}

/* The record of a pool frame through the kept per-packet APIs (DESIGN.md
 * "Record semantics" steps 3, 7, 8 for an untagged IPv4 frame). */
static int check_record(const uint8_t *f, uint32_t bytes, const struct pptk_rx_rec *r,
                        const uint8_t key[16])
{
  const uint8_t *ip = f + 14, *l4 = ip + 20;
  const uint16_t tl = (uint16_t)(bytes - 14);
  const uint8_t proto = ip[9];
  const uint16_t want_flags = PPTK_RX_F_PARSED | PPTK_RX_F_IP_OK | PPTK_RX_F_L4 | PPTK_RX_F_L4_OK;
  uint8_t t[40] = {0};
  if ((r->flags & want_flags) != want_flags || (r->flags & PPTK_RX_F_MALFORMED)) return 1;
  if (ip_hdr_cksum_calc(ip, 20) != 0 || r->ip_cksum != 0) return 1;
  if ((proto == 6 ? tcp_cksum_calc(ip, 20, l4, (uint16_t)(tl - 20))
                  : udp_cksum_calc(ip, 20, l4, (uint16_t)(tl - 20))) != r->l4_cksum)
    return 1;
  if (r->proto != proto || r->sport != tcp_src_port(l4) || r->dport != tcp_dst_port(l4))
    return 1;
  memcpy(t, ip + 12, 4);       /* src, then dst, 16 bytes each (v4 in the first 4) */
  memcpy(t + 16, ip + 16, 4);
  memcpy(t + 32, l4, 4);       /* be16 sport, be16 dport */
  t[36] = proto;
  return siphash_buf(key, t, sizeof(t)) != r->flow_hash;
}

static int cmp_float(const void *a, const void *b)
{
  const float x = *(const float *)a, y = *(const float *)b;
  return (x > y) - (x < y);
}

int main(int argc, char **argv)
{
  const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 0) : 16777216u;
  const uint32_t bytes = argc > 2 ? (uint32_t)atoi(argv[2]) : 1500u;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const int device = argc > 4 ? atoi(argv[4]) : 0;
  const uint8_t key[16] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  uint8_t *pool, *d_frames = NULL;
  struct pptk_rx_rec *d_recs = NULL, *recs;
  struct pptk_rx_opts o;
  struct pptk_rx_ctx *ctx;
  struct pptk_rx_dev_batch b;
  hipEvent_t e0, e1;
  float *ms;
  uint64_t have, i, bad = 0;
  int rc, k;
  if (n < 2 * POOL || bytes < 42 || bytes > 9000 || reps < 1) {
    fprintf(stderr, "usage: rx_perf [frames >= %u [bytes 42..9000 [reps [device]]]]\n",
            2 * POOL);
    return 2;
  }
  const char *ring_env = getenv("RX_PERF_RING");
  const int use_ring = !(ring_env && ring_env[0] == '0');
  struct pptk_rx_ring ring;
  memset(&ring, 0, sizeof(ring));
  pool = malloc((size_t)POOL * bytes);
  recs = malloc(2 * (size_t)POOL * sizeof(*recs));
  ms = malloc(sizeof(float) * (size_t)reps);
  if (!pool || !recs || !ms) return 1;
  for (i = 0; i < POOL; i++) make_frame(pool + i * bytes, bytes);
  pptk_rx_opts_default(&o);
  o.device = device;
  memcpy(o.key, key, 16);
  if (hipSetDevice(device) != hipSuccess || (rc = pptk_rx_ctx_create(&ctx, &o)) != 0) {
    fprintf(stderr, "pptk_rx_ctx_create: %d\n", rc);
    return 1;
  }
  if (use_ring) {   /* the library's placed rings (the product default) */
    struct pptk_rx_ring_spec spec;
    memset(&spec, 0, sizeof(spec));
    spec.frame_bytes = n * bytes;
    spec.nrec = n;
    spec.rec_bytes = sizeof(struct pptk_rx_rec);
    spec.probe_len = bytes < 64 ? 64 : bytes > 1536 ? 1536 : bytes;
    spec.flags = PPTK_RX_RING_SETTLE;
    if ((rc = pptk_rx_ring_alloc(ctx, &spec, &ring, NULL)) != 0) {
      fprintf(stderr, "pptk_rx_ring_alloc: %d\n", rc);
      return 1;
    }
    d_frames = ring.d_frames;
    d_recs = (struct pptk_rx_rec *)ring.d_recs;
  } else if (hipMalloc((void **)&d_frames, n * bytes + 64) != hipSuccess ||
             hipMalloc((void **)&d_recs, n * sizeof(*d_recs)) != hipSuccess) {
    fprintf(stderr, "device %d: allocation of %.1f GB failed\n", device, n * (bytes + 64.0) / 1e9);
    return 1;
  }
  /* the pool, then doubling copies on the device */
  if (hipMemcpy(d_frames, pool, (size_t)POOL * bytes, hipMemcpyHostToDevice) != hipSuccess)
    return 1;
  for (have = POOL; have < n; have *= 2) {
    const uint64_t m = have < n - have ? have : n - have;
    if (hipMemcpy(d_frames + have * bytes, d_frames, m * bytes, hipMemcpyDeviceToDevice) !=
        hipSuccess)
      return 1;
  }
  memset(&b, 0, sizeof(b));
  b.d_frames = d_frames;
  b.stride = bytes;
  b.fixed_len = bytes;
  b.n = n;
  b.d_recs = d_recs;
  /* this GPU's fastest interchangeable kernel shape (results identical) */
  if ((rc = pptk_rx_autotune(ctx, &b, 5, NULL)) != 0 ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    fprintf(stderr, "setup: %d\n", rc);
    return 1;
  }
  for (k = -3; k < reps; k++) {     /* three untimed warm-ups */
    float t = 0.f;
    if (hipEventRecord(e0, NULL) != hipSuccess || (rc = pptk_rx_batch_device(ctx, &b, NULL)) ||
        hipEventRecord(e1, NULL) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&t, e0, e1) != hipSuccess) {
      fprintf(stderr, "batch: %d\n", rc);
      return 1;
    }
    if (k >= 0) ms[k] = t;
  }
  qsort(ms, (size_t)reps, sizeof(float), cmp_float);
  if (hipMemcpy(recs, d_recs, POOL * sizeof(*recs), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(recs + POOL, d_recs + (n / POOL - 1) * POOL, POOL * sizeof(*recs),
                hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  for (i = 0; i < POOL; i++) {
    bad += (uint64_t)check_record(pool + i * bytes, bytes, &recs[i], key);
    bad += memcmp(&recs[i], &recs[POOL + i], sizeof(*recs)) != 0;
  }
  {
    const double med = ms[reps / 2];
    const double gbs = (double)n * bytes / (med * 1e-3) / 1e9;
    printf("rx_perf: %llu frames x %u B, %s, kernel variant %d: median %.4f ms (min %.4f) = "
           "%.1f Mpkt/s, %.1f GB/s of frames = %.3f of the 8 TB/s HBM peak; "
           "%u records checked against the host APIs, %llu mismatches\n",
           (unsigned long long)n, bytes, bytes < 54 ? "IPv4/UDP" : "IPv4/TCP",
           pptk_rx_last_variant(ctx), med, ms[0], n / (med * 1e-3) / 1e6, gbs, gbs / 8000.0,
           2 * POOL, (unsigned long long)bad);
    if (use_ring)
      printf("rx_perf: rings from pptk_rx_ring_alloc: %u x %u candidate pairs probed, plain "
             "allocation %.4f ms, kept pair %.4f ms, %.1f GB freed, %u ms settled\n",
             ring.frame_cands, ring.rec_cands, ring.first_ms, ring.chosen_ms,
             ring.freed_bytes / 1e9, ring.settle_ms);
    else
      printf("rx_perf: plain hipMalloc buffers (RX_PERF_RING=0)\n");
  }
  pptk_rx_ctx_destroy(ctx);
  if (use_ring) {
    pptk_rx_ring_free(&ring);
  } else {
    (void)hipFree(d_frames);
    (void)hipFree(d_recs);
  }
  free(pool);
  free(recs);
  free(ms);
  return bad ? 3 : 0;
}
