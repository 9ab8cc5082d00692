/* Property fuzzer for the host half of the kept API, built by
 * tests/test_capi.py with -fsanitize=address,undefined straight from
 * the sources under pptk_amd/csrc/host/ (no GPU, no libpptkrx.so).  Every
 * packet lives in a heap block of exactly its own length, so a walk or an
 * update that touches a byte past the packet is an ASan report.
 *
 *   usage: host_fuzz SEED ITERS
 *
 * Properties:
 *  - ip_cksum_feed at any length and alignment equals a byte-at-a-time sum;
 *  - a TCP/IPv4 packet with random (often malformed) options: the option
 *    walks stay inside [20, data offset) and agree with each other, and every
 *    incremental update (addresses, ports, seq/ack/window, ACK off, MSS,
 *    SACK disable/adjust, timestamps, TTL) leaves the IPv4 header and TCP
 *    checksums verifying;
 *  - the timer heap keeps its invariants under random add/remove/modify and
 *    pops in time order;
 *  - an ip_hash of random geometry survives permits, refills and give-backs,
 *    and ip_hash_free releases everything (LeakSanitizer). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hashseed.h"
#include "ipcksum.h"
#include "iphash.h"
#include "iphdr.h"
#include "timerlink.h"

static uint64_t rs;
static uint32_t rnd(void)
{
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)(rs >> 11);
}
static uint32_t rnd_below(uint32_t n) { return n ? rnd() % n : 0; }

#define CHECK(c)                                                               \
  do {                                                                         \
    if (!(c)) {                                                                \
      fprintf(stderr, "host_fuzz: %s:%d: %s (iteration %lu)\n", __FILE__,     \
              __LINE__, #c, iter);                                             \
      exit(2);                                                                 \
    }                                                                          \
  } while (0)

static unsigned long iter;
static unsigned long n_mss, n_ts, n_sack, n_disable, n_invalid;

/* ---- checksum feed vs a byte-wise RFC 1071 sum of big-endian 16-bit words */
static uint16_t naive_cksum(const unsigned char *p, size_t n)
{
  uint64_t s = 0;
  size_t i;
  for (i = 0; i + 1 < n; i += 2)
    s += ((uint32_t)p[i] << 8) | p[i + 1];
  if (n & 1)
    s += (uint32_t)p[n - 1] << 8;
  while (s >> 16)
    s = (s & 0xffff) + (s >> 16);
  return (uint16_t)~s;
}

static void fuzz_feed(void)
{
  const size_t n = rnd_below(4) == 0 ? rnd_below(9000) : rnd_below(80);
  const size_t skew = rnd_below(8);
  unsigned char *blk = malloc(n + skew + 1), *p = blk + skew;
  struct ip_cksum_ctx c = IP_CKSUM_CTX_INITER;
  size_t i, cut;
  for (i = 0; i < n; i++)
    p[i] = (unsigned char)(rnd_below(5) == 0 ? 0xff : rnd());
  /* two feeds split at an even offset sum the same as one */
  cut = n ? (rnd_below((uint32_t)n + 1) & ~(size_t)1) : 0;
  ip_cksum_feed(&c, p, cut);
  ip_cksum_feed(&c, p + cut, n - cut);
  {
    const uint16_t a = ip_cksum_postprocess(&c), b = naive_cksum(p, n);
    /* 0x0000 and 0xffff are the same one's-complement value */
    CHECK(a == b || (a == 0 && b == 0xffff) || (a == 0xffff && b == 0));
  }
  free(blk);
}

/* ---- TCP options */
static size_t put_option(unsigned char *o, size_t room)
{
  const uint32_t pick = rnd_below(14);
  size_t len, i;
  unsigned kind;
  switch (pick) {
  case 0: kind = 0; len = 1; break;
  case 1: case 2: kind = 1; len = 1; break;
  case 3: kind = 2; len = 4; break;
  case 4: kind = 3; len = 3; break;
  case 5: kind = 4; len = 2; break;
  case 6: case 7: kind = 5; len = 2 + 8 * rnd_below(5); break;
  case 8: case 9: kind = 8; len = 10; break;
  case 10: kind = rnd_below(256); len = 2 + rnd_below(12); break;
  default: kind = rnd_below(10); len = rnd_below(5); break;   /* malformed */
  }
  if (room == 0)
    return 0;
  o[0] = (unsigned char)kind;
  if (kind <= 1)
    return 1;
  if (room >= 2)
    o[1] = (unsigned char)(rnd_below(6) == 0 ? rnd() : len);
  for (i = 2; i < len && i < room; i++)
    o[i] = (unsigned char)rnd();
  return len < room ? (len ? len : 1) : room;
}

static void ip_tcp_verify(unsigned char *ip, size_t tcplen)
{
  CHECK(ip_hdr_cksum_calc(ip, 20) == 0);
  CHECK(tcp_cksum_calc(ip, 20, ip + 20, (uint16_t)tcplen) == 0);
}

static void fuzz_tcp(void)
{
  const size_t doff = 20 + 4 * rnd_below(11);
  const size_t paylen = rnd_below(2) ? 0 : rnd_below(40);
  const size_t tcplen = doff + paylen, n = 20 + tcplen;
  unsigned char *ip = malloc(n), *t = ip + 20;
  struct tcp_information info;
  struct sack_ts_headers hdrs;
  size_t off, i, sacklen = 0;
  int align = 0;
  void *sack;

  for (i = 0; i < n; i++)
    ip[i] = (unsigned char)rnd();
  ip[0] = 0x45;
  hdr_set16n(ip + 2, (uint16_t)n);
  ip[8] = (unsigned char)(1 + rnd_below(255));   /* TTL > 0 */
  ip[9] = 6;
  t[12] = (unsigned char)((doff / 4) << 4 | (t[12] & 0x0f));
  for (off = 20; off < doff;)
    off += put_option(t + off, doff - off);
  ip_set_hdr_cksum_calc(ip, 20);
  tcp_set_cksum_calc(ip, 20, t, (uint16_t)tcplen);
  ip_tcp_verify(ip, tcplen);

  tcp_parse_options(t, &info);
  tcp_find_sack_ts_headers(t, &hdrs);
  sack = tcp_find_sack_header(t, &sacklen, &align);
  if (info.mssoff)
    CHECK(info.mssoff >= 20 && info.mssoff + 4u <= doff && t[info.mssoff] == 2);
  if (hdrs.tsoff)
    CHECK(hdrs.tsoff >= 20 && hdrs.tsoff + 10u <= doff && t[hdrs.tsoff] == 8);
  if (hdrs.sackoff)
    CHECK(hdrs.sackoff >= 20 && hdrs.sackoff + (size_t)hdrs.sacklen <= doff &&
          t[hdrs.sackoff] == 5);
  if (sack) {
    const size_t so = (size_t)((unsigned char *)sack - t);
    CHECK(so >= 20 && so + sacklen <= doff && t[so] == 5);
    CHECK(align == !(so % 2));
  }

  /* every update keeps both checksums verifying */
  ip_set_src_cksum_update(ip, 20, 6, t, (uint16_t)tcplen, rnd());
  ip_tcp_verify(ip, tcplen);
  ip_set_dst_cksum_update(ip, 20, 6, t, (uint16_t)tcplen, rnd());
  ip_tcp_verify(ip, tcplen);
  tcp_set_src_port_cksum_update(t, (uint16_t)tcplen, (uint16_t)rnd());
  tcp_set_dst_port_cksum_update(t, (uint16_t)tcplen, (uint16_t)rnd());
  ip_tcp_verify(ip, tcplen);
  tcp_set_seq_number_cksum_update(t, (uint16_t)tcplen, rnd());
  tcp_set_ack_number_cksum_update(t, (uint16_t)tcplen, rnd());
  tcp_set_window_cksum_update(t, (uint16_t)tcplen, (uint16_t)rnd());
  ip_tcp_verify(ip, tcplen);
  tcp_set_ack_off_cksum_update(t);
  CHECK(!(t[13] & 0x10));
  ip_tcp_verify(ip, tcplen);
  if (info.options_valid && info.mssoff) {
    const uint16_t mss = (uint16_t)rnd();
    tcp_set_mss_cksum_update(t, &info, mss);
    n_mss++;
    CHECK(hdr_get16n(t + info.mssoff + 2) == mss);
    ip_tcp_verify(ip, tcplen);
  }
  n_ts += hdrs.tsoff != 0;
  n_invalid += !info.options_valid;
  tcp_adjust_tsval_cksum_update(t, &hdrs, rnd());
  tcp_adjust_tsecho_cksum_update(t, &hdrs, rnd());
  ip_tcp_verify(ip, tcplen);
  if (rnd_below(2)) {
    tcp_adjust_sack_cksum_update_2(t, &hdrs, rnd());
    n_sack += hdrs.sackoff != 0;
    ip_tcp_verify(ip, tcplen);
  }
  /* the disable form reads up to two bytes past the option (the word
   * straddling its end; ipcksum.h:425-458 reads the same bytes): keep it to
   * options with two bytes of packet after them */
  if (sack && (size_t)((unsigned char *)sack - t) + sacklen + 2 <= tcplen) {
    tcp_disable_sack_cksum_update(t, sack, sacklen, align);
    n_disable++;
    for (i = 0; i + 1 < sacklen; i++)
      CHECK(((unsigned char *)sack)[i] == 1);
    ip_tcp_verify(ip, tcplen);
  }
  while (ip[8] > 0) {
    const int alive = ip_decr_ttl_cksum_update(ip);
    CHECK(alive == (ip[8] > 0));
    CHECK(ip_hdr_cksum_calc(ip, 20) == 0);
  }
  free(ip);
}

/* ---- timer heap */
static void fuzz_timers(void)
{
  enum { NT = 97 };
  struct timer_link tl[NT];
  int in[NT] = {0};
  struct timer_linkheap heap;
  size_t size = 0;
  uint64_t last = 0;
  int k, op;
  memset(tl, 0, sizeof(tl));
  timer_linkheap_init(&heap);
  for (op = 0; op < 600; op++) {
    const int i = (int)rnd_below(NT);
    const uint64_t when = rnd_below(4) ? rnd_below(1000) : rnd_below(5);
    if (!in[i]) {
      tl[i].time64 = when;
      timer_linkheap_add(&heap, &tl[i]);
      in[i] = 1;
      size++;
    } else if (rnd_below(2)) {
      timer_linkheap_remove(&heap, &tl[i]);
      in[i] = 0;
      size--;
    } else {
      tl[i].time64 = when;
      timer_linkheap_modify(&heap, &tl[i]);
    }
    CHECK(heap.size == size);
    if (op % 16 == 0)
      CHECK(timer_linkheap_verify(&heap));
  }
  CHECK(timer_linkheap_verify(&heap));
  for (k = 0; heap.root; k++) {
    struct timer_link *t = timer_linkheap_next_expiry_timer(&heap);
    CHECK(t->time64 >= last && t->time64 == timer_linkheap_next_expiry_time(&heap));
    last = t->time64;
    timer_linkheap_remove(&heap, t);
  }
  CHECK((size_t)k == size && heap.size == 0);
  timer_linkheap_free(&heap);
}

/* ---- rate limiter */
static void fuzz_iphash(void)
{
  static const uint32_t initial[] = {1, 7, 255, 256, 4000, 65535, 65536, 1000000};
  struct timer_linkheap heap;
  struct ip_hash h;
  const uint32_t hash_size = 1u << (1 + rnd_below(10));
  const uint32_t batch_size = hash_size >> rnd_below(3);
  const uint8_t bits4 = (uint8_t)(1 + rnd_below(32)), bits6 = (uint8_t)(1 + rnd_below(128));
  uint64_t clock = 0;
  int i;
  timer_linkheap_init(&heap);
  memset(&h, 0, sizeof(h));
  h.hash_size = hash_size;
  h.batch_size = batch_size ? batch_size : 1;
  h.initial_tokens = initial[rnd_below(8)];
  h.timer_add = rnd_below(h.initial_tokens + 2);
  h.timer_period = 1 + rnd_below(1000);
  ip_hash_init(&h, &heap, NULL);
  CHECK(heap.size == hash_size / h.batch_size);
  /* ip_hash_init arms the timers on the wall clock; re-time them to 0 */
  for (i = 0; i < (int)heap.size; i++) {
    h.timers[i].time64 = (uint64_t)h.timer_period * (uint32_t)i / heap.size;
    timer_linkheap_modify(&heap, &h.timers[i]);
  }
  for (i = 0; i < 2000; i++) {
    unsigned char v6[16];
    int k;
    const uint32_t v4 = rnd_below(64) << 24 | rnd_below(3);
    for (k = 0; k < 16; k++)
      v6[k] = (unsigned char)(k < 2 ? rnd_below(4) : rnd());
    (void)ip_permitted(v4, bits4, &h);
    (void)ipv6_permitted(v6, bits6, &h);
    if (i % 5 == 0) {
      ip_increment_one(v4, bits4, &h);
      ipv6_increment_one(v6, bits6, &h);
    }
    if (i % 100 == 99) {
      clock += h.timer_period;
      /* every timer re-arms itself later, so this loop ends */
      while (timer_linkheap_next_expiry_time(&heap) <= clock) {
        struct timer_link *t = timer_linkheap_next_expiry_timer(&heap);
        timer_linkheap_remove(&heap, t);   /* as the timer loop does */
        t->fn(t, &heap, t->userdata, NULL);
      }
      CHECK(timer_linkheap_verify(&heap));
    }
  }
  ip_hash_free(&h, &heap);
  CHECK(heap.size == 0);
  timer_linkheap_free(&heap);
}

int main(int argc, char **argv)
{
  const unsigned long iters = argc > 2 ? strtoul(argv[2], NULL, 10) : 1000;
  rs = (argc > 1 ? strtoull(argv[1], NULL, 10) : 1) * 0x9e3779b97f4a7c15ull | 1;
  memset(hash_seed, 0x5a, sizeof(hash_seed));
  hash_seed_inited = 1;
  for (iter = 0; iter < iters; iter++) {
    fuzz_feed();
    fuzz_tcp();
    if (iter % 10 == 0)
      fuzz_timers();
    if (iter % 50 == 0)
      fuzz_iphash();
  }
  printf("host_fuzz ok: %lu iterations (mss %lu, ts %lu, sack adjust %lu, sack disable %lu, "
         "malformed %lu)\n", iters, n_mss, n_ts, n_sack, n_disable, n_invalid);
  return 0;
}
