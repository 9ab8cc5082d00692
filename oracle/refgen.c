/*
 * refgen.c -- TEST INFRASTRUCTURE ONLY.  Applies the record composition of
 * DESIGN.md ("Record semantics") using the REFERENCE's own functions,
 * compiled unmodified from /root/reference by oracle/Makefile into
 * oracle/_ref/libpptkref.so.  Used (a) in this container to generate the
 * golden fixtures under tests/golden/ and to cross-check the C restatement
 * (rx_oracle.c), and (b) on the GPU box as the "reference" CPU baseline.
 *
 * Nothing from the reference is copied here: this file only #includes the
 * reference headers in place (-I/root/reference/...) and calls:
 *   ether_type, ip_version, ip_hdr_len, ip_total_len, ip_proto,
 *   ip_frag_off, ip_more_frags, ip_dont_frag, ip_id, ip_src, ip_dst, ip_const_payload,
 *   ipv6_payload_len, ipv6_nexthdr, is_ipv6_nexthdr, ipv6_const_src/dst,
 *   ipv6_const_proto_hdr_2, ipv6_frag_off, ipv6_more_frags, tcp/udp_src_port, tcp/udp_dst_port, udp_cksum
 *                                                  (iphdr/iphdr.h)
 *   ip_hdr_cksum_calc, tcp_cksum_calc, udp_cksum_calc, tcp6_cksum_calc,
 *   udp6_cksum_calc, ip_cksum_feed, ip_cksum_postprocess  (iphdr/ipcksum.*)
 *   siphash_buf, siphash64                         (misc/siphash.h)
 *   ip_permitted, ipv6_permitted                   (iphash/iphash.c)
 *   ip_update_cksum16/32, ip_decr_ttl_cksum_update, ip_set_src/dst_cksum_update,
 *   tcp/udp_set_src/dst_port_cksum_update, ip_ttl   (iphdr/ipcksum.h, iphdr.h)
 *   tcp_parse_options, tcp_find_sack_ts_headers, tcp_find_sack_header,
 *   tcp_syn, tcp_data_offset                       (iphdr/iphdr.c, iphdr.h)
 *   tcp_set_mss_cksum_update, tcp_disable_sack_cksum_update,
 *   tcp_adjust_sack_cksum_update_2, tcp_adjust_tsval/tsecho_cksum_update,
 *   tcp_set_ack_off_cksum_update, tcp_set_seq/ack_number_cksum_update,
 *   tcp_set_window_cksum_update                    (iphdr/ipcksum.h)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hashseed.h"
#include "ipcksum.h"
#include "iphash.h"
#include "iphdr.h"
#include "siphash.h"

#include "../include/pptk_rx.h"

struct ref_opts {
  uint8_t key[16];
  uint8_t bits4;
  uint8_t bits6;
  uint16_t pad;
  uint32_t hash_size;
};

/* ---- thin exported wrappers over single reference primitives ---------- */
uint16_t ref_cksum_buf(const void *buf, size_t sz)
{
  struct ip_cksum_ctx ctx = IP_CKSUM_CTX_INITER;
  ip_cksum_feed(&ctx, buf, sz);
  return ip_cksum_postprocess(&ctx);
}

uint16_t ref_ip_hdr_cksum_calc(const void *ip, uint16_t iplen)
{
  return ip_hdr_cksum_calc(ip, iplen);
}
uint16_t ref_tcp_cksum_calc(const void *ip, uint16_t iplen, const void *l4, uint16_t l4len)
{
  return tcp_cksum_calc(ip, iplen, l4, l4len);
}
uint16_t ref_udp_cksum_calc(const void *ip, uint16_t iplen, const void *l4, uint16_t l4len)
{
  return udp_cksum_calc(ip, iplen, l4, l4len);
}
uint16_t ref_tcp6_cksum_calc(const void *ip, uint16_t iplen, const void *l4, uint16_t l4len)
{
  return tcp6_cksum_calc(ip, iplen, l4, l4len);
}
uint16_t ref_udp6_cksum_calc(const void *ip, uint16_t iplen, const void *l4, uint16_t l4len)
{
  return udp6_cksum_calc(ip, iplen, l4, l4len);
}

uint64_t ref_siphash_buf(const void *key, const void *buf, size_t len)
{
  return siphash_buf(key, buf, len);
}

uint64_t ref_siphash64(const void *key, uint64_t v)
{
  return siphash64(key, v);
}

/* ipv6_const_proto_hdr_2 -> offset of the returned pointer, or -1 (NULL). */
int ref_ipv6_proto_hdr(const void *ip6, uint8_t *proto, int *frag,
                       uint16_t *frag_hdr_off)
{
  uint16_t fo = 0, pfo = 0;
  const char *p = ipv6_const_proto_hdr_2(ip6, proto, frag, &fo, &pfo);
  if (p == NULL)
    return -1;
  if (frag_hdr_off)
    *frag_hdr_off = fo;
  return (int)(p - (const char *)ip6);
}

/* ---- ip_permitted / ipv6_permitted used as black boxes: every bucket
 * starts with one token, the call consumes one, and the bucket whose token
 * went to zero is the reference's hash value (iphash/iphash.c:162, :120). */
static uint32_t bucket_probe(int v6, const void *src6, uint32_t src4,
                             uint8_t bits, uint32_t hash_size)
{
  struct ip_hash h;
  uint32_t i, found = 0xffffffffu;
  memset(&h, 0, sizeof(h));
  h.hash_size = hash_size;
  h.initial_tokens = 1; /* use_tiny() */
  h.u.entries_tiny = malloc(hash_size * sizeof(*h.u.entries_tiny));
  for (i = 0; i < hash_size; i++)
    h.u.entries_tiny[i].tokens = 1;
  if (v6)
    ipv6_permitted(src6, bits, &h);
  else
    ip_permitted(src4, bits, &h);
  for (i = 0; i < hash_size; i++)
    if (h.u.entries_tiny[i].tokens == 0)
      found = i;
  free(h.u.entries_tiny);
  return found;
}

static void set_seed(const uint8_t key[16])
{
  memcpy(hash_seed, key, 16);
  hash_seed_inited = 1;
}

uint32_t ref_ip_bucket(const uint8_t key[16], uint32_t src_host, uint8_t bits,
                       uint32_t hash_size)
{
  set_seed(key);
  return bucket_probe(0, NULL, src_host, bits, hash_size);
}

uint32_t ref_ipv6_bucket(const uint8_t key[16], const uint8_t src[16],
                         uint8_t bits, uint32_t hash_size)
{
  set_seed(key);
  return bucket_probe(1, src, 0, bits, hash_size);
}

/* ---- record composition with reference functions ---------------------- */
static void to_malformed(struct pptk_rx_rec *r)
{
  uint16_t keep = r->flags & (PPTK_RX_F_VLAN | PPTK_RX_F_IPV6);
  uint16_t et = r->ethertype;
  uint8_t l3 = r->l3_off, ver = r->ip_version;
  memset(r, 0, sizeof(*r));
  r->flags = (uint16_t)(keep | PPTK_RX_F_MALFORMED);
  r->ethertype = et;
  r->l3_off = l3;
  r->ip_version = ver;
}

void ref_rx_one(const uint8_t *f, uint32_t len, const struct ref_opts *o,
                struct pptk_rx_rec *r, int with_bucket)
{
  const char *ip, *l4 = NULL;
  uint16_t et, ihl = 0, l4len = 0;
  uint32_t l3;
  uint8_t proto = 0;
  int frag = 0, v6 = 0;
  unsigned char tuple[40];

  memset(r, 0, sizeof(*r));
  if (len > 65535u || len < 14) {
    r->flags = PPTK_RX_F_MALFORMED;
    return;
  }
  et = ether_type(f);
  l3 = ETHER_HDR_LEN;
  if (et == 0x8100) {
    r->flags |= PPTK_RX_F_VLAN;
    if (len < 18) {
      r->flags |= PPTK_RX_F_MALFORMED;
      return;
    }
    et = ether_type(f + 4);
    l3 = ETHER_HDR_LEN + 4;
  }
  r->ethertype = et;
  r->l3_off = (uint8_t)l3;
  ip = (const char *)f + l3;

  if (et == ETHER_TYPE_IP) {
    uint16_t tl;
    if (len < l3 + 20) {
      to_malformed(r);
      return;
    }
    r->ip_version = ip_version(ip);
    ihl = ip_hdr_len(ip);
    tl = ip_total_len(ip);
    if (r->ip_version != 4 || ihl < 20 || tl < ihl || l3 + tl > len) {
      to_malformed(r);
      return;
    }
    r->flags |= PPTK_RX_F_PARSED;
    r->ip_cksum = ip_hdr_cksum_calc(ip, ihl);
    if (r->ip_cksum == 0)
      r->flags |= PPTK_RX_F_IP_OK;
    hdr_set32n(r->src, ip_src(ip));
    hdr_set32n(r->dst, ip_dst(ip));
    proto = ip_proto(ip);
    frag = ip_frag_off(ip) != 0 || ip_more_frags(ip);
    l4 = ip_const_payload(ip);
    l4len = (uint16_t)(tl - ihl);
  } else if (et == ETHER_TYPE_IPV6) {
    uint32_t tlen;
    uint16_t fo = 0, pfo = 0;
    r->flags |= PPTK_RX_F_IPV6;
    if (len < l3 + 40) {
      to_malformed(r);
      return;
    }
    r->ip_version = ip_version(ip);
    tlen = (uint32_t)ipv6_payload_len(ip) + 40u;
    if (r->ip_version != 6 || l3 + tlen > len) {
      to_malformed(r);
      return;
    }
    l4 = ipv6_const_proto_hdr_2(ip, &proto, &frag, &fo, &pfo);
    if (l4 == NULL) {
      to_malformed(r);
      return;
    }
    v6 = 1;
    if (is_ipv6_nexthdr(ipv6_nexthdr(ip)))
      r->flags |= PPTK_RX_F_V6_EXT;
    r->flags |= PPTK_RX_F_PARSED | PPTK_RX_F_IP_OK;
    memcpy(r->src, ipv6_const_src(ip), 16);
    memcpy(r->dst, ipv6_const_dst(ip), 16);
    l4len = (uint16_t)(tlen - (uint32_t)(l4 - ip));
  } else {
    return;
  }

  if (frag)
    r->flags |= PPTK_RX_F_FRAGMENT;
  r->proto = proto;
  r->l4_off = (uint16_t)(l4 - (const char *)f);
  r->l4_len = l4len;
  if (!frag && ((proto == 6 && l4len >= 20) || (proto == 17 && l4len >= 8))) {
    r->flags |= PPTK_RX_F_L4;
    if (proto == 6) {
      r->sport = tcp_src_port(l4);
      r->dport = tcp_dst_port(l4);
      r->l4_cksum = v6 ? tcp6_cksum_calc(ip, 40, l4, l4len)
                       : tcp_cksum_calc(ip, ihl, l4, l4len);
    } else {
      r->sport = udp_src_port(l4);
      r->dport = udp_dst_port(l4);
      r->l4_cksum = v6 ? udp6_cksum_calc(ip, 40, l4, l4len)
                       : udp_cksum_calc(ip, ihl, l4, l4len);
      if (udp_cksum(l4) == 0)
        r->flags |= PPTK_RX_F_UDP_ZERO;
    }
    if (r->l4_cksum == 0)
      r->flags |= PPTK_RX_F_L4_OK;
  }

  memcpy(tuple, r->src, 16);
  memcpy(tuple + 16, r->dst, 16);
  hdr_set16n(tuple + 32, r->sport);
  hdr_set16n(tuple + 34, r->dport);
  tuple[36] = proto;
  tuple[37] = tuple[38] = tuple[39] = 0;
  r->flow_hash = siphash_buf(o->key, tuple, sizeof(tuple));

  if (with_bucket) {
    if (!v6 && o->bits4)
      r->src_bucket = ref_ip_bucket(o->key, hdr_get32n(r->src), o->bits4, o->hash_size);
    else if (v6 && o->bits6)
      r->src_bucket = ref_ipv6_bucket(o->key, r->src, o->bits6, o->hash_size);
  }
}

/* ---- fragment side record (struct pptk_rx_frag) with the reference's
 * getters: ip_id, ip_frag_off, ip_more_frags, ip_dont_frag, ip_total_len,
 * ip_hdr_len, ip_proto (iphdr/iphdr.h), and for IPv6 the outputs of
 * ipv6_const_proto_hdr_2 (frag flag, frag_hdr_off, proto_hdr_off_from_frag)
 * with ipv6_frag_off / ipv6_more_frags on the fragment header it found.
 * The 32-bit IPv6 Identification has no reference getter: hdr_get32n of
 * the fragment header's bytes 4..7 (misc/hdr.h). */
void ref_frag_batch(const uint8_t *buf, const uint64_t *off, const uint16_t *len,
                    uint64_t stride, uint32_t fixed_len, size_t n, struct pptk_rx_frag *out)
{
  struct ref_opts o;
  memset(&o, 0, sizeof(o));
  o.hash_size = 1;
  for (size_t i = 0; i < n; i++) {
    const uint8_t *f = buf + (off ? off[i] : (uint64_t)i * stride);
    uint32_t l = len ? len[i] : fixed_len;
    struct pptk_rx_rec r;
    struct pptk_rx_frag *fr = &out[i];
    const char *ip;
    memset(fr, 0, sizeof(*fr));
    ref_rx_one(f, l, &o, &r, 0);
    if ((r.flags & (PPTK_RX_F_PARSED | PPTK_RX_F_MALFORMED)) != PPTK_RX_F_PARSED)
      continue;
    ip = (const char *)f + r.l3_off;
    if (!(r.flags & PPTK_RX_F_IPV6)) {
      fr->ident = ip_id(ip);
      fr->frag_off = ip_frag_off(ip);
      fr->data_len = (uint16_t)(ip_total_len(ip) - ip_hdr_len(ip));
      fr->next_hdr = ip_proto(ip);
      fr->flags = (uint8_t)(((ip_frag_off(ip) != 0 || ip_more_frags(ip)) ? PPTK_RX_FRAG_IS : 0) |
                            (ip_more_frags(ip) ? PPTK_RX_FRAG_MF : 0) |
                            (ip_dont_frag(ip) ? PPTK_RX_FRAG_DF : 0));
    } else {
      uint8_t proto;
      int frag = 0;
      uint16_t fo = 0, pfo = 0;
      const char *fh;
      if (ipv6_const_proto_hdr_2(ip, &proto, &frag, &fo, &pfo) == NULL || !frag)
        continue;
      fh = ip + fo;
      fr->ident = hdr_get32n(fh + 4);
      fr->frag_off = ipv6_frag_off(fh);
      fr->data_len = (uint16_t)(ipv6_payload_len(ip) + 40u - fo - 8u);
      fr->frag_hdr_off = fo;
      fr->proto_hdr_off_from_frag = pfo;
      fr->next_hdr = (uint8_t)fh[0];
      fr->flags = (uint8_t)(PPTK_RX_FRAG_IS | PPTK_RX_FRAG_V6 |
                            (ipv6_more_frags(fh) ? PPTK_RX_FRAG_MF : 0));
    }
  }
}

/* ---- threaded batch: the "reference" CPU baseline of bench.py ---------- */
struct ref_job {
  const uint8_t *buf;
  const uint64_t *off;
  const uint16_t *len;
  uint64_t stride;
  uint32_t fixed_len;
  size_t lo, hi;
  const struct ref_opts *o;
  struct pptk_rx_rec *recs;
  int with_bucket;
};

static void *ref_worker(void *arg)
{
  struct ref_job *j = arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    uint64_t off = j->off ? j->off[i] : (uint64_t)i * j->stride;
    uint32_t len = j->len ? j->len[i] : j->fixed_len;
    ref_rx_one(j->buf + off, len, j->o, &j->recs[i], j->with_bucket);
  }
  return NULL;
}

int ref_rx_batch(const uint8_t *buf, const uint64_t *off, const uint16_t *len,
                 uint64_t stride, uint32_t fixed_len, size_t n,
                 const struct ref_opts *o, struct pptk_rx_rec *recs,
                 int nthreads, int with_bucket)
{
  pthread_t th[256];
  struct ref_job jobs[256];
  int t;
  if (nthreads < 1)
    nthreads = 1;
  if (nthreads > 256)
    nthreads = 256;
  if (with_bucket)
    nthreads = 1; /* the black-box bucket probe touches the global seed */
  for (t = 0; t < nthreads; t++) {
    jobs[t].buf = buf;
    jobs[t].off = off;
    jobs[t].len = len;
    jobs[t].stride = stride;
    jobs[t].fixed_len = fixed_len;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    jobs[t].o = o;
    jobs[t].recs = recs;
    jobs[t].with_bucket = with_bucket;
  }
  if (nthreads == 1) {
    ref_worker(&jobs[0]);
    return 0;
  }
  for (t = 0; t < nthreads; t++)
    if (pthread_create(&th[t], NULL, ref_worker, &jobs[t]) != 0)
      return -1;
  for (t = 0; t < nthreads; t++)
    pthread_join(th[t], NULL);
  return 0;
}

/* ipcksumperf loop shape (iphdr/ipcksumperf.c:21-29). */
uint32_t ref_cksum_loop(const uint8_t *buf, size_t sz, uint64_t iters)
{
  uint32_t x = 0;
  for (uint64_t i = 0; i < iters; i++) {
    struct ip_cksum_ctx ctx = IP_CKSUM_CTX_INITER;
    ip_cksum_feed(&ctx, buf, sz);
    x ^= ip_cksum_postprocess(&ctx) + (uint32_t)i;
  }
  return x;
}

/* ---- the reference's own rate limiter over a batch: ip_permitted /
 * ipv6_permitted called once per subject frame in frame order on a struct
 * ip_hash whose entries (tiny / small / full, chosen by initial_tokens as
 * iphash.h:53-61 does) hold `tokens` (copied in, and back out after).  The
 * source address comes from the record (its src bytes); the reference
 * recomputes the bucket from it, so this pins the record's src_bucket too. */
static void entries_alloc(struct ip_hash *h)
{
  if (use_tiny(h))
    h->u.entries_tiny = calloc(h->hash_size, sizeof(*h->u.entries_tiny));
  else if (use_small(h))
    h->u.entries_small = calloc(h->hash_size, sizeof(*h->u.entries_small));
  else
    h->u.entries = calloc(h->hash_size, sizeof(*h->u.entries));
}

static void entries_set(struct ip_hash *h, const uint32_t *tokens)
{
  uint32_t i;
  for (i = 0; i < h->hash_size; i++) {
    if (use_tiny(h))
      h->u.entries_tiny[i].tokens = (uint8_t)tokens[i];
    else if (use_small(h))
      h->u.entries_small[i].tokens = (uint16_t)tokens[i];
    else
      h->u.entries[i].tokens = tokens[i];
  }
}

static void entries_get(struct ip_hash *h, uint32_t *tokens)
{
  uint32_t i;
  for (i = 0; i < h->hash_size; i++) {
    if (use_tiny(h))
      tokens[i] = h->u.entries_tiny[i].tokens;
    else if (use_small(h))
      tokens[i] = h->u.entries_small[i].tokens;
    else
      tokens[i] = h->u.entries[i].tokens;
  }
}

static void entries_free(struct ip_hash *h)
{
  if (use_tiny(h))
    free(h->u.entries_tiny);
  else if (use_small(h))
    free(h->u.entries_small);
  else
    free(h->u.entries);
}

void ref_permit_batch(const uint8_t key[16], const struct pptk_rx_rec *recs, size_t n,
                      int family, uint8_t bits, const uint8_t *subject,
                      uint32_t hash_size, uint32_t initial_tokens, uint32_t *tokens,
                      uint8_t *verdict)
{
  struct ip_hash h;
  size_t i;
  set_seed(key);
  memset(&h, 0, sizeof(h));
  h.hash_size = hash_size;
  h.initial_tokens = initial_tokens;
  entries_alloc(&h);
  entries_set(&h, tokens);
  for (i = 0; i < n; i++) {
    const struct pptk_rx_rec *r = &recs[i];
    const int v6 = (r->flags & PPTK_RX_F_IPV6) != 0;
    if (!(r->flags & PPTK_RX_F_PARSED) || v6 != (family == 6) ||
        (subject && !subject[i])) {
      verdict[i] = 2;
      continue;
    }
    if (v6)
      verdict[i] = (uint8_t)ipv6_permitted(r->src, bits, &h);
    else
      verdict[i] = (uint8_t)ip_permitted(((uint32_t)r->src[0] << 24) | ((uint32_t)r->src[1] << 16) |
                                         ((uint32_t)r->src[2] << 8) | r->src[3], bits, &h);
  }
  entries_get(&h, tokens);
  entries_free(&h);
}

/* The reference's refill timer itself: ip_hash_init() registers
 * batch_timer_fn for every batch_size buckets; as the timer loop would,
 * take batch k's timer off the heap and run it. */
void ref_tokens_refill(uint32_t hash_size, uint32_t batch_size, uint32_t initial_tokens,
                       uint32_t timer_add, uint32_t k, uint32_t *tokens)
{
  struct ip_hash h;
  struct timer_linkheap heap;
  timer_linkheap_init(&heap);
  memset(&h, 0, sizeof(h));
  h.hash_size = hash_size;
  h.batch_size = batch_size;
  h.initial_tokens = initial_tokens;
  h.timer_add = timer_add;
  h.timer_period = 1000;
  ip_hash_init(&h, &heap, NULL);
  entries_set(&h, tokens);
  timer_linkheap_remove(&heap, &h.timers[k]);
  h.timers[k].fn(&h.timers[k], &heap, h.timers[k].userdata, NULL);
  entries_get(&h, tokens);
  ip_hash_free(&h, &heap);
  timer_linkheap_free(&heap);
}

/* ---- tx side: the reference's own setters (iphdr/ipcksum.h:101-211) on
 * every frame the record composition parses, located by that composition:
 * ip_set_hdr_cksum_calc(ip, ihl) for IPv4, then tcp/udp(6)_set_cksum_calc
 * (ip, ihl | 40, l4, l4_len) when the record has an L4 header. */
void ref_tx_batch(uint8_t *buf, const uint64_t *off, const uint16_t *len, uint64_t stride,
                  uint32_t fixed_len, size_t n)
{
  struct ref_opts o;
  size_t i;
  memset(&o, 0, sizeof(o));
  for (i = 0; i < n; i++) {
    uint8_t *f = buf + (off ? off[i] : i * stride);
    const uint32_t flen = len ? len[i] : fixed_len;
    struct pptk_rx_rec r;
    uint8_t *ip, *l4;
    ref_rx_one(f, flen, &o, &r, 0);
    if (!(r.flags & PPTK_RX_F_PARSED) || (r.flags & PPTK_RX_F_MALFORMED))
      continue;
    ip = f + r.l3_off;
    l4 = f + r.l4_off;
    if (!(r.flags & PPTK_RX_F_IPV6))
      ip_set_hdr_cksum_calc(ip, ip_hdr_len(ip));
    if (!(r.flags & PPTK_RX_F_L4))
      continue;
    if (r.flags & PPTK_RX_F_IPV6) {
      if (r.proto == 6)
        tcp6_set_cksum_calc(ip, 40, l4, r.l4_len);
      else
        udp6_set_cksum_calc(ip, 40, l4, r.l4_len);
    } else {
      if (r.proto == 6)
        tcp_set_cksum_calc(ip, ip_hdr_len(ip), l4, r.l4_len);
      else
        udp_set_cksum_calc(ip, ip_hdr_len(ip), l4, r.l4_len);
    }
  }
}

/* ---- header rewrite: the reference's own incremental-update functions
 * (iphdr/ipcksum.h:213-393), called in the order and under the conditions
 * pptk_tx_rewrite_device defines (include/pptk_rx.h): on frames the record
 * composition parses as IPv4; L4 follow-ups only with an L4 header (proto
 * passed as 0 otherwise, which makes ip_set_src/dst_cksum_update touch the
 * IP header alone); TTL 0 under DECR_TTL skipped (the reference abort()s). */
void ref_rewrite_batch(uint8_t *buf, const uint64_t *off, const uint16_t *len, uint64_t stride,
                       uint32_t fixed_len, size_t n, const struct pptk_rewrite *rw,
                       uint64_t rw_count, uint8_t *status)
{
  struct ref_opts o;
  size_t i;
  memset(&o, 0, sizeof(o));
  for (i = 0; i < n; i++) {
    uint8_t *f = buf + (off ? off[i] : i * stride);
    const uint32_t flen = len ? len[i] : fixed_len;
    const struct pptk_rewrite *w = &rw[rw_count == 1 ? 0 : i];
    struct pptk_rx_rec r;
    uint8_t *ip, *l4, st = 0;
    int l4ok;
    ref_rx_one(f, flen, &o, &r, 0);
    if ((r.flags & (PPTK_RX_F_PARSED | PPTK_RX_F_MALFORMED | PPTK_RX_F_IPV6)) != PPTK_RX_F_PARSED)
      goto done;
    ip = f + r.l3_off;
    l4 = f + r.l4_off;
    l4ok = (r.flags & PPTK_RX_F_L4) != 0;
    if ((w->ops & PPTK_RW_DECR_TTL) && ip_ttl(ip) == 0) {
      st = PPTK_RW_ST_TTL_ZERO;
      goto done;
    }
    st = PPTK_RW_ST_IP | (l4ok ? PPTK_RW_ST_L4 : 0);
    if (w->ops & PPTK_RW_DECR_TTL) {
      if (!ip_decr_ttl_cksum_update(ip))
        st |= PPTK_RW_ST_EXPIRED;
    }
    if (w->ops & PPTK_RW_SRC)
      ip_set_src_cksum_update(ip, ip_hdr_len(ip), l4ok ? r.proto : 0, l4, r.l4_len, w->src);
    if (w->ops & PPTK_RW_DST)
      ip_set_dst_cksum_update(ip, ip_hdr_len(ip), l4ok ? r.proto : 0, l4, r.l4_len, w->dst);
    if (l4ok && (w->ops & PPTK_RW_SPORT)) {
      if (r.proto == 6)
        tcp_set_src_port_cksum_update(l4, r.l4_len, w->sport);
      else
        udp_set_src_port_cksum_update(l4, r.l4_len, w->sport);
    }
    if (l4ok && (w->ops & PPTK_RW_DPORT)) {
      if (r.proto == 6)
        tcp_set_dst_port_cksum_update(l4, r.l4_len, w->dport);
      else
        udp_set_dst_port_cksum_update(l4, r.l4_len, w->dport);
    }
    if ((w->ops & PPTK_RW_ICMP_ID) && r.proto == 1 && !(r.flags & PPTK_RX_F_FRAGMENT) &&
        r.l4_len >= 8 && (icmp_type(l4) == 8 || icmp_type(l4) == 0)) {
      icmp_set_echo_identifier_cksum_update(l4, r.l4_len, w->sport);
      st |= PPTK_RW_ST_ICMP;
    }
done:
    if (status)
      status[i] = st;
  }
}

uint16_t ref_update_cksum16(uint16_t c, uint16_t o, uint16_t nw)
{
  return ip_update_cksum16(c, o, nw);
}

uint16_t ref_update_cksum32(uint16_t c, uint32_t o, uint32_t nw)
{
  return (uint16_t)ip_update_cksum32(c, o, nw);
}

/* ---- MSS clamping: the reference's tcp_parse_options (iphdr/iphdr.c:4-132)
 * and tcp_set_mss_cksum_update (iphdr/ipcksum.h:466-489), composed as
 * pptk_tcp_mss_clamp_device defines (include/pptk_rx.h). */
void ref_mss_clamp_batch(uint8_t *buf, const uint64_t *off, const uint16_t *len, uint64_t stride,
                         uint32_t fixed_len, size_t n, uint16_t mss, uint32_t flags,
                         uint8_t *status)
{
  struct ref_opts o;
  size_t i;
  memset(&o, 0, sizeof(o));
  for (i = 0; i < n; i++) {
    uint8_t *f = buf + (off ? off[i] : i * stride);
    const uint32_t flen = len ? len[i] : fixed_len;
    struct pptk_rx_rec r;
    struct tcp_information info;
    uint8_t *t, st = 0;
    ref_rx_one(f, flen, &o, &r, 0);
    if ((r.flags & (PPTK_RX_F_PARSED | PPTK_RX_F_MALFORMED | PPTK_RX_F_L4)) !=
            (PPTK_RX_F_PARSED | PPTK_RX_F_L4) ||
        r.proto != 6)
      goto done;
    t = f + r.l4_off;
    if ((flags & PPTK_MSS_SYN_ONLY) && !tcp_syn(t))
      goto done;
    st = PPTK_MSS_ST_TCP;
    if (tcp_data_offset(t) > r.l4_len) {
      st |= PPTK_MSS_ST_BADOPT;
      goto done;
    }
    tcp_parse_options(t, &info);
    if (!info.options_valid) {
      st |= PPTK_MSS_ST_BADOPT;
      goto done;
    }
    if (info.mssoff == 0)
      goto done;
    st |= PPTK_MSS_ST_FOUND;
    if (info.mss > mss) {
      tcp_set_mss_cksum_update(t, &info, mss);
      st |= PPTK_MSS_ST_CLAMPED;
    }
done:
    if (status)
      status[i] = st;
  }
}

/* The kept TCP option API, one frame's TCP header at a time, for the
 * host-API parity tests (tests/test_capi.py): parse results packed as
 * valid | wscale<<8 | sack_perm<<16 | ts_present<<17 | mssoff<<24, mss,
 * ts, tsecho; and the SACK/timestamp walk. */
uint32_t ref_tcp_parse_options(uint8_t *t, uint16_t *mss, uint32_t *ts, uint32_t *tsecho)
{
  struct tcp_information info;
  tcp_parse_options(t, &info);
  *mss = info.mss;
  *ts = info.ts;
  *tsecho = info.tsecho;
  return (uint32_t)info.options_valid | ((uint32_t)info.wscale << 8) |
         ((uint32_t)info.sack_permitted << 16) | ((uint32_t)info.ts_present << 17) |
         ((uint32_t)info.mssoff << 24);
}

uint32_t ref_tcp_find_sack_ts(uint8_t *t)
{
  struct sack_ts_headers h;
  tcp_find_sack_ts_headers(t, &h);
  return (uint32_t)h.sackoff | ((uint32_t)h.sacklen << 8) | ((uint32_t)h.tsoff << 16);
}

int64_t ref_tcp_find_sack(uint8_t *t, uint32_t *sacklen, int *align)
{
  size_t l = 0;
  uint8_t *p = tcp_find_sack_header(t, &l, align);
  *sacklen = (uint32_t)l;
  return p ? (int64_t)(p - t) : -1;
}

/* Option rewrites on one TCP header (op: 0 set_mss(v), 1 disable_sack,
 * 2 adjust_sack_2(v), 3 adjust_tsval(v), 4 adjust_tsecho(v), 5 ack_off,
 * 6 seq(v), 7 ack(v), 8 window(v)); option offsets from the reference's
 * own walks. */
void ref_tcp_opt_op(uint8_t *t, int op, uint32_t v)
{
  struct tcp_information info;
  struct sack_ts_headers h;
  size_t sl = 0;
  int al = 0;
  void *sack;
  switch (op) {
  case 0:
    tcp_parse_options(t, &info);
    if (info.options_valid && info.mssoff)
      tcp_set_mss_cksum_update(t, &info, (uint16_t)v);
    break;
  case 1:
    sack = tcp_find_sack_header(t, &sl, &al);
    if (sack)
      tcp_disable_sack_cksum_update(t, sack, sl, al);
    break;
  case 2:
    tcp_find_sack_ts_headers(t, &h);
    tcp_adjust_sack_cksum_update_2(t, &h, v);
    break;
  case 3:
    tcp_find_sack_ts_headers(t, &h);
    tcp_adjust_tsval_cksum_update(t, &h, v);
    break;
  case 4:
    tcp_find_sack_ts_headers(t, &h);
    tcp_adjust_tsecho_cksum_update(t, &h, v);
    break;
  case 5: tcp_set_ack_off_cksum_update(t); break;
  case 6: tcp_set_seq_number_cksum_update(t, 0, v); break;
  case 7: tcp_set_ack_number_cksum_update(t, 0, v); break;
  case 8: tcp_set_window_cksum_update(t, 0, (uint16_t)v); break;
  default: break;
  }
}
