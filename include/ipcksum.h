/*
 * ipcksum.h -- Internet checksum API (RFC 1071), per packet, on the host.
 *
 * Same names, signatures and results as the reference's iphdr/ipcksum.h:11-99
 * (implementation in pptk_amd/csrc/host/ipcksum.c), plus its tx-side setters
 * (:101-211) and incremental updates (:213-393; the batch form is
 * pptk_tx_rewrite_device in pptk_rx.h).  Every *_calc returns
 * the checksum over the given bytes as ntohs(~folded sum): 0 means a packet
 * whose checksum field is correct.  Caller contract violations abort() as in
 * the reference (ihl > iplen, iplen < 20 / 40, version not 4/6, proto != 6
 * in tcp46_cksum_calc).
 *
 * Batches should not loop over these: pptk_rx_batch() (pptk_rx.h) computes
 * the same values for a whole rx batch on the GPU.
 */
#ifndef _IPCKSUM_H_
#define _IPCKSUM_H_

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "hdr.h"
#include "iphdr.h"

#ifdef __cplusplus
extern "C" {
#endif

struct ip_cksum_ctx {
  uint32_t sum;
};

#define IP_CKSUM_CTX_INITER { .sum = 0 }

/* fold with end-around carry, complement, to network order */
static inline uint16_t ip_cksum_postprocess(struct ip_cksum_ctx *ctx)
{
  uint32_t s = ctx->sum;
  s = (s >> 16) + (s & 0xffff);
  s = (s >> 16) + (s & 0xffff);
  return ntohs((uint16_t)~s);
}

static inline void ip_cksum_add16(struct ip_cksum_ctx *ctx, uint16_t val16)
{
  ctx->sum += val16;
}

/* odd trailing byte: contributes as the first byte of a zero-padded word */
static inline void ip_cksum_add_leftover(struct ip_cksum_ctx *ctx, uint8_t val)
{
  ctx->sum += htons((uint16_t)(val << 8));
}

static inline void ip_cksum_feed32ptr(struct ip_cksum_ctx *ctx, const void *buf)
{
  ctx->sum += hdr_get16h(buf);
  ctx->sum += hdr_get16h((const unsigned char *)buf + 2);
}

void ip_cksum_feed(struct ip_cksum_ctx *ctx, const void *buf, size_t sz);

uint16_t ip_hdr_cksum_calc(const void *iphdr, uint16_t iplen);

static inline uint16_t ip46_hdr_cksum_calc(const void *iphdr)
{
  int v = pptk_ipver_or_die(iphdr);
  return v == 4 ? ip_hdr_cksum_calc(iphdr, ip_hdr_len(iphdr)) : 0;
}

uint16_t tcp_cksum_calc(const void *iphdr, uint16_t iplen, const void *tcphdr,
                        uint16_t tcplen);
uint16_t udp_cksum_calc(const void *iphdr, uint16_t iplen, const void *udphdr,
                        uint16_t udplen);
uint16_t tcp6_cksum_calc(const void *iphdr, uint16_t iplen, const void *tcphdr,
                         uint16_t tcplen);
uint16_t udp6_cksum_calc(const void *iphdr, uint16_t iplen, const void *udphdr,
                         uint16_t udplen);

/* v4/v6 TCP dispatch; L4 at the fixed header length (no extension walk),
 * as in the reference (ipcksum.h:74-96). */
static inline uint16_t tcp46_cksum_calc(const void *iphdr)
{
  uint16_t tcplen = ip46_payload_len(iphdr);
  uint16_t iplen = ip46_hdr_len(iphdr);
  const void *tcphdr = ip46_const_payload(iphdr);
  if (ip46_proto(iphdr) != 6)
    abort();
  return ip_version(iphdr) == 4 ? tcp_cksum_calc(iphdr, iplen, tcphdr, tcplen)
                                : tcp6_cksum_calc(iphdr, iplen, tcphdr, tcplen);
}

/* ---- tx side: set a checksum field to the value that makes the packet
 * verify (ipcksum.h:101-211): zero the field, compute, store. */
static inline void ip_set_hdr_cksum_calc(void *iphdr, uint16_t iplen)
{
  if (iplen < 20)
    abort();
  ip_set_hdr_cksum(iphdr, 0);
  ip_set_hdr_cksum(iphdr, ip_hdr_cksum_calc(iphdr, iplen));
}

/* ipcksum.h:113-128: IPv6 has no header checksum (nothing to do) */
static inline void ip46_set_hdr_cksum_calc(void *iphdr)
{
  if (pptk_ipver_or_die(iphdr) == 4)
    ip_set_hdr_cksum_calc(iphdr, ip_hdr_len(iphdr));
}

static inline void tcp_set_cksum_calc(void *iphdr, uint16_t iplen, void *tcphdr, uint16_t tcplen)
{
  if (iplen < 20 || tcplen < 20)
    abort();
  tcp_set_cksum(tcphdr, 0);
  tcp_set_cksum(tcphdr, tcp_cksum_calc(iphdr, iplen, tcphdr, tcplen));
}

static inline void udp_set_cksum_calc(void *iphdr, uint16_t iplen, void *udphdr, uint16_t udplen)
{
  if (iplen < 20 || udplen < 8)
    abort();
  udp_set_cksum(udphdr, 0);
  udp_set_cksum(udphdr, udp_cksum_calc(iphdr, iplen, udphdr, udplen));
}

static inline void tcp6_set_cksum_calc(void *iphdr, uint16_t iplen, void *tcphdr, uint16_t tcplen)
{
  if (iplen < 40 || tcplen < 20)
    abort();
  tcp_set_cksum(tcphdr, 0);
  tcp_set_cksum(tcphdr, tcp6_cksum_calc(iphdr, iplen, tcphdr, tcplen));
}

static inline void udp6_set_cksum_calc(void *iphdr, uint16_t iplen, void *udphdr, uint16_t udplen)
{
  if (iplen < 40 || udplen < 8)
    abort();
  udp_set_cksum(udphdr, 0);
  udp_set_cksum(udphdr, udp6_cksum_calc(iphdr, iplen, udphdr, udplen));
}

/* ipcksum.h:160-181: TCP at the fixed header length, as tcp46_cksum_calc */
static inline void tcp46_set_cksum_calc(void *iphdr)
{
  uint16_t tcplen = ip46_payload_len(iphdr);
  uint16_t iplen = ip46_hdr_len(iphdr);
  void *tcphdr = (unsigned char *)iphdr + iplen;
  if (ip46_proto(iphdr) != 6)
    abort();
  if (ip_version(iphdr) == 4)
    tcp_set_cksum_calc(iphdr, iplen, tcphdr, tcplen);
  else
    tcp6_set_cksum_calc(iphdr, iplen, tcphdr, tcplen);
}

/* ---- incremental update (RFC 1624 eqn. 3), ipcksum.h:213-236: the new
 * checksum after a 16-bit field changes from old16 to new16 (host-order
 * values of big-endian fields); 32-bit = high half, then low half. */
static inline uint16_t ip_update_cksum16(uint16_t old_cksum16, uint16_t old16, uint16_t new16)
{
  uint32_t s = (uint16_t)~old_cksum16;
  s += (uint16_t)~old16;
  s += new16;
  s = (s & 0xffff) + (s >> 16);
  s = (s & 0xffff) + (s >> 16);
  return (uint16_t)~s;
}

static inline uint32_t ip_update_cksum32(uint16_t old_cksum, uint32_t old32, uint32_t new32)
{
  return ip_update_cksum16(ip_update_cksum16(old_cksum, (uint16_t)(old32 >> 16),
                                             (uint16_t)(new32 >> 16)),
                           (uint16_t)old32, (uint16_t)new32);
}

/* L4 follow-up of an IPv4 address change: TCP always, UDP unless its
 * checksum is 0 ("none"), ipcksum.h:245-260 / :356-371 */
static inline void pptk_l4_addr_update(void *payhdr, uint8_t proto, uint32_t old32,
                                       uint32_t new32)
{
  if (proto == 6) {
    tcp_set_cksum(payhdr, (uint16_t)ip_update_cksum32(tcp_cksum(payhdr), old32, new32));
  } else if (proto == 17) {
    uint16_t c = udp_cksum(payhdr);
    if (c != 0)
      udp_set_cksum(payhdr, (uint16_t)ip_update_cksum32(c, old32, new32));
  }
}

static inline void ip_set_src_cksum_update(void *iphdr, uint16_t iplen, uint8_t proto,
                                           void *payhdr, uint16_t paylen, uint32_t src)
{
  uint32_t old = ip_src(iphdr);
  (void)iplen;
  (void)paylen;
  ip_set_hdr_cksum(iphdr, (uint16_t)ip_update_cksum32(ip_hdr_cksum(iphdr), old, src));
  pptk_l4_addr_update(payhdr, proto, old, src);
  ip_set_src(iphdr, src);
}

static inline void ip_set_dst_cksum_update(void *iphdr, uint16_t iplen, uint8_t proto,
                                           void *payhdr, uint16_t paylen, uint32_t dst)
{
  uint32_t old = ip_dst(iphdr);
  (void)iplen;
  (void)paylen;
  ip_set_hdr_cksum(iphdr, (uint16_t)ip_update_cksum32(ip_hdr_cksum(iphdr), old, dst));
  pptk_l4_addr_update(payhdr, proto, old, dst);
  ip_set_dst(iphdr, dst);
}

/* port rewrites, ipcksum.h:263-281 (TCP) and :323-347 (UDP, 0 stays 0) */
static inline void tcp_set_src_port_cksum_update(void *tcphdr, uint16_t tcplen, uint16_t port)
{
  (void)tcplen;
  tcp_set_cksum(tcphdr, ip_update_cksum16(tcp_cksum(tcphdr), tcp_src_port(tcphdr), port));
  tcp_set_src_port(tcphdr, port);
}

static inline void tcp_set_dst_port_cksum_update(void *tcphdr, uint16_t tcplen, uint16_t port)
{
  (void)tcplen;
  tcp_set_cksum(tcphdr, ip_update_cksum16(tcp_cksum(tcphdr), tcp_dst_port(tcphdr), port));
  tcp_set_dst_port(tcphdr, port);
}

static inline void udp_set_src_port_cksum_update(void *udphdr, uint16_t udplen, uint16_t port)
{
  uint16_t c = udp_cksum(udphdr);
  (void)udplen;
  if (c != 0)
    udp_set_cksum(udphdr, ip_update_cksum16(c, udp_src_port(udphdr), port));
  udp_set_src_port(udphdr, port);
}

static inline void udp_set_dst_port_cksum_update(void *udphdr, uint16_t udplen, uint16_t port)
{
  uint16_t c = udp_cksum(udphdr);
  (void)udplen;
  if (c != 0)
    udp_set_cksum(udphdr, ip_update_cksum16(c, udp_dst_port(udphdr), port));
  udp_set_dst_port(udphdr, port);
}

/* ipcksum.h:374-393: TTL and protocol share a 16-bit word; returns ttl > 0
 * after the decrement; TTL 0 is a caller contract violation (abort). */
static inline int ip_decr_ttl_cksum_update(void *pkt)
{
  uint8_t ttl = ip_ttl(pkt), proto = ip_proto(pkt);
  if (ttl == 0)
    abort();
  ip_set_hdr_cksum(pkt, ip_update_cksum16(ip_hdr_cksum(pkt), (uint16_t)((ttl << 8) | proto),
                                          (uint16_t)(((ttl - 1) << 8) | proto)));
  ip_set_ttl(pkt, (uint8_t)(ttl - 1));
  return ttl - 1 > 0;
}

/* ---- TCP / ICMP field rewrites with incremental update, ipcksum.h:283-321 */
static inline void icmp_set_echo_identifier_cksum_update(void *icmphdr, uint16_t icmplen,
                                                         uint16_t id)
{
  (void)icmplen;
  icmp_set_checksum(icmphdr, ip_update_cksum16(icmp_checksum(icmphdr),
                                               icmp_echo_identifier(icmphdr), id));
  icmp_set_echo_identifier(icmphdr, id);
}

static inline void tcp_set_seq_number_cksum_update(void *tcphdr, uint16_t tcplen, uint32_t seq)
{
  (void)tcplen;
  tcp_set_cksum(tcphdr, (uint16_t)ip_update_cksum32(tcp_cksum(tcphdr), tcp_seq_number(tcphdr), seq));
  tcp_set_seq_number(tcphdr, seq);
}

static inline void tcp_set_ack_number_cksum_update(void *tcphdr, uint16_t tcplen, uint32_t ack)
{
  (void)tcplen;
  tcp_set_cksum(tcphdr, (uint16_t)ip_update_cksum32(tcp_cksum(tcphdr), tcp_ack_number(tcphdr), ack));
  tcp_set_ack_number(tcphdr, ack);
}

static inline void tcp_set_window_cksum_update(void *tcphdr, uint16_t tcplen, uint16_t window)
{
  (void)tcplen;
  tcp_set_cksum(tcphdr, ip_update_cksum16(tcp_cksum(tcphdr), tcp_window(tcphdr), window));
  tcp_set_window(tcphdr, window);
}

/* ipcksum.h:395-406: clear ACK; the flags byte shares a word with the data
 * offset (bytes 12-13) */
static inline void tcp_set_ack_off_cksum_update(void *pkt)
{
  unsigned char *t = (unsigned char *)pkt;
  uint16_t w_old = hdr_get16n(t + 12);
  t[13] &= (unsigned char)~0x10;
  tcp_set_cksum(pkt, ip_update_cksum16(tcp_cksum(pkt), w_old, hdr_get16n(t + 12)));
}

/* ---- TCP option rewrites, ipcksum.h:408-650.  The checksum sums 16-bit
 * words from the start of the TCP header, so a field at an odd offset is
 * folded in through the two words that straddle it: each straddling word is
 * read before and after the field is written, and the updates are applied
 * in the reference's order (one's-complement results can differ between
 * orders only in the representation of zero, so the order is kept). */
/* ipcksum.h:408-464: overwrite a SACK option with NOPs (kind 1); the
 * "unaligned" form updates the two words straddling each rewritten pair
 * (reading the byte before the option and the one after each pair). */
static inline void tcp_disable_sack_cksum_update(void *pkt, void *sackhdr, size_t sacklen,
                                                 int sixteen_bit_align)
{
  unsigned char *h = (unsigned char *)sackhdr;
  uint16_t c = tcp_cksum(pkt);
  size_t k = 0;
  for (; k + 1 <= sacklen; k += 2) {
    const int whole = k + 2 <= sacklen;   /* a pair, or the odd last byte */
    if (sixteen_bit_align) {
      uint16_t o = hdr_get16n(h + k);
      uint16_t nw = whole ? 0x0101 : (uint16_t)((o & 0xff) | 0x0100);
      c = ip_update_cksum16(c, o, nw);
      hdr_set16n(h + k, nw);
    } else {
      uint16_t o1 = hdr_get16n(h + k - 1), o2 = hdr_get16n(h + k + 1);
      uint16_t nw = whole ? 0x0101 : (uint16_t)((hdr_get16n(h + k) & 0xff) | 0x0100);
      hdr_set16n(h + k, nw);
      c = ip_update_cksum16(c, o1, hdr_get16n(h + k - 1));
      c = ip_update_cksum16(c, o2, hdr_get16n(h + k + 1));
    }
    if (!whole)
      break;
  }
  tcp_set_cksum(pkt, c);
}

/* ipcksum.h:466-489: set the MSS option's value (mssoff from
 * tcp_parse_options) */
static inline void tcp_set_mss_cksum_update(void *pkt, struct tcp_information *opts, uint16_t mss)
{
  unsigned char *t = (unsigned char *)pkt;
  const size_t f = (size_t)opts->mssoff + 2;   /* the value field */
  uint16_t c = tcp_cksum(pkt);
  if (f % 2 == 0) {
    c = ip_update_cksum16(c, hdr_get16n(t + f), mss);
    hdr_set16n(t + f, mss);
  } else {
    uint16_t o1 = hdr_get16n(t + f - 1), o2 = hdr_get16n(t + f + 1);
    hdr_set16n(t + f, mss);
    c = ip_update_cksum16(c, o1, hdr_get16n(t + f - 1));
    c = ip_update_cksum16(c, o2, hdr_get16n(t + f + 1));
  }
  tcp_set_cksum(pkt, c);
}

/* ipcksum.h:491-537: add `adjustment` to every SACK block edge (8-byte
 * blocks from option offset 2).  In the reference's unaligned branch the
 * block loop never advances (no `curoff += 8`, :512-535), so for a SACK
 * option of 10 or more bytes at an odd offset it does not return; here each
 * block is adjusted once, the evident intent (parity unpinned for that
 * branch; the aligned branch and short unaligned options match). */
static inline void tcp_adjust_sack_cksum_update(void *pkt, void *sackhdr, size_t sacklen,
                                                int sixteen_bit_align, uint32_t adjustment)
{
  unsigned char *h = (unsigned char *)sackhdr;
  uint16_t c = tcp_cksum(pkt);
  size_t k;
  for (k = 2; k + 8 <= sacklen; k += 8) {
    const uint32_t s_new = hdr_get32n(h + k) + adjustment;
    const uint32_t e_new = hdr_get32n(h + k + 4) + adjustment;
    if (sixteen_bit_align) {
      c = (uint16_t)ip_update_cksum32(c, hdr_get32n(h + k), s_new);
      c = (uint16_t)ip_update_cksum32(c, hdr_get32n(h + k + 4), e_new);
      hdr_set32n(h + k, s_new);
      hdr_set32n(h + k + 4, e_new);
    } else {
      uint16_t o1 = hdr_get16n(h + k - 1);
      uint32_t o2 = hdr_get32n(h + k + 1), o3 = hdr_get32n(h + k + 5);
      hdr_set32n(h + k, s_new);
      hdr_set32n(h + k + 4, e_new);
      c = ip_update_cksum16(c, o1, hdr_get16n(h + k - 1));
      c = (uint16_t)ip_update_cksum32(c, o2, hdr_get32n(h + k + 1));
      c = (uint16_t)ip_update_cksum32(c, o3, hdr_get32n(h + k + 5));
    }
  }
  tcp_set_cksum(pkt, c);
}

/* ipcksum.h:539-611: add `adjustment` to the timestamp value (field at
 * tsoff + 2) or echo reply (tsoff + 6); nothing without a timestamp option */
static inline void pptk_tcp_adjust_ts32(void *pkt, size_t f, uint32_t adjustment)
{
  unsigned char *t = (unsigned char *)pkt;
  uint16_t c = tcp_cksum(pkt);
  const uint32_t nw = hdr_get32n(t + f) + adjustment;
  if (f % 2 == 0) {
    c = (uint16_t)ip_update_cksum32(c, hdr_get32n(t + f), nw);
    hdr_set32n(t + f, nw);
  } else {
    uint16_t o[3];
    int i;
    for (i = 0; i < 3; i++)
      o[i] = hdr_get16n(t + f - 1 + 2 * i);
    hdr_set32n(t + f, nw);
    for (i = 0; i < 3; i++)
      c = ip_update_cksum16(c, o[i], hdr_get16n(t + f - 1 + 2 * i));
  }
  tcp_set_cksum(pkt, c);
}

static inline void tcp_adjust_tsval_cksum_update(void *pkt, struct sack_ts_headers *hdrs,
                                                 uint32_t adjustment)
{
  if (hdrs->tsoff != 0)
    pptk_tcp_adjust_ts32(pkt, (size_t)hdrs->tsoff + 2, adjustment);
}

static inline void tcp_adjust_tsecho_cksum_update(void *pkt, struct sack_ts_headers *hdrs,
                                                  uint32_t adjustment)
{
  if (hdrs->tsoff != 0)
    pptk_tcp_adjust_ts32(pkt, (size_t)hdrs->tsoff + 6, adjustment);
}

/* ipcksum.h:613-623 */
static inline void tcp_adjust_sack_cksum_update_2(void *pkt, struct sack_ts_headers *hdrs,
                                                  uint32_t adjustment)
{
  if (hdrs->sackoff != 0)
    tcp_adjust_sack_cksum_update(pkt, (unsigned char *)pkt + hdrs->sackoff, hdrs->sacklen,
                                 !(hdrs->sackoff % 2), adjustment);
}

#ifdef __cplusplus
}
#endif

#endif
