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
  ip_set_hdr_cksum(iphdr, 0);
  ip_set_hdr_cksum(iphdr, ip_hdr_cksum_calc(iphdr, iplen));
}

static inline void tcp_set_cksum_calc(void *iphdr, uint16_t iplen, void *tcphdr, uint16_t tcplen)
{
  tcp_set_cksum(tcphdr, 0);
  tcp_set_cksum(tcphdr, tcp_cksum_calc(iphdr, iplen, tcphdr, tcplen));
}

static inline void udp_set_cksum_calc(void *iphdr, uint16_t iplen, void *udphdr, uint16_t udplen)
{
  udp_set_cksum(udphdr, 0);
  udp_set_cksum(udphdr, udp_cksum_calc(iphdr, iplen, udphdr, udplen));
}

static inline void tcp6_set_cksum_calc(void *iphdr, uint16_t iplen, void *tcphdr, uint16_t tcplen)
{
  tcp_set_cksum(tcphdr, 0);
  tcp_set_cksum(tcphdr, tcp6_cksum_calc(iphdr, iplen, tcphdr, tcplen));
}

static inline void udp6_set_cksum_calc(void *iphdr, uint16_t iplen, void *udphdr, uint16_t udplen)
{
  udp_set_cksum(udphdr, 0);
  udp_set_cksum(udphdr, udp6_cksum_calc(iphdr, iplen, udphdr, udplen));
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

#ifdef __cplusplus
}
#endif

#endif
