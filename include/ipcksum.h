/*
 * ipcksum.h -- Internet checksum API (RFC 1071), per packet, on the host.
 *
 * Same names, signatures and results as the reference's iphdr/ipcksum.h:11-99
 * (implementation in pptk_amd/csrc/host/ipcksum.c).  Every *_calc returns
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

#ifdef __cplusplus
}
#endif

#endif
