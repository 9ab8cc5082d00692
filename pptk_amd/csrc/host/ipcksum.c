/*
 * ipcksum.c -- host implementation of the per-packet checksum API
 * (include/ipcksum.h; reference iphdr/ipcksum.c:9-181).
 *
 * ip_cksum_feed sums 8-byte words into a 64-bit accumulator (carries land
 * in the high half and are folded back once), which yields exactly the
 * reference's sum of little-endian 16-bit words modulo 0xffff; the final
 * value is re-expressed in the reference's 32-bit accumulator so that
 * ip_cksum_postprocess() sees an identical folded result, including the
 * all-zero case (0 stays 0, RFC 1071 "negative zero" never appears).
 */
#include <string.h>

#include "../../../include/ipcksum.h"

static uint32_t fold64_to32(uint64_t s)
{
  /* any non-zero value congruent mod 0xffff folds to the same 16 bits */
  s = (s & 0xffffffffu) + (s >> 32);
  s = (s & 0xffffffffu) + (s >> 32);
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  return (uint32_t)s;
}

void ip_cksum_feed(struct ip_cksum_ctx *ctx, const void *buf, size_t sz)
{
  const unsigned char *p = (const unsigned char *)buf;
  uint64_t acc = 0, w;
  /* 8 bytes per step: words 0 and 2 in one pass, words 1 and 3 in the
   * other; a carry out of bit 31 is worth 2^32 == 1 (mod 0xffff) */
  while (sz >= 8) {
    memcpy(&w, p, 8);
    acc += w & 0x0000ffff0000ffffull;
    acc += (w >> 16) & 0x0000ffff0000ffffull;
    p += 8;
    sz -= 8;
  }
  while (sz >= 2) {
    acc += hdr_get16h(p);
    p += 2;
    sz -= 2;
  }
  if (sz)
    acc += htons((uint16_t)(p[0] << 8));
  ctx->sum += fold64_to32(acc);
}

uint16_t ip_hdr_cksum_calc(const void *iphdr, uint16_t iplen)
{
  uint8_t ihl = ip_hdr_len(iphdr);
  struct ip_cksum_ctx c = IP_CKSUM_CTX_INITER;
  if (ihl > iplen)
    abort();
  ip_cksum_feed(&c, iphdr, ihl);
  return ip_cksum_postprocess(&c);
}

static uint16_t l4_v4(const void *iphdr, uint16_t iplen, const void *l4,
                      uint16_t l4len, uint8_t proto)
{
  struct ip_cksum_ctx c = IP_CKSUM_CTX_INITER;
  if (iplen < 20)
    abort();
  ip_cksum_feed32ptr(&c, ip_const_src_ptr(iphdr));
  ip_cksum_feed32ptr(&c, ip_const_dst_ptr(iphdr));
  ip_cksum_add16(&c, htons(proto));
  ip_cksum_add16(&c, htons(l4len));
  ip_cksum_feed(&c, l4, l4len);
  return ip_cksum_postprocess(&c);
}

static uint16_t l4_v6(const void *iphdr, uint16_t iplen, const void *l4,
                      uint16_t l4len, uint8_t proto)
{
  struct ip_cksum_ctx c = IP_CKSUM_CTX_INITER;
  uint32_t be;
  if (iplen < 40)
    abort();
  /* RFC 2460 pseudo-header from the fixed header (routing header ignored,
   * as in the reference, ipcksum.c:70-73) */
  ip_cksum_feed(&c, ipv6_const_src(iphdr), 16);
  ip_cksum_feed(&c, ipv6_const_dst(iphdr), 16);
  be = htonl(l4len);
  ip_cksum_feed32ptr(&c, &be);
  be = htonl(proto);
  ip_cksum_feed32ptr(&c, &be);
  ip_cksum_feed(&c, l4, l4len);
  return ip_cksum_postprocess(&c);
}

uint16_t tcp_cksum_calc(const void *iphdr, uint16_t iplen, const void *tcphdr, uint16_t tcplen)
{
  return l4_v4(iphdr, iplen, tcphdr, tcplen, 6);
}

uint16_t udp_cksum_calc(const void *iphdr, uint16_t iplen, const void *udphdr, uint16_t udplen)
{
  return l4_v4(iphdr, iplen, udphdr, udplen, 17);
}

uint16_t tcp6_cksum_calc(const void *iphdr, uint16_t iplen, const void *tcphdr, uint16_t tcplen)
{
  return l4_v6(iphdr, iplen, tcphdr, tcplen, 6);
}

uint16_t udp6_cksum_calc(const void *iphdr, uint16_t iplen, const void *udphdr, uint16_t udplen)
{
  return l4_v6(iphdr, iplen, udphdr, udplen, 17);
}
