/*
 * iphdr.h -- fixed-format Ethernet / IPv4 / IPv6 / TCP / UDP field access.
 *
 * The subset of the reference's iphdr/iphdr.h that the receive transform
 * reads, with the same names, argument
 * meaning and results: multi-byte fields come back in host order, pointer
 * accessors point into the frame.  Reference line numbers are given per
 * group.  Like the reference, the ip46_* dispatchers abort() on a version
 * that is neither 4 nor 6 (a caller contract violation).
 */
#ifndef _IPHDR_H_
#define _IPHDR_H_

#include <stdint.h>
#include <stdlib.h>

#include "hdr.h"

#define ETHER_HDR_LEN 14U
#define ETHER_TYPE_IP ((uint16_t)0x0800)
#define ETHER_TYPE_ARP ((uint16_t)0x0806)
#define ETHER_TYPE_IPV6 ((uint16_t)0x86DD)
#define IP_HDR_MINLEN 20U

#define PPTK_AT(p, k) ((const unsigned char *)(p) + (k))

/* ---- Ethernet: iphdr.h:379-431 */
static inline const void *ether_const_dst(const void *pkt) { return PPTK_AT(pkt, 0); }
static inline const void *ether_const_src(const void *pkt) { return PPTK_AT(pkt, 6); }
static inline uint16_t ether_type(const void *pkt) { return hdr_get16n(PPTK_AT(pkt, 12)); }
static inline const void *ether_const_payload(const void *pkt) { return PPTK_AT(pkt, ETHER_HDR_LEN); }
static inline void *ether_payload(void *pkt) { return (unsigned char *)pkt + ETHER_HDR_LEN; }

/* ---- IPv4: iphdr.h:435, 876, 943, 1023, 1124, 1145, 1171, 1247, 1259-1296 */
static inline uint8_t ip_version(const void *pkt) { return *PPTK_AT(pkt, 0) >> 4; }
static inline uint8_t ip_hdr_len(const void *pkt) { return (uint8_t)((*PPTK_AT(pkt, 0) & 0x0f) << 2); }
static inline uint16_t ip_total_len(const void *pkt) { return hdr_get16n(PPTK_AT(pkt, 2)); }
static inline uint16_t ip_id(const void *pkt) { return hdr_get16n(PPTK_AT(pkt, 4)); }
static inline int ip_more_frags(const void *pkt) { return *PPTK_AT(pkt, 6) & 0x20; }
static inline int ip_dont_frag(const void *pkt) { return *PPTK_AT(pkt, 6) & 0x40; }
static inline uint16_t ip_frag_off(const void *pkt)
{
  return (uint16_t)((hdr_get16n(PPTK_AT(pkt, 6)) & 0x1fff) << 3);
}
static inline uint8_t ip_ttl(const void *pkt) { return *PPTK_AT(pkt, 8); }
static inline uint8_t ip_proto(const void *pkt) { return *PPTK_AT(pkt, 9); }
static inline uint16_t ip_hdr_cksum(const void *pkt) { return hdr_get16n(PPTK_AT(pkt, 10)); }
static inline uint32_t ip_src(const void *pkt) { return hdr_get32n(PPTK_AT(pkt, 12)); }
static inline uint32_t ip_dst(const void *pkt) { return hdr_get32n(PPTK_AT(pkt, 16)); }
static inline const void *ip_const_src_ptr(const void *pkt) { return PPTK_AT(pkt, 12); }
static inline const void *ip_const_dst_ptr(const void *pkt) { return PPTK_AT(pkt, 16); }
static inline const void *ip_const_payload(const void *pkt) { return PPTK_AT(pkt, ip_hdr_len(pkt)); }

/* ---- IPv6 fixed header: iphdr.h:527-579 */
static inline uint16_t ipv6_payload_len(const void *pkt) { return hdr_get16n(PPTK_AT(pkt, 4)); }
static inline uint8_t ipv6_nexthdr(const void *pkt) { return *PPTK_AT(pkt, 6); }
static inline uint8_t ipv6_hop_limit(const void *pkt) { return *PPTK_AT(pkt, 7); }
static inline const void *ipv6_const_src(const void *pkt) { return PPTK_AT(pkt, 8); }
static inline const void *ipv6_const_dst(const void *pkt) { return PPTK_AT(pkt, 24); }
static inline const void *ipv6_nexthdr_const_ptr(const void *pkt) { return PPTK_AT(pkt, 40); }

/* ---- v4/v6 dispatch: iphdr.h:670-700, 882-893, 991-1021, 1177-1191, 1298 */
static inline int pptk_ipver_or_die(const void *pkt)
{
  int v = ip_version(pkt);
  if (v != 4 && v != 6)
    abort();
  return v;
}
static inline uint8_t ip46_hdr_len(const void *pkt)
{
  return pptk_ipver_or_die(pkt) == 4 ? ip_hdr_len(pkt) : 40;
}
static inline uint16_t ip46_total_len(const void *pkt)
{
  return pptk_ipver_or_die(pkt) == 4 ? ip_total_len(pkt)
                                     : (uint16_t)(ipv6_payload_len(pkt) + 40);
}
static inline uint16_t ip46_payload_len(const void *pkt)
{
  return pptk_ipver_or_die(pkt) == 4 ? (uint16_t)(ip_total_len(pkt) - ip_hdr_len(pkt))
                                     : ipv6_payload_len(pkt);
}
static inline uint8_t ip46_proto(const void *pkt)
{
  return pptk_ipver_or_die(pkt) == 4 ? ip_proto(pkt) : ipv6_nexthdr(pkt);
}
static inline const void *ip46_const_payload(const void *pkt)
{
  return PPTK_AT(pkt, ip46_hdr_len(pkt));
}
static inline const void *ip46_const_src(const void *pkt)
{
  return pptk_ipver_or_die(pkt) == 4 ? ip_const_src_ptr(pkt) : ipv6_const_src(pkt);
}
static inline const void *ip46_const_dst(const void *pkt)
{
  return pptk_ipver_or_die(pkt) == 4 ? ip_const_dst_ptr(pkt) : ipv6_const_dst(pkt);
}

/* ---- IPv6 extension headers: iphdr.h:702-737, 804-865.  The walk keeps
 * the reference's exact behaviour, including deriving the length of the
 * header at `off` from the type of the header that follows it. */
static inline uint32_t ipv6_extlen(uint8_t nexthdr, uint8_t lenfield)
{
  switch (nexthdr) {
  case 44: return 8;
  case 51: return (uint32_t)lenfield * 4 + 8;
  default: return (uint32_t)lenfield * 8 + 8;
  }
}
static inline int is_ipv6_nexthdr(uint8_t nh)
{
  switch (nh) {
  case 0: case 43: case 44: case 51: case 60: return 1;
  default: return 0;
  }
}
static inline uint16_t ipv6_frag_off(const void *frag) { return hdr_get16n(PPTK_AT(frag, 2)) & 0xfff8; }
static inline uint16_t ipv6_more_frags(const void *frag) { return hdr_get16n(PPTK_AT(frag, 2)) & 1; }

static inline const void *ipv6_const_proto_hdr_2(
  const void *ipv6, uint8_t *proto, int *is_fragmented_ptr,
  uint16_t *frag_hdr_off_ptr, uint16_t *proto_hdr_off_from_frag)
{
  const unsigned char *b = (const unsigned char *)ipv6;
  const uint32_t tlen = (uint32_t)ipv6_payload_len(ipv6) + 40u;
  uint16_t off = 40, frag_at = 0;
  uint8_t nh = ipv6_nexthdr(ipv6);
  int fragmented = 0;
  for (; is_ipv6_nexthdr(nh);) {
    uint32_t step;
    if (off + 8u > tlen)
      return NULL;
    if (nh == 44) {
      fragmented = 1;
      frag_at = off;
      if (ipv6_frag_off(b + off))
        break;
    }
    nh = b[off];
    step = ipv6_extlen(nh, b[off + 1]);
    if (off + step > tlen)
      return NULL;
    off = (uint16_t)(off + step);
  }
  if (proto)
    *proto = nh;
  if (is_fragmented_ptr)
    *is_fragmented_ptr = fragmented;
  if (fragmented) {
    if (frag_hdr_off_ptr)
      *frag_hdr_off_ptr = frag_at;
    if (proto_hdr_off_from_frag)
      *proto_hdr_off_from_frag = (uint16_t)(off - frag_at);
  }
  return b + off;
}
static inline const void *ipv6_const_proto_hdr(const void *ipv6, uint8_t *proto)
{
  return ipv6_const_proto_hdr_2(ipv6, proto, NULL, NULL, NULL);
}

/* ---- TCP / UDP: iphdr.h:1303-1313, 1381-1403, 1417-1433, 1491-1495 */
static inline uint16_t tcp_src_port(const void *l4) { return hdr_get16n(PPTK_AT(l4, 0)); }
static inline uint16_t tcp_dst_port(const void *l4) { return hdr_get16n(PPTK_AT(l4, 2)); }
static inline uint16_t tcp_cksum(const void *l4) { return hdr_get16n(PPTK_AT(l4, 16)); }
static inline uint8_t tcp_data_offset(const void *l4) { return (uint8_t)((*PPTK_AT(l4, 12) >> 4) << 2); }
static inline uint16_t udp_src_port(const void *l4) { return hdr_get16n(PPTK_AT(l4, 0)); }
static inline uint16_t udp_dst_port(const void *l4) { return hdr_get16n(PPTK_AT(l4, 2)); }
static inline uint16_t udp_total_len(const void *l4) { return hdr_get16n(PPTK_AT(l4, 4)); }
static inline uint16_t udp_cksum(const void *l4) { return hdr_get16n(PPTK_AT(l4, 6)); }

/* ---- setters used by the tx side and the incremental updates:
 * iphdr.h:1152-1156 (ttl), 1253-1257 (hdr cksum), 1271-1281 (src/dst),
 * 1315-1325, 1387-1391 (tcp), 1405-1415, 1435-1439 (udp); host-order values
 * stored big-endian. */
#define PPTK_W(p, k) ((unsigned char *)(p) + (k))
static inline void ip_set_ttl(void *pkt, uint8_t ttl) { *PPTK_W(pkt, 8) = ttl; }
static inline void ip_set_hdr_cksum(void *pkt, uint16_t c) { hdr_set16n(PPTK_W(pkt, 10), c); }
static inline void ip_set_src(void *pkt, uint32_t src) { hdr_set32n(PPTK_W(pkt, 12), src); }
static inline void ip_set_dst(void *pkt, uint32_t dst) { hdr_set32n(PPTK_W(pkt, 16), dst); }
static inline void tcp_set_src_port(void *l4, uint16_t p) { hdr_set16n(PPTK_W(l4, 0), p); }
static inline void tcp_set_dst_port(void *l4, uint16_t p) { hdr_set16n(PPTK_W(l4, 2), p); }
static inline void tcp_set_cksum(void *l4, uint16_t c) { hdr_set16n(PPTK_W(l4, 16), c); }
static inline void udp_set_src_port(void *l4, uint16_t p) { hdr_set16n(PPTK_W(l4, 0), p); }
static inline void udp_set_dst_port(void *l4, uint16_t p) { hdr_set16n(PPTK_W(l4, 2), p); }
static inline void udp_set_cksum(void *l4, uint16_t c) { hdr_set16n(PPTK_W(l4, 6), c); }

/* ---- TCP flags, sequence space, window: iphdr.h:1327-1379, 1441-1489.
 * tcp_set_data_offset abort()s on a value that is not a multiple of 4 or
 * exceeds 60, as the reference does (a caller contract violation). */
static inline int tcp_ack(const void *l4) { return !!(*PPTK_AT(l4, 13) & 0x10); }
static inline int tcp_rst(const void *l4) { return !!(*PPTK_AT(l4, 13) & 0x04); }
static inline int tcp_syn(const void *l4) { return !!(*PPTK_AT(l4, 13) & 0x02); }
static inline int tcp_fin(const void *l4) { return !!(*PPTK_AT(l4, 13) & 0x01); }
static inline void tcp_set_ack_on(void *l4) { *PPTK_W(l4, 13) |= 0x10; }
static inline void tcp_set_ack_off(void *l4) { *PPTK_W(l4, 13) &= (unsigned char)~0x10; }
static inline void tcp_set_rst_on(void *l4) { *PPTK_W(l4, 13) |= 0x04; }
static inline void tcp_set_syn_on(void *l4) { *PPTK_W(l4, 13) |= 0x02; }
static inline void tcp_set_fin_on(void *l4) { *PPTK_W(l4, 13) |= 0x01; }
static inline uint32_t tcp_seq_number(const void *l4) { return hdr_get32n(PPTK_AT(l4, 4)); }
static inline uint32_t tcp_ack_number(const void *l4) { return hdr_get32n(PPTK_AT(l4, 8)); }
static inline void tcp_set_seq_number(void *l4, uint32_t v) { hdr_set32n(PPTK_W(l4, 4), v); }
static inline void tcp_set_ack_number(void *l4, uint32_t v) { hdr_set32n(PPTK_W(l4, 8), v); }
static inline uint16_t tcp_window(const void *l4) { return hdr_get16n(PPTK_AT(l4, 14)); }
static inline void tcp_set_window(void *l4, uint16_t v) { hdr_set16n(PPTK_W(l4, 14), v); }
static inline void tcp_set_data_offset(void *l4, uint8_t data_off)
{
  if (data_off % 4 != 0 || data_off > 60)
    abort();
  *PPTK_W(l4, 12) = (unsigned char)((*PPTK_AT(l4, 12) & 0x0f) | ((data_off / 4) << 4));
}

/* ---- ICMP echo fields: iphdr.h:197-250 */
static inline uint8_t icmp_type(const void *l4) { return *PPTK_AT(l4, 0); }
static inline uint8_t icmp_code(const void *l4) { return *PPTK_AT(l4, 1); }
static inline uint16_t icmp_checksum(const void *l4) { return hdr_get16n(PPTK_AT(l4, 2)); }
static inline uint32_t icmp_header_data(const void *l4) { return hdr_get32n(PPTK_AT(l4, 4)); }
static inline uint16_t icmp_echo_identifier(const void *l4) { return hdr_get16n(PPTK_AT(l4, 4)); }
static inline void icmp_set_type(void *l4, uint8_t v) { *PPTK_W(l4, 0) = v; }
static inline void icmp_set_code(void *l4, uint8_t v) { *PPTK_W(l4, 1) = v; }
static inline void icmp_set_checksum(void *l4, uint16_t v) { hdr_set16n(PPTK_W(l4, 2), v); }
static inline void icmp_set_header_data(void *l4, uint32_t v) { hdr_set32n(PPTK_W(l4, 4), v); }
static inline void icmp_set_echo_identifier(void *l4, uint16_t v) { hdr_set16n(PPTK_W(l4, 4), v); }

/* ---- TCP options: iphdr.h:1497-1545, iphdr/iphdr.c:4-246.  Offsets are
 * from the start of the TCP header; the walks read bytes [20, data offset)
 * of it (pptk_amd/csrc/host/tcpopt.c). */
struct sack_ts_headers {
  uint8_t sackoff;   /* SACK option (kind 5), 0 = none */
  uint8_t sacklen;
  uint8_t tsoff;     /* timestamp option (kind 8, length 10), 0 = none */
};

struct tcp_information {
  uint8_t options_valid;
  uint8_t wscale;
  uint16_t mss;      /* 536 unless an MSS option is present */
  uint8_t sack_permitted;
  uint8_t mssoff;    /* from the beginning of the TCP header, 0 = none */
  uint8_t ts_present;
  uint32_t ts;
  uint32_t tsecho;
};

void tcp_parse_options(void *pkt, struct tcp_information *info);
void tcp_find_sack_ts_headers(void *pkt, struct sack_ts_headers *hdrs);
void *tcp_find_sack_header(void *pkt, size_t *sacklen, int *sixteen_bit_align);

static inline uint32_t tcp_tsval(const void *l4, struct sack_ts_headers *hdrs)
{
  if (hdrs->tsoff < 20)
    abort();
  return hdr_get32n(PPTK_AT(l4, hdrs->tsoff + 2));
}

static inline uint32_t tcp_tsecho(const void *l4, struct sack_ts_headers *hdrs)
{
  if (hdrs->tsoff < 20)
    abort();
  return hdr_get32n(PPTK_AT(l4, hdrs->tsoff + 6));
}

#endif
