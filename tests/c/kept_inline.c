/* Wraps the kept inline APIs of include/ipcksum.h (tx setters, incremental
 * updates) as exported functions, so tests/test_capi.py can compare them
 * with the reference's (oracle/_ref) through ctypes.  Built by the test. */
#include <stdint.h>

#include "ipcksum.h"

uint16_t kept_update16(uint16_t c, uint16_t o, uint16_t n) { return ip_update_cksum16(c, o, n); }
uint16_t kept_update32(uint16_t c, uint32_t o, uint32_t n) { return (uint16_t)ip_update_cksum32(c, o, n); }

/* one frame: ops as pptk_rewrite (bit 0 ttl, 1 src, 2 dst, 3 sport, 4 dport)
 * applied with the kept inline functions; ip/l4 offsets and proto given */
int kept_rewrite(uint8_t *f, int l3, int l4, int proto, int l4ok, uint32_t ops, uint32_t src,
                 uint32_t dst, uint16_t sport, uint16_t dport, int l4len, int frag)
{
  uint8_t *ip = f + l3, *p = f + l4;
  int alive = 1;
  if (ops & 1)
    alive = ip_decr_ttl_cksum_update(ip);
  if (ops & 2)
    ip_set_src_cksum_update(ip, ip_hdr_len(ip), (uint8_t)(l4ok ? proto : 0), p, 0, src);
  if (ops & 4)
    ip_set_dst_cksum_update(ip, ip_hdr_len(ip), (uint8_t)(l4ok ? proto : 0), p, 0, dst);
  if (l4ok && (ops & 8)) {
    if (proto == 6) tcp_set_src_port_cksum_update(p, 0, sport);
    else udp_set_src_port_cksum_update(p, 0, sport);
  }
  if (l4ok && (ops & 16)) {
    if (proto == 6) tcp_set_dst_port_cksum_update(p, 0, dport);
    else udp_set_dst_port_cksum_update(p, 0, dport);
  }
  /* bit 5: ICMP echo identifier (the new id in sport) */
  if ((ops & 32) && proto == 1 && !frag && l4len >= 8 && (icmp_type(p) == 8 || icmp_type(p) == 0))
    icmp_set_echo_identifier_cksum_update(p, (uint16_t)l4len, sport);
  return alive;
}

/* the tx setters on one IPv4/IPv6 frame */
void kept_set_cksums(uint8_t *f, int l3, int l4, int v6, int proto, int l4ok, uint16_t l4len)
{
  uint8_t *ip = f + l3, *p = f + l4;
  if (!v6)
    ip_set_hdr_cksum_calc(ip, ip_hdr_len(ip));
  if (!l4ok)
    return;
  if (v6) {
    if (proto == 6) tcp6_set_cksum_calc(ip, 40, p, l4len);
    else udp6_set_cksum_calc(ip, 40, p, l4len);
  } else {
    if (proto == 6) tcp_set_cksum_calc(ip, ip_hdr_len(ip), p, l4len);
    else udp_set_cksum_calc(ip, ip_hdr_len(ip), p, l4len);
  }
}

/* The kept TCP option API (include/iphdr.h walks, include/ipcksum.h option
 * rewrites), packed exactly as oracle/refgen.c's ref_tcp_* wrappers pack the
 * reference's results, so the two compare field for field. */
uint32_t kept_tcp_parse_options(uint8_t *t, uint16_t *mss, uint32_t *ts, uint32_t *tsecho)
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

uint32_t kept_tcp_find_sack_ts(uint8_t *t)
{
  struct sack_ts_headers h;
  tcp_find_sack_ts_headers(t, &h);
  return (uint32_t)h.sackoff | ((uint32_t)h.sacklen << 8) | ((uint32_t)h.tsoff << 16);
}

int64_t kept_tcp_find_sack(uint8_t *t, uint32_t *sacklen, int *align)
{
  size_t l = 0;
  uint8_t *p = tcp_find_sack_header(t, &l, align);
  *sacklen = (uint32_t)l;
  return p ? (int64_t)(p - t) : -1;
}

void kept_tcp_opt_op(uint8_t *t, int op, uint32_t v)
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
