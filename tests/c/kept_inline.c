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
                 uint32_t dst, uint16_t sport, uint16_t dport)
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
