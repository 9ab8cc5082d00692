/*
 * capi_dropin.c -- compiled by tests/test_capi.py with plain gcc against
 * include/ and linked to pptk_amd/libpptkrx.so, the way an LDP application
 * would use the library.  Checks the kept per-packet APIs against the
 * reference's known answers (iphdr/ipcksumtest.c, iphdr/iphdrtest.c,
 * misc/siphashtest.c) and the C-ABI error behaviour.  Exit 0 = pass.
 */
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include "hashseed.h"
#include "ipcksum.h"
#include "iphdr.h"
#include "pptk_rx.h"
#include "siphash.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

static uint16_t feed(const char *s, size_t n)
{
  struct ip_cksum_ctx c = IP_CKSUM_CTX_INITER;
  ip_cksum_feed(&c, s, n);
  return ip_cksum_postprocess(&c);
}

int main(int argc, char **argv)
{
  static const char tcp6[] = "\x60\x0\x0\x0\x0\x17\x6\x40\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x1\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x1\x0\x14\x0\x50\x0\x0\x0\x0\x0\x0\x0\x0\x50\x2\x20\x0\xba\xa\x0\x0\x66\x6f\x6f";
  static const char udp6[] = "\x60\x0\x0\x0\x0\xb\x11\x40\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x1\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x1\x0\x35\x0\x35\x0\xb\x29\xfd\x66\x6f\x6f";
  static const char ip4[] = "\x45\x0\x0\x14\x0\x1\x0\x0\x40\x0\x7c\xe7\x7f\x0\x0\x1\x7f\x0\x0\x1";
  static const char tcp4[] = "\x45\x00\x00\x2b\x00\x01\x00\x00\x40\x06\x7c\xca\x7f\x00\x00\x01\x7f\x00\x00\x01\x00\x14\x00\x50\x00\x00\x00\x00\x00\x00\x00\x00\x50\x02\x20\x00\xbc\x09\x00\x00\x66\x6f\x6f";
  static const char udp4[] = "\x45\x0\x0\x1f\x0\x1\x0\x0\x40\x11\x7c\xcb\x7f\x0\x0\x1\x7f\x0\x0\x1\x0\x35\x0\x35\x0\xb\x2b\xfc\x66\x6f\x6f";
  static const char frag6[] = "\x60\x0\x0\x0\x0\x1f\x2c\x40\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x1\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x0\x1\x6\x0\x0\x8\x0\x0\x0\x0\x0\x14\x0\x50\x0\x0\x0\x0\x0\x0\x0\x0\x50\x2\x20\x0\xba\xa\x0\x0\x66\x6f\x6f";
  const unsigned char z16[16] = {0};
  const unsigned char k[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  unsigned char msg[15];
  uint8_t proto = 0;
  int i;

  CHECK(feed("abcdef", 6) == 54738);
  CHECK(feed("abcdefg", 7) == 28370);
  CHECK(feed("abcdefghijklmnopqrstuvwxyz", 26) == 29028);
  CHECK(ip_hdr_cksum_calc(ip4, sizeof(ip4) - 1) == 0);
  CHECK(ip46_hdr_cksum_calc(ip4) == 0);
  CHECK(tcp_cksum_calc(tcp4, 20, tcp4 + 20, sizeof(tcp4) - 20 - 1) == 0);
  CHECK(udp_cksum_calc(udp4, 20, udp4 + 20, sizeof(udp4) - 20 - 1) == 0);
  CHECK(tcp6_cksum_calc(tcp6, 40, tcp6 + 40, sizeof(tcp6) - 40 - 1) == 0);
  CHECK(udp6_cksum_calc(udp6, 40, udp6 + 40, sizeof(udp6) - 40 - 1) == 0);
  CHECK(tcp46_cksum_calc(tcp4) == 0);
  CHECK(tcp46_cksum_calc(tcp6) == 0);
  CHECK(ip_version(tcp4) == 4 && ip_hdr_len(tcp4) == 20 && ip_total_len(tcp4) == 43);
  CHECK(ip_proto(tcp4) == 6 && ip_src(tcp4) == 0x7f000001 && tcp_dst_port(tcp4 + 20) == 80);
  CHECK(ipv6_payload_len(tcp6) == 23 && ip46_payload_len(tcp6) == 23);
  {
    const char *p = ipv6_const_proto_hdr(frag6, &proto);
    CHECK(p == frag6 + 40 && proto == 44 && ipv6_frag_off(p) == 8 && !ipv6_more_frags(p));
  }

  CHECK(siphash_buf(z16, z16, 16) == 0x32caecc280172976ULL);
  for (i = 0; i < 15; i++)
    msg[i] = (unsigned char)i;
  CHECK(siphash_buf(k, msg, 0) == 0x726fdb47dd0e0e31ULL);
  CHECK(siphash_buf(k, msg, 8) == 0x93f5f5799a932462ULL);
  CHECK(siphash_buf(k, msg, 15) == 0xa129ca6149be45e5ULL);
  CHECK(siphash64((const char *)k, hdr_get64h(msg)) == 0x93f5f5799a932462ULL);
  {
    struct siphash_ctx c;
    siphash_init(&c, k);
    siphash_feed_buf(&c, msg, 8);   /* non-spec form: extra tail block */
    CHECK(siphash_get(&c) == 0x49edd52a0ca45d7fULL);
  }

  CHECK(hash_seed_get() == NULL);
  hash_seed_init();
  CHECK(hash_seed_get() != NULL);

  {
    struct pptk_rx_opts o;
    struct pptk_rx_ctx *ctx = (struct pptk_rx_ctx *)1;
    pptk_rx_opts_default(&o);
    CHECK(memcmp(o.key, hash_seed, 16) == 0);
    CHECK(pptk_rx_ctx_create(NULL, &o) == -EINVAL);
    o.iphash_bits4 = 33;
    CHECK(pptk_rx_ctx_create(&ctx, &o) == -EINVAL && ctx == NULL);
    o.iphash_bits4 = 24;
    o.iphash_size = 1000;                    /* not a power of two */
    CHECK(pptk_rx_ctx_create(&ctx, &o) == -EINVAL);
    CHECK(pptk_rx_batch(NULL, NULL, 1, NULL) == -EINVAL);
    CHECK(pptk_rx_batch_device(NULL, NULL, NULL) == -EINVAL);
    CHECK(sizeof(struct pptk_rx_rec) == 64 && sizeof(struct ldp_packet) == 24);
    if (argc > 1 && strcmp(argv[1], "nogpu") == 0) {
      o.iphash_size = 1024;
      CHECK(pptk_rx_ctx_create(&ctx, &o) < 0);   /* no device: error, not abort */
    }
  }
  printf("capi_dropin ok (%s)\n", pptk_rx_version());
  return 0;
}
