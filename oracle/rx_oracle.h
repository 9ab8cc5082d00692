/*
 * rx_oracle.h -- TEST INFRASTRUCTURE ONLY (see rx_oracle.c).  CPU
 * restatement of the PPTK rx transform used as parity checker and as the
 * "port" CPU baseline.  Never linked into pptk_amd/.
 */
#ifndef RX_ORACLE_H
#define RX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/pptk_rx.h"

struct orc_opts {
  uint8_t key[16];
  uint8_t bits4;      /* 0 = no IPv4 bucket */
  uint8_t bits6;      /* 0 = no IPv6 bucket */
  uint16_t pad;
  uint32_t hash_size; /* power of two */
};

uint32_t orc_sum_feed(uint32_t sum, const uint8_t *buf, size_t sz);
uint16_t orc_finish(uint32_t sum);
uint16_t orc_cksum_buf(const uint8_t *buf, size_t sz);
uint16_t orc_ip_hdr_cksum(const uint8_t *ip);
uint16_t orc_l4_cksum_v4(const uint8_t *ip, const uint8_t *l4, uint16_t l4len,
                         uint8_t proto);
uint16_t orc_l4_cksum_v6(const uint8_t *ip, const uint8_t *l4, uint16_t l4len,
                         uint8_t proto);
int orc_v6_walk(const uint8_t *ip6, uint8_t *proto, int *fragmented,
                uint16_t *l4off, int *walked);
uint64_t orc_siphash(const uint8_t key[16], const uint8_t *msg, size_t len);
uint64_t orc_siphash64(const uint8_t key[16], uint64_t val);
uint32_t orc_ip_bucket(const uint8_t key[16], uint32_t src_host, uint8_t bits,
                       uint32_t hash_size);
uint32_t orc_ipv6_bucket(const uint8_t key[16], const uint8_t src[16],
                         uint8_t bits, uint32_t hash_size);
void orc_rx_one(const uint8_t *frame, uint32_t len, const struct orc_opts *o,
                struct pptk_rx_rec *rec);
int orc_rx_batch(const uint8_t *buf, const uint64_t *off, const uint16_t *len,
                 uint64_t stride, uint32_t fixed_len, size_t n,
                 const struct orc_opts *o, struct pptk_rx_rec *recs,
                 int nthreads);
void orc_frag_one(const uint8_t *frame, uint32_t len, struct pptk_rx_frag *fr);
void orc_frag_batch(const uint8_t *buf, const uint64_t *off, const uint16_t *len,
                    uint64_t stride, uint32_t fixed_len, size_t n, struct pptk_rx_frag *out);
uint32_t orc_cksum_loop(const uint8_t *buf, size_t sz, uint64_t iters);
void orc_permit_batch(const struct pptk_rx_rec *recs, size_t n, int family,
                      const uint8_t *subject, uint32_t *tokens, uint8_t *verdict);
void orc_tx_batch(uint8_t *buf, const uint64_t *off, const uint16_t *len, uint64_t stride,
                  uint32_t fixed_len, size_t n);
void orc_tokens_refill(uint32_t *tokens, uint32_t start, uint32_t end,
                       uint32_t add, uint32_t initial);
uint16_t orc_update_cksum16(uint16_t cksum, uint16_t old16, uint16_t new16);
uint16_t orc_update_cksum32(uint16_t cksum, uint32_t old32, uint32_t new32);
void orc_rewrite_batch(uint8_t *buf, const uint64_t *off, const uint16_t *len, uint64_t stride,
                       uint32_t fixed_len, size_t n, const struct pptk_rewrite *rw,
                       uint64_t rw_count, uint8_t *status);
void orc_mss_clamp_batch(uint8_t *buf, const uint64_t *off, const uint16_t *len, uint64_t stride,
                         uint32_t fixed_len, size_t n, uint16_t mss, uint32_t flags,
                         uint8_t *status);

#endif
