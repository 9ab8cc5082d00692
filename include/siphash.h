/*
 * siphash.h -- SipHash-2-4, header-only, host side.
 *
 * Same API and results as the reference's misc/siphash.h:
 *   siphash_init / siphash_feed_u64 / siphash_get   (:25-121)
 *   siphash64(key, u64)                              (:123-130)
 *   siphash_feed_remaining                           (:132-172)
 *   siphash_feed_buf  -- the reference's NON-spec incremental form that
 *                        always feeds one extra tail block (:174-212)
 *   siphash_buf       -- spec-compliant SipHash-2-4 (:214-229)
 * The GPU computes the flow hash of pptk_rx_rec with siphash_buf semantics.
 */
#ifndef _SIPHASH_H_
#define _SIPHASH_H_

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "hdr.h"

#define cROUNDS 2
#define dROUNDS 4

struct siphash_ctx {
  uint64_t v0;
  uint64_t v1;
  uint64_t v2;
  uint64_t v3;
  uint64_t inlen;
  uint64_t b;
};

static inline uint64_t pptk_rotl64(uint64_t x, unsigned b)
{
  return (x << b) | (x >> (64 - b));
}

static inline void pptk_sipround(struct siphash_ctx *c)
{
  c->v0 += c->v1; c->v1 = pptk_rotl64(c->v1, 13); c->v1 ^= c->v0; c->v0 = pptk_rotl64(c->v0, 32);
  c->v2 += c->v3; c->v3 = pptk_rotl64(c->v3, 16); c->v3 ^= c->v2;
  c->v0 += c->v3; c->v3 = pptk_rotl64(c->v3, 21); c->v3 ^= c->v0;
  c->v2 += c->v1; c->v1 = pptk_rotl64(c->v1, 17); c->v1 ^= c->v2; c->v2 = pptk_rotl64(c->v2, 32);
}

static inline void siphash_init(struct siphash_ctx *ctx, const void *k)
{
  const uint64_t k0 = hdr_get64h(k);
  const uint64_t k1 = hdr_get64h((const unsigned char *)k + 8);
  ctx->v0 = 0x736f6d6570736575ULL ^ k0;
  ctx->v1 = 0x646f72616e646f6dULL ^ k1;
  ctx->v2 = 0x6c7967656e657261ULL ^ k0;
  ctx->v3 = 0x7465646279746573ULL ^ k1;
  ctx->inlen = 0;
  ctx->b = 0;
}

static inline void siphash_feed_u64(struct siphash_ctx *ctx, uint64_t in)
{
  int r;
  ctx->v3 ^= in;
  for (r = 0; r < cROUNDS; r++)
    pptk_sipround(ctx);
  ctx->v0 ^= in;
  ctx->inlen += 8;
}

static inline uint64_t siphash_get(struct siphash_ctx *ctx)
{
  int r;
  const uint64_t last = ctx->b | (ctx->inlen << 56);
  ctx->b = last;
  ctx->v3 ^= last;
  for (r = 0; r < cROUNDS; r++)
    pptk_sipround(ctx);
  ctx->v0 ^= last;
  ctx->v2 ^= 0xff;
  for (r = 0; r < dROUNDS; r++)
    pptk_sipround(ctx);
  return ctx->v0 ^ ctx->v1 ^ ctx->v2 ^ ctx->v3;
}

static inline uint64_t siphash64(const char key[16], uint64_t val64)
{
  struct siphash_ctx ctx;
  siphash_init(&ctx, key);
  siphash_feed_u64(&ctx, val64);
  return siphash_get(&ctx);
}

static inline uint64_t pptk_sip_tail(const unsigned char *in, size_t n)
{
  uint64_t b = 0;
  while (n--)
    b = (b << 8) | in[n];
  return b;
}

static inline void siphash_feed_remaining(struct siphash_ctx *ctx, const void *buf,
                                          size_t remaining)
{
  if (remaining >= 8 || ctx->b != 0)
    abort();
  ctx->b = pptk_sip_tail((const unsigned char *)buf, remaining);
  ctx->inlen += remaining;
}

static inline void siphash_feed_buf(struct siphash_ctx *ctx, const void *buf, size_t buflen)
{
  const unsigned char *p = (const unsigned char *)buf;
  for (; buflen >= 8; p += 8, buflen -= 8)
    siphash_feed_u64(ctx, hdr_get64h(p));
  siphash_feed_u64(ctx, pptk_sip_tail(p, buflen));
}

static inline uint64_t siphash_buf(const void *key, const void *buf, size_t buflen)
{
  struct siphash_ctx ctx;
  const unsigned char *p = (const unsigned char *)buf;
  siphash_init(&ctx, key);
  for (; buflen >= 8; p += 8, buflen -= 8)
    siphash_feed_u64(&ctx, hdr_get64h(p));
  siphash_feed_remaining(&ctx, p, buflen);
  return siphash_get(&ctx);
}

#endif
