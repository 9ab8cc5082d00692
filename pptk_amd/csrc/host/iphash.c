/*
 * iphash.c -- the kept per-packet rate limiter of include/iphash.h (the
 * reference's iphash/iphash.c:1-350, same results).  The three entry widths
 * are handled by one accessor pair instead of three copies of each
 * function; the bucket of a source is the reference's: SipHash-2-4 under
 * hash_seed_get() of the masked IPv4 address (siphash64, host order) or of
 * the 16 masked IPv6 bytes (siphash_buf), reduced mod hash_size.
 */
#include <stdlib.h>
#include <string.h>

#include "hashseed.h"
#include "iphash.h"
#include "siphash.h"

struct batch_timer_userdata {
  struct ip_hash *hash;
  pthread_rwlock_t *lock;
  size_t start;
  size_t end;
};

static int power_of_2(size_t x) { return x > 0 && (x & (x - 1)) == 0; }

static void check_sizes(const struct ip_hash *hash)
{
  if (!power_of_2(hash->hash_size) || !power_of_2(hash->batch_size) ||
      hash->hash_size < hash->batch_size)
    abort();
}

/* gettimeofday in microseconds (the reference's misc/time64.h clock) */
static uint64_t now64(void)
{
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return (uint64_t)tv.tv_sec * 1000000ull + (uint64_t)tv.tv_usec;
}

static uint32_t get_tokens(struct ip_hash *h, size_t i)
{
  if (use_tiny(h))
    return h->u.entries_tiny[i].tokens;
  if (use_small(h))
    return h->u.entries_small[i].tokens;
  return h->u.entries[i].tokens;
}

static void set_tokens(struct ip_hash *h, size_t i, uint32_t v)
{
  if (use_tiny(h))
    h->u.entries_tiny[i].tokens = (uint8_t)v;
  else if (use_small(h))
    h->u.entries_small[i].tokens = (uint16_t)v;
  else
    h->u.entries[i].tokens = v;
}

/* iphash.c:290-350: refill this timer's buckets, re-arm one period later */
static void batch_timer_fn(struct timer_link *timer, struct timer_linkheap *heap, void *ud,
                           void *td)
{
  struct batch_timer_userdata *args = (struct batch_timer_userdata *)ud;
  struct ip_hash *h = args->hash;
  size_t i;
  (void)td;
  if (args->lock)
    pthread_rwlock_wrlock(args->lock);
  for (i = args->start; i < args->end; i++) {
    uint32_t t = get_tokens(h, i) + h->timer_add;
    set_tokens(h, i, t >= h->initial_tokens ? h->initial_tokens : t);
  }
  timer->time64 += h->timer_period;
  timer_linkheap_add(heap, timer);
  if (args->lock)
    pthread_rwlock_unlock(args->lock);
}

/* iphash.c:25-75: timers spread evenly over one period, full buckets */
void ip_hash_init(struct ip_hash *hash, struct timer_linkheap *heap, pthread_rwlock_t *lock)
{
  size_t i, timercnt;
  check_sizes(hash);
  timercnt = hash->hash_size / hash->batch_size;
  hash->timers = (struct timer_link *)malloc(timercnt * sizeof(*hash->timers));
  hash->timerud = (struct batch_timer_userdata *)malloc(timercnt * sizeof(*hash->timerud));
  if (!hash->timers || !hash->timerud)
    abort();
  for (i = 0; i < timercnt; i++) {
    hash->timerud[i].hash = hash;
    hash->timerud[i].start = (size_t)hash->batch_size * i;
    hash->timerud[i].end = (size_t)hash->batch_size * (i + 1);
    hash->timerud[i].lock = lock;
    hash->timers[i].fn = batch_timer_fn;
    hash->timers[i].userdata = &hash->timerud[i];
    hash->timers[i].time64 = now64() + (uint64_t)hash->timer_period * i / timercnt;
    timer_linkheap_add(heap, &hash->timers[i]);
  }
  if (use_tiny(hash))
    hash->u.entries_tiny = malloc(hash->hash_size * sizeof(*hash->u.entries_tiny));
  else if (use_small(hash))
    hash->u.entries_small = malloc(hash->hash_size * sizeof(*hash->u.entries_small));
  else
    hash->u.entries = malloc(hash->hash_size * sizeof(*hash->u.entries));
  if (!hash->u.entries)
    abort();
  for (i = 0; i < hash->hash_size; i++)
    set_tokens(hash, i, hash->initial_tokens);
}

/* iphash.c:77-106 */
void ip_hash_free(struct ip_hash *hash, struct timer_linkheap *heap)
{
  size_t i, timercnt;
  check_sizes(hash);
  timercnt = hash->hash_size / hash->batch_size;
  for (i = 0; i < timercnt; i++)
    timer_linkheap_remove(heap, &hash->timers[i]);
  free(hash->timerud);
  free(hash->timers);
  free(hash->u.entries);   /* the union's one allocation, whatever its width */
}

/* bucket of an IPv4 source: its /bits network, host order (iphash.c:160-162) */
static uint32_t bucket4(uint32_t src_ip, uint8_t bits, const struct ip_hash *hash)
{
  const uint32_t mask = ~((1u << (32 - bits)) - 1u);
  return (uint32_t)siphash64((const char *)hash_seed_get(), src_ip & mask) &
         (hash->hash_size - 1);
}

/* bucket of an IPv6 source: the 16 bytes with the host bits cleared
 * (iphash.c:111-120) */
static uint32_t bucket6(const void *src_ip, uint8_t bits, const struct ip_hash *hash)
{
  uint8_t net[16];
  const size_t zero = (128u - bits) / 8;
  const int partial = (128u - bits) % 8;
  memcpy(net, src_ip, 16);
  memset(net + 16 - zero, 0, zero);
  net[16 - zero - 1] &= (uint8_t)~((1u << partial) - 1u);
  return (uint32_t)siphash_buf((const char *)hash_seed_get(), net, 16) & (hash->hash_size - 1);
}

static int take(struct ip_hash *hash, uint32_t b)
{
  const uint32_t t = get_tokens(hash, b);
  if (t == 0)
    return 0;
  set_tokens(hash, b, t - 1);
  return 1;
}

static void give(struct ip_hash *hash, uint32_t b)
{
  const uint32_t t = get_tokens(hash, b);
  if (t < hash->initial_tokens)
    set_tokens(hash, b, t + 1);
}

int ip_permitted(uint32_t src_ip, uint8_t bits, struct ip_hash *hash)
{
  return take(hash, bucket4(src_ip, bits, hash));
}

int ipv6_permitted(const void *src_ip, uint8_t bits, struct ip_hash *hash)
{
  return take(hash, bucket6(src_ip, bits, hash));
}

void ip_increment_one(uint32_t src_ip, uint8_t bits, struct ip_hash *hash)
{
  give(hash, bucket4(src_ip, bits, hash));
}

void ipv6_increment_one(const void *src_ip, uint8_t bits, struct ip_hash *hash)
{
  give(hash, bucket6(src_ip, bits, hash));
}
