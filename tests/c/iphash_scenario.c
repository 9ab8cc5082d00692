/* A rate-limiter scenario written against the iphash.h / timerlink.h /
 * hashseed.h API only, so the same source is built twice by
 * tests/test_capi.py: against include/ + libpptkrx.so (the kept API) and
 * against the reference's headers and objects in oracle/_ref (where the
 * reference tree exists).  Both runs must agree bit for bit.
 *
 * n sources (IPv4 host order in src4, or 16-byte IPv6 in src6) are offered
 * in chunks; after each chunk a virtual clock advances by period/3 and every
 * expired refill timer runs, as an application's timer loop would.  Every
 * 7th source is also given back (ip_increment_one).  The timers are re-timed
 * to a deterministic start (i * period / timercnt) instead of the wall clock
 * ip_hash_init uses. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hashseed.h"
#include "iphash.h"
#include "timerlink.h"

uint32_t iphash_scenario(const uint8_t *key, int family, uint8_t bits, const uint32_t *src4,
                         const uint8_t *src6, size_t n, uint32_t hash_size, uint32_t batch_size,
                         uint32_t initial, uint32_t timer_add, uint32_t period, size_t chunk,
                         uint8_t *verdict, uint32_t *tokens_out)
{
  struct timer_linkheap heap;
  struct ip_hash h;
  size_t i, start, tc = hash_size / batch_size;
  uint64_t clock = 0;
  uint32_t fired = 0;
  memcpy(hash_seed, key, 16);
  hash_seed_inited = 1;
  timer_linkheap_init(&heap);
  memset(&h, 0, sizeof(h));
  h.hash_size = hash_size;
  h.batch_size = batch_size;
  h.initial_tokens = initial;
  h.timer_add = timer_add;
  h.timer_period = period;
  ip_hash_init(&h, &heap, NULL);
  for (i = 0; i < tc; i++) {
    h.timers[i].time64 = (uint64_t)period * i / tc;
    timer_linkheap_modify(&heap, &h.timers[i]);
  }
  for (start = 0; start < n; start += chunk) {
    const size_t end = start + chunk < n ? start + chunk : n;
    for (i = start; i < end; i++) {
      if (family == 4) {
        verdict[i] = (uint8_t)ip_permitted(src4[i], bits, &h);
        if (i % 7 == 3)
          ip_increment_one(src4[i], bits, &h);
      } else {
        verdict[i] = (uint8_t)ipv6_permitted(src6 + 16 * i, bits, &h);
        if (i % 7 == 3)
          ipv6_increment_one(src6 + 16 * i, bits, &h);
      }
    }
    clock += period / 3;
    while (timer_linkheap_next_expiry_time(&heap) <= clock) {
      struct timer_link *t = timer_linkheap_next_expiry_timer(&heap);
      timer_linkheap_remove(&heap, t);
      t->fn(t, &heap, t->userdata, NULL);
      fired++;
    }
  }
  for (i = 0; i < hash_size; i++)
    tokens_out[i] = use_tiny(&h) ? h.u.entries_tiny[i].tokens
                    : use_small(&h) ? h.u.entries_small[i].tokens
                                    : h.u.entries[i].tokens;
  ip_hash_free(&h, &heap);
  timer_linkheap_free(&heap);
  return fired;
}

/* The timer heap alone: a seeded sequence of adds, removes (of random
 * members), time changes and pops; returns the popped times in order
 * (out, up to nout) and the count, -1 if a pop was not the minimum. */
long timer_heap_exercise(uint64_t seed, size_t ntimers, size_t nops, uint64_t *out, size_t nout)
{
  struct timer_linkheap heap;
  struct timer_link *t = calloc(ntimers, sizeof(*t));
  char *in = calloc(ntimers, 1);
  size_t k, npop = 0;
  uint64_t s = seed;
  timer_linkheap_init(&heap);
  for (k = 0; k < nops; k++) {
    size_t j;
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    j = (size_t)(s >> 33) % ntimers;
    switch ((s >> 20) % 4) {
    case 0:
    case 1:
      if (!in[j]) {
        t[j].time64 = (s >> 40) % 1000;
        timer_linkheap_add(&heap, &t[j]);
        in[j] = 1;
      }
      break;
    case 2:
      if (in[j]) {
        t[j].time64 = (s >> 40) % 1000;
        timer_linkheap_modify(&heap, &t[j]);
      }
      break;
    default:
      if (in[j]) {
        timer_linkheap_remove(&heap, &t[j]);
        in[j] = 0;
      }
    }
  }
  while (heap.root) {
    struct timer_link *r = timer_linkheap_next_expiry_timer(&heap);
    if (npop && npop <= nout && r->time64 < out[npop - 1]) {
      free(t);
      free(in);
      return -1;
    }
    if (npop < nout)
      out[npop] = r->time64;
    timer_linkheap_remove(&heap, r);
    npop++;
  }
  timer_linkheap_free(&heap);
  free(t);
  free(in);
  return (long)npop;
}

/* One ip_permitted / ipv6_permitted call per frame in frame order from the
 * given token state (tok_in), as the permit.npz fixture was made: frames
 * with use[i] == 0 are not subjects (verdict 2). */
void iphash_permit_seq(const uint8_t *key, int family, uint8_t bits, const uint32_t *src4,
                       const uint8_t *src6, const uint8_t *use, size_t n, uint32_t hash_size,
                       uint32_t initial, const uint32_t *tok_in, uint8_t *verdict,
                       uint32_t *tok_out)
{
  struct timer_linkheap heap;
  struct ip_hash h;
  size_t i;
  memcpy(hash_seed, key, 16);
  hash_seed_inited = 1;
  timer_linkheap_init(&heap);
  memset(&h, 0, sizeof(h));
  h.hash_size = hash_size;
  h.batch_size = hash_size;
  h.initial_tokens = initial;
  h.timer_period = 1000000;
  ip_hash_init(&h, &heap, NULL);
  for (i = 0; i < hash_size; i++) {
    if (use_tiny(&h)) h.u.entries_tiny[i].tokens = (uint8_t)tok_in[i];
    else if (use_small(&h)) h.u.entries_small[i].tokens = (uint16_t)tok_in[i];
    else h.u.entries[i].tokens = tok_in[i];
  }
  for (i = 0; i < n; i++) {
    if (!use[i]) {
      verdict[i] = 2;
      continue;
    }
    verdict[i] = (uint8_t)(family == 4 ? ip_permitted(src4[i], bits, &h)
                                       : ipv6_permitted(src6 + 16 * i, bits, &h));
  }
  for (i = 0; i < hash_size; i++)
    tok_out[i] = use_tiny(&h) ? h.u.entries_tiny[i].tokens
                 : use_small(&h) ? h.u.entries_small[i].tokens
                                 : h.u.entries[i].tokens;
  ip_hash_free(&h, &heap);
  timer_linkheap_free(&heap);
}
