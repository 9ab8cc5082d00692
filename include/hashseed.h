/*
 * hashseed.h -- process-wide 16-byte SipHash key.
 * Same API as the reference's misc/hashseed.h:6-18 / misc/hashseed.c:6-29:
 * hash_seed_init() fills the key from /dev/urandom once; hash_seed_get()
 * returns NULL before that.  pptk_rx_opts_default() copies the key into the
 * rx context when it has been initialised.
 */
#ifndef _HASH_SEED_H_
#define _HASH_SEED_H_

#ifdef __cplusplus
extern "C" {
#endif

extern char hash_seed[16];
extern int hash_seed_inited;

static inline void *hash_seed_get(void)
{
  return hash_seed_inited ? (void *)hash_seed : (void *)0;
}

void hash_seed_init(void);

#ifdef __cplusplus
}
#endif

#endif
