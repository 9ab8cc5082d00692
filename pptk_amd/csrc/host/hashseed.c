/* hashseed.c -- see include/hashseed.h (reference misc/hashseed.c:6-29:
 * re-initialisation and an unreadable /dev/urandom are fatal there too). */
#include <stdio.h>
#include <stdlib.h>

#include "../../../include/hashseed.h"

char hash_seed[16];
int hash_seed_inited;

void hash_seed_init(void)
{
  FILE *f;
  if (hash_seed_inited) {
    fprintf(stderr, "HASHSEED: trying to reinit hash seed\n");
    exit(1);
  }
  f = fopen("/dev/urandom", "r");
  if (f == NULL || fread(hash_seed, sizeof(hash_seed), 1, f) != 1) {
    fprintf(stderr, "HASHSEED: can't initialize hash seed\n");
    exit(1);
  }
  fclose(f);
  hash_seed_inited = 1;
}
