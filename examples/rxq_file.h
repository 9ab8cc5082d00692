/*
 * rxq_file.h -- the frame-set file of the examples (written by
 * tests/test_examples.py from the golden fixtures): a stand-in for the
 * frames an LDP interface's rx queues would hand out.
 *
 *   header   struct rxq_hdr (32 bytes)
 *   u64      off[n]        frame i starts at buf + off[i]
 *   u16      len[n]        frame i is len[i] bytes
 *   u8       buf[buf_bytes]
 *   u8       recs[n][64]   expected struct pptk_rx_rec of every frame
 */
#ifndef RXQ_FILE_H
#define RXQ_FILE_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pptk_rx.h"

#define RXQ_MAGIC 0x31515852u /* "RXQ1" */

struct rxq_hdr {
  uint32_t magic;
  uint32_t n;
  uint64_t buf_bytes;
  uint8_t key[16];   /* SipHash key the records were made with */
};

struct rxq_set {
  struct rxq_hdr h;
  uint64_t *off;
  uint16_t *len;
  uint8_t *buf;
  struct pptk_rx_rec *want;
};

static int rxq_load(const char *path, struct rxq_set *s)
{
  FILE *f = fopen(path, "rb");
  int ok;
  memset(s, 0, sizeof(*s));
  if (!f)
    return -1;
  ok = fread(&s->h, sizeof(s->h), 1, f) == 1 && s->h.magic == RXQ_MAGIC;
  if (ok) {
    s->off = malloc((size_t)s->h.n * 8 + 8);
    s->len = malloc((size_t)s->h.n * 2 + 2);
    s->buf = malloc(s->h.buf_bytes + 64);   /* + the 16-byte read slack */
    s->want = malloc((size_t)s->h.n * sizeof(struct pptk_rx_rec) + 64);
    ok = s->off && s->len && s->buf && s->want &&
         fread(s->off, 8, s->h.n, f) == s->h.n && fread(s->len, 2, s->h.n, f) == s->h.n &&
         fread(s->buf, 1, s->h.buf_bytes, f) == s->h.buf_bytes &&
         fread(s->want, sizeof(struct pptk_rx_rec), s->h.n, f) == s->h.n;
    if (ok)
      memset(s->buf + s->h.buf_bytes, 0, 64);
  }
  fclose(f);
  return ok ? 0 : -1;
}

static void rxq_free(struct rxq_set *s)
{
  free(s->off);
  free(s->len);
  free(s->buf);
  free(s->want);
}

#endif
