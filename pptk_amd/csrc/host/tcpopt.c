/*
 * tcpopt.c -- TCP option walks of the kept iphdr.h API (include/iphdr.h),
 * same names, arguments and results as the reference's iphdr/iphdr.c:4-246.
 *
 * All three walk the options [20, data offset) of a TCP header: kind 0
 * ends the list, kind 1 is a one-byte NOP, every other option has a length
 * byte, taken as min(length byte, bytes left) and -- except where noted --
 * a list whose next option has no room for its length byte or claims a
 * length below 2 is malformed and ends the walk.
 */
#include <stddef.h>
#include <stdint.h>

#include "iphdr.h"

/* Length of the option at `off` as the reference takes it: the length byte
 * capped at the bytes left, or the bytes left when the length byte lies past
 * the options (then always 1). */
static size_t opt_len(const unsigned char *t, size_t off, size_t end)
{
  const size_t left = end - off;
  if (off + 1 < end && t[off + 1] < left)
    return t[off + 1];
  return left;
}

/* iphdr.c:4-132.  For the kinds it decodes (2 MSS, 3 window scale, 4 SACK
 * permitted, 8 timestamp) the reference takes the length as opt_len() and
 * gives up below 2; for the others it gives up when the length byte is past
 * the options, then takes the same capped length -- which is opt_len() == 1
 * there -- so one rule covers every kind. */
void tcp_parse_options(void *pkt, struct tcp_information *info)
{
  const unsigned char *t = (const unsigned char *)pkt;
  const size_t end = tcp_data_offset(pkt);
  size_t off = 20;
  info->mss = 536;
  info->wscale = 0;
  info->options_valid = 0;
  info->sack_permitted = 0;
  info->mssoff = 0;
  info->ts_present = 0;
  info->ts = 0;
  info->tsecho = 0;
  while (off < end) {
    const unsigned kind = t[off];
    size_t len;
    if (kind == 0)
      break;
    if (kind == 1) {
      off++;
      continue;
    }
    len = opt_len(t, off, end);
    if (len < 2)
      return;   /* malformed: options_valid stays 0 */
    if (kind == 2 && len == 4) {
      info->mss = hdr_get16n(t + off + 2);
      info->mssoff = (uint8_t)off;
    } else if (kind == 3 && len == 3) {
      info->wscale = t[off + 2];
    } else if (kind == 4 && len == 2) {
      info->sack_permitted = 1;
    } else if (kind == 8 && len == 10) {
      info->ts = hdr_get32n(t + off + 2);
      info->tsecho = hdr_get32n(t + off + 6);
      info->ts_present = 1;
    }
    off += len;
  }
  info->options_valid = 1;
}

/* iphdr.c:134-199.  SACK (5) and timestamp (8) take opt_len() without the
 * "below 2" check: a length byte of 1 advances by one byte, and a length
 * byte of 0 makes the reference loop forever (it adds 0); here the walk
 * stops there instead, with the SACK fields recorded as the reference had
 * recorded them (parity unpinned for that input, the reference never
 * returns). */
void tcp_find_sack_ts_headers(void *pkt, struct sack_ts_headers *hdrs)
{
  const unsigned char *t = (const unsigned char *)pkt;
  const size_t end = tcp_data_offset(pkt);
  size_t off = 20;
  hdrs->sackoff = 0;
  hdrs->sacklen = 0;
  hdrs->tsoff = 0;
  while (off < end) {
    const unsigned kind = t[off];
    size_t len;
    if (kind == 0)
      return;
    if (kind == 1) {
      off++;
      continue;
    }
    len = opt_len(t, off, end);
    if (kind == 5) {
      hdrs->sacklen = (uint8_t)len;
      hdrs->sackoff = (uint8_t)off;
    } else if (kind == 8) {
      if (len == 10)
        hdrs->tsoff = (uint8_t)off;
    } else if (len < 2) {
      return;
    }
    if (len == 0)
      return;
    off += len;
  }
}

/* iphdr.c:201-246: the first SACK option, NULL if none before the end of
 * the list or a malformed option. */
void *tcp_find_sack_header(void *pkt, size_t *sacklen, int *sixteen_bit_align)
{
  unsigned char *t = (unsigned char *)pkt;
  const size_t end = tcp_data_offset(pkt);
  size_t off = 20;
  while (off < end) {
    const unsigned kind = t[off];
    size_t len;
    if (kind == 0)
      return NULL;
    if (kind == 1) {
      off++;
      continue;
    }
    len = opt_len(t, off, end);
    if (kind == 5) {
      if (sacklen)
        *sacklen = len;
      if (sixteen_bit_align)
        *sixteen_bit_align = !(off % 2);
      return t + off;
    }
    if (len < 2)
      return NULL;
    off += len;
  }
  return NULL;
}
