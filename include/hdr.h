/*
 * hdr.h -- unaligned host-order / network-order loads and stores.
 * Same API as the reference's misc/hdr.h:7-75 ("h" = host byte order,
 * "n" = network byte order); implemented with memcpy so any alignment works.
 */
#ifndef _HDR_H_
#define _HDR_H_

#include <stdint.h>
#include <string.h>
#include <arpa/inet.h>

#define PPTK_HDR_LOAD(name, type)                        \
  static inline type name(const void *buf)               \
  {                                                      \
    type v;                                              \
    memcpy(&v, buf, sizeof(v));                          \
    return v;                                            \
  }
#define PPTK_HDR_STORE(name, type)                       \
  static inline void name(void *buf, type v)             \
  {                                                      \
    memcpy(buf, &v, sizeof(v));                          \
  }

PPTK_HDR_LOAD(hdr_get64h, uint64_t)
PPTK_HDR_LOAD(hdr_get32h, uint32_t)
PPTK_HDR_LOAD(hdr_get16h, uint16_t)
PPTK_HDR_LOAD(hdr_get8h, uint8_t)
PPTK_HDR_STORE(hdr_set64h, uint64_t)
PPTK_HDR_STORE(hdr_set32h, uint32_t)
PPTK_HDR_STORE(hdr_set16h, uint16_t)
PPTK_HDR_STORE(hdr_set8h, uint8_t)

static inline uint32_t hdr_get32n(const void *buf) { return ntohl(hdr_get32h(buf)); }
static inline uint16_t hdr_get16n(const void *buf) { return ntohs(hdr_get16h(buf)); }
static inline void hdr_set32n(void *buf, uint32_t v) { hdr_set32h(buf, htonl(v)); }
static inline void hdr_set16n(void *buf, uint16_t v) { hdr_set16h(buf, htons(v)); }

#endif
