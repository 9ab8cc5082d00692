/*
 * ldp_packet.h -- the rx batch element handed out by ldp_in_nextpkts().
 *
 * Layout-compatible with `struct ldp_packet` of the reference
 * (ldp/ldp.h:98-108): a borrowed frame pointer, its length without FCS, and
 * 8 bytes of backend state (netmap buf_idx, socket slot, ...) that the rx
 * transform passes through untouched.  24 bytes on LP64.
 *
 * When the reference's ldp.h is already included, define LDP_PACKET_DEFINED
 * (or include this header first) so the struct is not declared twice.
 */
#ifndef PPTK_LDP_PACKET_H
#define PPTK_LDP_PACKET_H

#include <stdint.h>
#include <stddef.h>

#ifndef LDP_PACKET_DEFINED
#define LDP_PACKET_DEFINED
struct ldp_packet {
  void *data;
  uint32_t sz;
  union {
    uint32_t ancillary;
    uint64_t ancillary64;
    size_t ancillarysz;
    void *ancillaryptr;
    char ancillarydata[sizeof(void *)];
  };
};
#endif

#endif /* PPTK_LDP_PACKET_H */
