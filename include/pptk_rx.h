/*
 * pptk_rx.h -- C-ABI of the MI355X batch receive transform.
 *
 * One call turns a batch of Ethernet frames into one 64-byte record per
 * frame: IPv4 header checksum, TCP/UDP (v4/v6) checksum, fixed-format
 * L2/L3/L4 field extraction and a SipHash-2-4 flow hash of the 5-tuple.
 *
 * Where it plugs in: between ldp_in_nextpkts() and ldp_in_deallocate_some()
 * of an LDP rx loop (reference ldp/ldprecv.c:60-70, ldp/ldprecvmt.c:54-64,
 * ldp/ldpfwdmt.c:72-89).  The reference has no batch entry point: its rx
 * loops call the per-packet primitives below, one packet at a time:
 *   ip_hdr_cksum_calc      iphdr/ipcksum.c:39-49
 *   tcp_cksum_calc         iphdr/ipcksum.c:51-68
 *   tcp6_cksum_calc        iphdr/ipcksum.c:74-115
 *   udp_cksum_calc         iphdr/ipcksum.c:117-134
 *   udp6_cksum_calc        iphdr/ipcksum.c:140-181
 *   ipv6_const_proto_hdr_2 iphdr/iphdr.h:804-860
 *   siphash_buf            misc/siphash.h:214-229
 *   ip_permitted hashing   iphash/iphash.c:157-162 (v4), :108-120 (v6)
 * pptk_rx_batch() replaces that per-packet loop; its record carries exactly
 * the values those functions return for the same frame.
 *
 * Plain C types only: no HIP, torch or RCCL types appear in signatures.
 * Every function returns 0 or a negative errno (-EINVAL, -ENOMEM, -EIO for
 * HIP/RCCL failures; the multi-GPU calls also -ETIMEDOUT, -ECANCELED and
 * -ENOSYS, see there).  Nothing aborts on packet content: per-packet problems
 * are reported in pptk_rx_rec.flags.
 */
#ifndef PPTK_RX_H
#define PPTK_RX_H

#include <stddef.h>
#include <stdint.h>

#include "ldp_packet.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-packet record (64 bytes, one per frame, written at the frame's
 * index).  Multi-byte integers are host (little-endian) order unless noted. */
struct pptk_rx_rec {
  uint64_t flow_hash;  /*  0 siphash_buf(key, tuple, 40); 0 if !PARSED      */
  uint8_t src[16];     /*  8 network-order address; IPv4 uses bytes 0..3    */
  uint8_t dst[16];     /* 24 idem                                           */
  uint16_t sport;      /* 40 host order (tcp_src_port / udp_src_port)       */
  uint16_t dport;      /* 42                                                */
  uint16_t ip_cksum;   /* 44 ip_hdr_cksum_calc(ip, ihl); 0 == valid; 0 v6   */
  uint16_t l4_cksum;   /* 46 tcp/udp(6)_cksum_calc(...); 0 == valid         */
  uint16_t l4_off;     /* 48 frame offset of the L4 header                  */
  uint16_t l4_len;     /* 50 L4 length = ip_total_len - ihl (v6: tlen - off)*/
  uint8_t l3_off;      /* 52 14, or 18 behind an 802.1Q tag                 */
  uint8_t proto;       /* 53 ip_proto / final IPv6 next header              */
  uint16_t flags;      /* 54 PPTK_RX_F_*                                    */
  uint32_t src_bucket; /* 56 ip_permitted/ipv6_permitted bucket, 0 if off   */
  uint16_t ethertype;  /* 60 (inner) ethertype, host order                  */
  uint8_t ip_version;  /* 62 version nibble of the L3 header (0 if none)    */
  uint8_t reserved;    /* 63 always 0                                       */
};

/* ---- compact record (32 bytes): the same values minus the raw checksum
 * words, ethertype, version and the IPv6 addresses (IPv6 frames carry 0 in
 * src4/dst4; the addresses are at frame + l3_off + 8 / + 24).  Written
 * instead of pptk_rx_rec when pptk_rx_dev_batch.d_recs32 is set: half the
 * record bytes, which is what bounds small frames. */
struct pptk_rx_rec32 {
  uint64_t flow_hash;  /*  0 as pptk_rx_rec.flow_hash                       */
  uint32_t src4;       /*  8 IPv4 source, network byte order; 0 for IPv6    */
  uint32_t dst4;       /* 12 IPv4 destination; 0 for IPv6                   */
  uint16_t sport;      /* 16 host order                                     */
  uint16_t dport;      /* 18                                                */
  uint16_t flags;      /* 20 PPTK_RX_F_*                                    */
  uint8_t proto;       /* 22                                                */
  uint8_t l3_off;      /* 23                                                */
  uint16_t l4_off;     /* 24                                                */
  uint16_t l4_len;     /* 26                                                */
  uint32_t src_bucket; /* 28                                                */
};

/* ---- fragment side record (16 bytes, one per frame, written at the
 * frame's index when pptk_rx_dev_batch.d_frag is set): what an IP
 * reassembler needs -- reference ipfrag/ipreass.c:118-124 and
 * ipfrag/rfc815.c:145-151 key on ip_frag_off, ip_more_frags, ip_total_len
 * and ip_hdr_len -- so fragments can be handed on without parsing the frame
 * a second time.  All zero for frames that are not PARSED, are MALFORMED,
 * or are IPv6 without a fragment header.  Fields are host order. */
struct pptk_rx_frag {
  uint32_t ident;        /*  0 IPv4 ip_id (iphdr/iphdr.h:1093-1097); IPv6 the
                                fragment header's 32-bit Identification     */
  uint16_t frag_off;     /*  4 data offset in bytes: ip_frag_off (:1124-1128)
                                / ipv6_frag_off (:727-731)                  */
  uint16_t data_len;     /*  6 fragment data bytes: IPv4 ip_total_len - ihl;
                                IPv6 40 + payload_len - (frag_hdr_off + 8)  */
  uint16_t frag_hdr_off; /*  8 IPv6: *frag_hdr_off_ptr of
                                ipv6_const_proto_hdr_2 (:804-860), counted
                                from the IPv6 header (the last fragment
                                header of the chain); IPv4: 0               */
  uint16_t proto_hdr_off_from_frag; /* 10 IPv6: its *proto_hdr_off_from_frag
                                (0 for a non-first fragment); IPv4: 0       */
  uint8_t next_hdr;      /* 12 IPv4 ip_proto; IPv6 the fragment header's
                                Next Header byte                            */
  uint8_t flags;         /* 13 PPTK_RX_FRAG_*                               */
  uint16_t reserved;     /* 14 always 0                                     */
};

#define PPTK_RX_FRAG_IS 0x01u   /* a fragment: PPTK_RX_F_FRAGMENT            */
#define PPTK_RX_FRAG_MF 0x02u   /* ip_more_frags (:1023-1027) /
                                   ipv6_more_frags (:733-737)               */
#define PPTK_RX_FRAG_DF 0x04u   /* ip_dont_frag (:1040-1044), IPv4 only      */
#define PPTK_RX_FRAG_V6 0x08u   /* fields taken from an IPv6 fragment header */

#define PPTK_RX_F_PARSED 0x0001u      /* IPv4/IPv6 header parsed            */
#define PPTK_RX_F_IP_OK 0x0002u       /* ip_cksum == 0 (always for IPv6)    */
#define PPTK_RX_F_L4_OK 0x0004u       /* L4 present and l4_cksum == 0       */
#define PPTK_RX_F_L4 0x0008u          /* TCP/UDP header present             */
#define PPTK_RX_F_IPV6 0x0010u        /* L3 is IPv6                         */
#define PPTK_RX_F_VLAN 0x0020u        /* one 802.1Q tag was skipped         */
#define PPTK_RX_F_FRAGMENT 0x0040u    /* IPv4 MF/offset or IPv6 frag header */
#define PPTK_RX_F_UDP_ZERO 0x0080u    /* UDP checksum field transmitted 0   */
#define PPTK_RX_F_MALFORMED 0x0100u   /* lengths/IHL/ext chain inconsistent */
#define PPTK_RX_F_V6_EXT 0x0200u      /* IPv6 extension headers walked      */

/* ---- context ------------------------------------------------------------ */
struct pptk_rx_ctx;

struct pptk_rx_opts {
  int device;           /* HIP device ordinal                              */
  uint8_t key[16];      /* SipHash key (hash_seed in the reference)        */
  uint8_t iphash_bits4; /* ip_permitted prefix bits, 1..32; 0 = no bucket  */
  uint8_t iphash_bits6; /* ipv6_permitted prefix bits, 1..128; 0 = off     */
  uint16_t gather_threads; /* host threads gathering staged frames (0 = 1) */
  uint32_t iphash_size; /* struct ip_hash.hash_size (power of two)         */
  uint32_t max_batch;   /* pptk_rx_batch chunk (frames per staged transfer) */
  uint32_t max_frame;   /* largest frame accepted by pptk_rx_batch (<=65535)*/
  uint32_t comm_timeout_ms; /* bound on every multi-GPU wait (communicator
                           creation, a gather's enqueue, pptk_rx_comm_sync,
                           teardown); 0 = PPTK_RX_COMM_TIMEOUT_MS          */
};

#define PPTK_RX_COMM_TIMEOUT_MS 60000u

void pptk_rx_opts_default(struct pptk_rx_opts *opts);

int pptk_rx_ctx_create(struct pptk_rx_ctx **ctx, const struct pptk_rx_opts *opts);
void pptk_rx_ctx_destroy(struct pptk_rx_ctx *ctx);

/* Host in -> host out.  Gathers the borrowed ldp_packet frames into pinned
 * staging (or reads them in place from a registered ring, see below), copies
 * them to HBM, runs the transform and copies the records back, in chunks of
 * opts.max_batch frames, up to four in flight on their own streams (each
 * with its own staging, allocated when a call first has that many chunks);
 * synchronous: on
 * return recs[0..num) are final and no pointer in pkts is retained.
 * ancillary fields are neither read nor written.  Frames longer than
 * opts.max_frame get PPTK_RX_F_MALFORMED only. */
int pptk_rx_batch(struct pptk_rx_ctx *ctx, const struct ldp_packet *pkts,
                  int num, struct pptk_rx_rec *recs);

/* The same with compact 32-byte records (struct pptk_rx_rec32, the values
 * of pptk_rx_rec minus the raw checksum words, ethertype, version and the
 * IPv6 addresses): half the record bytes back over PCIe, which is what
 * bounds small frames host to host (a 64-byte frame's 64-byte record moves
 * as many bytes up as the frame moved down).  Same rules as pptk_rx_batch,
 * including records written in place into a registered region. */
int pptk_rx_batch32(struct pptk_rx_ctx *ctx, const struct ldp_packet *pkts,
                    int num, struct pptk_rx_rec32 *recs);

/* pptk_rx_batch split in two, so that an rx loop overlaps one batch's GPU
 * round trip with fetching and submitting the next (the synchronous call
 * leaves the host idle for the whole launch-to-completion latency, which
 * dominates LDP-sized batches; DESIGN.md "Pipelined host batches"):
 *
 *   ldp_in_nextpkts(q, pkts[k], ...);  pptk_rx_batch_submit(ctx, pkts[k], n, recs[k]);
 *   if (pptk_rx_batch_pending(ctx) == DEPTH) {   -- DEPTH <= PPTK_RX_MAX_INFLIGHT
 *     pptk_rx_batch_complete(ctx);      -- batch k-DEPTH+1: recs final, frames free
 *     ... use its recs ...;  ldp_in_deallocate_some(q, its pkts, ...);
 *   }
 *
 * submit gathers and enqueues one batch of 1..opts.max_batch frames (one
 * chunk) and returns without waiting; the frames and recs[0, num) must stay
 * valid and untouched until the batch is completed.  complete waits for the
 * OLDEST outstanding submission (FIFO) and returns its frame count (> 0):
 * after it its records are final and none of its pointers is retained.
 * Results are those of pptk_rx_batch.  At most PPTK_RX_MAX_INFLIGHT
 * submissions are outstanding per context (submit returns -EBUSY beyond;
 * each depth in use keeps its own staging buffers, allocated on first use);
 * pptk_rx_batch returns -EBUSY while any is; num == 0 submits nothing and
 * returns 0; num > opts.max_batch is -EINVAL (use pptk_rx_batch);
 * complete with nothing outstanding returns -ENOENT.  A failed submit
 * leaves nothing outstanding.  pptk_rx_ctx_destroy waits for (and drops)
 * outstanding submissions. */
#define PPTK_RX_MAX_INFLIGHT 4
int pptk_rx_batch_submit(struct pptk_rx_ctx *ctx, const struct ldp_packet *pkts, int num,
                         struct pptk_rx_rec *recs);
/* pptk_rx_batch_submit with compact records (as pptk_rx_batch32); completed
 * by pptk_rx_batch_complete like any other submission. */
int pptk_rx_batch_submit32(struct pptk_rx_ctx *ctx, const struct ldp_packet *pkts, int num,
                           struct pptk_rx_rec32 *recs);
int pptk_rx_batch_complete(struct pptk_rx_ctx *ctx);
int pptk_rx_batch_pending(const struct pptk_rx_ctx *ctx);

/* Zero-copy rx rings: register a host region (e.g. a netmap ring's buffer
 * area or a socket ring) once; pptk_rx_batch() calls whose frames all lie in
 * one registered ring skip the host gather into staging: a chunk whose
 * frames fill >= 80 % of the ring span they cover (and that span > 2 MiB)
 * is copied down by DMA as one span, any other chunk is read by the GPU in
 * place over PCIe (PPTK_RX_RING_DMA_PCT sets the fraction).  Every frame's
 * end rounded up to 16 bytes must lie inside the region.  A registered
 * region that holds a call's whole record array (recs[0, num)) receives the
 * records in place: the kernel writes them there over PCIe and the host
 * copies nothing back -- register the rx loop's record array once.
 * Unregister before freeing the memory. */
int pptk_rx_register_ring(struct pptk_rx_ctx *ctx, void *base, size_t bytes);
int pptk_rx_unregister_ring(struct pptk_rx_ctx *ctx, void *base);

/* Device-resident batch (asynchronous on `stream`, a hipStream_t or NULL).
 * Frame i starts at d_frames + (d_off ? d_off[i] : i * stride) and is
 * (d_len ? d_len[i] : fixed_len) bytes long.  d_perm (nullable) gives the
 * processing order (a permutation of 0..n-1, e.g. from
 * pptk_rx_bin_device); records always land at d_recs[i] (or d_recs32[i]
 * when that is set: compact records, d_recs unused) for frame i.
 * d_hash (nullable) additionally receives flow_hash[i] as a dense u64 array,
 * the send buffer of the multi-GPU all-gather; d_frag (nullable) receives
 * the fragment side record of every frame (struct pptk_rx_frag).
 * The frame buffer must stay readable up to the next 16-byte boundary past
 * the last frame (any hipMalloc allocation is); the 16-byte chunk holding
 * the start of an empty (0-byte) frame is read too. */
struct pptk_rx_dev_batch {
  const uint8_t *d_frames;
  const uint64_t *d_off;  /* nullable: fixed stride                       */
  const uint16_t *d_len;  /* nullable: fixed_len                          */
  const uint32_t *d_perm; /* nullable: identity order                     */
  uint64_t stride;
  uint32_t fixed_len;
  uint32_t max_len;       /* upper bound of frame lengths (tuning only)   */
  uint64_t n;
  struct pptk_rx_rec *d_recs;     /* nullable when d_recs32 is set     */
  uint64_t *d_hash;       /* nullable                                     */
  struct pptk_rx_rec32 *d_recs32; /* nullable: compact records instead */
  struct pptk_rx_frag *d_frag;    /* nullable: fragment side records    */
  uint32_t *d_key;        /* nullable: dense rate-limiter key per frame:
                             src_bucket of a PARSED IPv4 frame, src_bucket |
                             0x80000000 of a PARSED IPv6 frame, 0xffffffff
                             otherwise (pptk_rx_permit_keys_device)      */
};

int pptk_rx_batch_device(struct pptk_rx_ctx *ctx,
                         const struct pptk_rx_dev_batch *b, void *stream);

/* Length binning for mixed-size batches: writes into d_perm a stable
 * permutation of 0..n-1 ordered by length group (the groups of
 * pptk_rx_batch_device_mixed), so the lanes of one wavefront sum frames of
 * similar length.  d_scratch must hold
 * pptk_rx_bin_scratch_bytes(n) bytes.  Asynchronous on `stream`. */
size_t pptk_rx_bin_scratch_bytes(uint64_t n);
int pptk_rx_bin_device(struct pptk_rx_ctx *ctx, const uint16_t *d_len,
                       uint64_t n, uint32_t *d_perm, void *d_scratch,
                       void *stream);

/* Mixed-size batch in one call.  Length binning pays on MI355X only when a
 * batch mixes jumbo frames (> 1521 bytes, which batch order would stream
 * with the 64-lane jumbo shape) with shorter ones; every split of 64..1521 B
 * frames into groups measured slower than batch order (DESIGN.md "Binned
 * order").  So: with b->max_len (a hint) at most 1521 the call runs the
 * batch in batch order, as pptk_rx_batch_device; otherwise a device pass
 * counts the length groups (..113, ..1521 bytes, longer) and, when the
 * batch holds frames of the last group and shorter ones, bins it
 * (pptk_rx_bin_device into the permutation) and runs one launch per group,
 * each streamed by the kernel shape sized for it; else batch order by the
 * launch of the highest non-empty group.  Results are identical either way.
 * Requires d_len; b->d_perm is ignored.  d_perm (nullable) receives the
 * processing order: the binned permutation, or the identity.  d_scratch:
 * pptk_rx_bin_scratch_bytes(n) bytes (counters, group table, the binned
 * descriptors the group launches stream, and the permutation when d_perm
 * is NULL); both stay in use until the stream reaches the end of the call.
 * Records land at d_recs[i] for frame i. */
int pptk_rx_batch_device_mixed(struct pptk_rx_ctx *ctx,
                               const struct pptk_rx_dev_batch *b, uint32_t *d_perm,
                               void *d_scratch, void *stream);

/* Batched rate limiting: ip_permitted / ipv6_permitted (reference
 * iphash/iphash.c:108-197) for a device batch, with the result the
 * reference gives when called once per frame in frame order.  The subject
 * frames are the PARSED frames of `family` (4 or 6; the context must have
 * that family's iphash_bits set, so the records carry its bucket) for which
 * d_subject[i] != 0 (d_subject nullable = all of them).  d_tokens holds
 * opts.iphash_size u32 counters (the entries of struct ip_hash, widened to
 * u32); verdict[i] = 1 permitted (a token was consumed), 0 denied, 2 not a
 * subject.  Reads one of d_recs / d_recs32 (the other NULL).  d_scratch:
 * pptk_rx_permit_scratch_bytes(n, opts.iphash_size) bytes.  Asynchronous. */
size_t pptk_rx_permit_scratch_bytes(uint64_t n, uint32_t hash_size);
int pptk_rx_permit_device(struct pptk_rx_ctx *ctx, const struct pptk_rx_rec *d_recs,
                          const struct pptk_rx_rec32 *d_recs32, uint64_t n, int family,
                          const uint8_t *d_subject, uint32_t *d_tokens,
                          uint8_t *d_verdict, void *d_scratch, void *stream);

/* The same from the dense keys the receive transform wrote into
 * pptk_rx_dev_batch.d_key (4 bytes per frame instead of a 16-byte slice of
 * each record).  Results are those of pptk_rx_permit_device on the
 * records of the same batch; same scratch size.  A key whose bucket (bits
 * 0..30) is >= opts.iphash_size -- only caller-made keys can be -- is not a
 * subject (verdict 2, no token touched).  Up to 2^16 buckets and 16 M
 * frames (65 536 per CU) this runs as one persistent launch that reads the
 * keys once (DESIGN.md section 5 "Rate limiter"); beyond, or with
 * PPTK_RX_TUNE_PERMIT_PASSES set (pptk_rx_set_tuning, or the PPTK_RX_TUNE
 * environment word), as four launches.  The persistent launch needs all its
 * workgroups resident at once: the library orders every such launch of a
 * device behind the previous one, whatever stream or context issued it, so
 * concurrent calls never starve each other; calls that share one scratch
 * buffer must still be ordered on one stream.  Should the workgroups not
 * all become resident within 2 s (e.g. another process's kernels hold the
 * CUs), the launch aborts and fails closed: every subject frame's verdict
 * is 0 (denied, as the reference denies a frame it has no token for), the
 * others 2, the token counts are left as they were before the call (nothing
 * half-updated: all workgroups act on one commit-or-abort decision), and
 * pptk_rx_permit_status reports -ETIMEDOUT; never a hang.  The scratch
 * needs no initialisation. */
int pptk_rx_permit_keys_device(struct pptk_rx_ctx *ctx, const uint32_t *d_keys, uint64_t n,
                               int family, const uint8_t *d_subject, uint32_t *d_tokens,
                               uint8_t *d_verdict, void *d_scratch, void *stream);

/* Whether every pptk_rx_permit_keys_device call on d_scratch since the last
 * status query completed: 0, or -ETIMEDOUT if one aborted (its subject
 * frames were denied and its tokens left unchanged: repeat it, e.g. with
 * PPTK_RX_TUNE_PERMIT_PASSES, to get the verdicts the tokens allow).
 * Synchronises `stream` (the stream those calls ran on).  -EIO on a HIP
 * error.  The library tracks up to 1024 scratch buffers; a buffer not
 * queried while 1024 others were used since reports 0. */
int pptk_rx_permit_status(struct pptk_rx_ctx *ctx, const void *d_scratch, void *stream);

/* The token refill timer (batch_timer_fn, reference iphash/iphash.c:
 * 290-350) for buckets [start, end): tokens = min(tokens + add, initial).
 * Asynchronous; order it with pptk_rx_permit_device on one stream. */
int pptk_rx_tokens_refill_device(struct pptk_rx_ctx *ctx, uint32_t *d_tokens,
                                 uint32_t start, uint32_t end, uint32_t add,
                                 uint32_t initial_tokens, void *stream);

/* Tx side (reference iphdr/ipcksum.h:101-211, callers ldp/ldpsend.c:
 * 162-167): set, in place, the checksums of every frame of a device batch as
 * ip46_set_hdr_cksum_calc + tcp/udp(6)_set_cksum_calc would -- the IPv4
 * header checksum of every parsed IPv4 frame, the TCP/UDP checksum of every
 * frame with an L4 header (PPTK_RX_F_L4: not a fragment, long enough),
 * located exactly as pptk_rx_batch_device parses.  Frames the receive
 * transform would not parse are left untouched.  After it, the receive
 * transform verifies every such frame (IP_OK / L4_OK).  Layout arguments as
 * in pptk_rx_dev_batch; max_len is a tuning hint.  Asynchronous.
 * Fixed-stride batches run in two passes (checksums into a side array of 8
 * bytes per frame, then the field writes).  The side array is allocated and
 * freed on `stream` from a stream-ordered pool the context owns, so tx calls
 * of one context may run concurrently on different streams. */
int pptk_tx_cksum_device(struct pptk_rx_ctx *ctx, uint8_t *d_frames, const uint64_t *d_off,
                         const uint16_t *d_len, uint64_t stride, uint32_t fixed_len,
                         uint64_t n, uint32_t max_len, void *stream);

/* The two-pass side array from the caller: `frames` * 8 bytes of device
 * memory (8-byte aligned) that the context uses instead of its pool, e.g. a
 * buffer placed like a record ring (its writes beside the frame reads cost
 * what record writes cost: pptk_rx_place_records).  Every tx call of the
 * context that fits uses this ONE buffer: such calls must not overlap (use
 * one stream, or order the streams).  The buffer must stay valid until the
 * context is destroyed or another buffer (or NULL: back to the pool) is
 * set; batches larger than `frames` use the pool. */
int pptk_tx_set_side_buffer(struct pptk_rx_ctx *ctx, void *d_side, uint64_t frames);

/* Header rewrite with incremental checksum update (NAT / forwarding),
 * reference iphdr/ipcksum.h:213-393: per frame, in this order,
 *   PPTK_RW_DECR_TTL  ip_decr_ttl_cksum_update          (:374-393)
 *   PPTK_RW_SRC       ip_set_src_cksum_update(src)      (:238-261)
 *   PPTK_RW_DST       ip_set_dst_cksum_update(dst)      (:349-372)
 *   PPTK_RW_SPORT     tcp/udp_set_src_port_cksum_update (:263-271, :323-334)
 *   PPTK_RW_DPORT     tcp/udp_set_dst_port_cksum_update (:273-281, :336-347)
 *   PPTK_RW_ICMP_ID   icmp_set_echo_identifier_cksum_update (:283-291), with
 *                     the new identifier in `sport`
 * each computing the new checksum from the old one with ip_update_cksum16/32
 * (:213-236), results identical to calling those functions in that order.
 * Applies to every frame the receive transform parses as IPv4; the TCP/UDP
 * parts (the L4 checksum follow-up of an address change, the port writes)
 * only when its record has PPTK_RX_F_L4 (an L4 header, not a fragment), and
 * a UDP checksum of 0 stays 0 as in the reference; the ICMP identifier
 * only on an echo request or reply (type 8 / 0) that is not a fragment and
 * has its 8-byte header inside the packet.  A frame whose TTL is 0
 * under PPTK_RW_DECR_TTL (the reference abort()s) is left untouched.
 * Addresses and ports are host order, as the reference's setters take them.
 * d_rw holds rw_count = 1 (one rewrite for every frame) or n entries.
 * d_status (nullable) receives per frame PPTK_RW_ST_* bits.  Layout
 * arguments as in pptk_tx_cksum_device.  Asynchronous on `stream`. */
struct pptk_rewrite {
  uint32_t ops;    /* PPTK_RW_* */
  uint32_t src;    /* new IPv4 source (host order) */
  uint32_t dst;    /* new IPv4 destination (host order) */
  uint16_t sport;  /* new TCP/UDP source port (host order) */
  uint16_t dport;  /* new TCP/UDP destination port (host order) */
};
#define PPTK_RW_DECR_TTL 0x1u
#define PPTK_RW_SRC 0x2u
#define PPTK_RW_DST 0x4u
#define PPTK_RW_SPORT 0x8u
#define PPTK_RW_DPORT 0x10u
#define PPTK_RW_ICMP_ID 0x20u
#define PPTK_RW_ST_IP 0x1u         /* parsed IPv4: the IP-level ops applied */
#define PPTK_RW_ST_L4 0x2u         /* L4 header present: the L4 ops applied */
#define PPTK_RW_ST_TTL_ZERO 0x4u   /* TTL was 0: frame left untouched      */
#define PPTK_RW_ST_EXPIRED 0x8u    /* TTL reached 0 (reference returns 0)  */
#define PPTK_RW_ST_ICMP 0x10u      /* ICMP echo: the identifier op applied  */
int pptk_tx_rewrite_device(struct pptk_rx_ctx *ctx, uint8_t *d_frames, const uint64_t *d_off,
                           const uint16_t *d_len, uint64_t stride, uint32_t fixed_len,
                           uint64_t n, const struct pptk_rewrite *d_rw, uint64_t rw_count,
                           uint8_t *d_status, void *stream);

/* TCP MSS clamping with incremental checksum update (middlebox / tunnel
 * ingress), reference iphdr/iphdr.c:4-132 (tcp_parse_options) and
 * iphdr/ipcksum.h:466-489 (tcp_set_mss_cksum_update): per frame with a TCP
 * header (the receive transform's record: PPTK_RX_F_L4 and proto 6, IPv4 or
 * IPv6, with or without a VLAN tag; with PPTK_MSS_SYN_ONLY also the SYN flag
 * set), whose options lie inside the segment (l4_off + data offset <= L4
 * end), tcp_parse_options is applied to the TCP header; if the option list
 * is valid and holds an MSS option whose value exceeds `mss`, the value
 * becomes `mss` through tcp_set_mss_cksum_update -- results identical to
 * those two calls.  Everything else is left untouched.  d_status (nullable)
 * receives per frame PPTK_MSS_ST_* bits.  Layout arguments as in
 * pptk_tx_cksum_device.  Asynchronous on `stream`. */
#define PPTK_MSS_SYN_ONLY 0x1u
#define PPTK_MSS_ST_TCP 0x1u       /* TCP header present (and SYN if asked) */
#define PPTK_MSS_ST_FOUND 0x2u     /* valid options with an MSS option      */
#define PPTK_MSS_ST_CLAMPED 0x4u   /* MSS lowered to `mss`                  */
#define PPTK_MSS_ST_BADOPT 0x8u    /* options past the segment or malformed */
int pptk_tcp_mss_clamp_device(struct pptk_rx_ctx *ctx, uint8_t *d_frames, const uint64_t *d_off,
                              const uint16_t *d_len, uint64_t stride, uint32_t fixed_len,
                              uint64_t n, uint16_t mss, uint32_t flags, uint8_t *d_status,
                              void *stream);

/* Tuning: force kernel variant `variant` (0 .. pptk_rx_variant_count()-1)
 * and/or memory-policy flags for every later batch of this context; -1
 * restores the automatic choice (variant by frame length and alignment).
 * flags: PPTK_RX_TUNE_NT_LOADS (non-temporal frame loads),
 * PPTK_RX_TUNE_NO_STAGING (store records per lane, not via LDS),
 * PPTK_RX_TUNE_NT_STORES (non-temporal record stores),
 * PPTK_RX_TUNE_SC1_STORES (write-through record stores),
 * PPTK_RX_TUNE_BLOCKED (each wavefront takes a contiguous block of tiles
 * instead of every nwaves-th tile), PPTK_RX_TUNE_PERMIT_PASSES (the rate
 * limiter's four-launch path instead of its fused one-launch path; a flags
 * word holding only this bit leaves the receive transform's memory policy
 * automatic).
 * Variants and flags change speed only: results are identical for every
 * setting on every input.  Any other flag bit is rejected with -EINVAL
 * (PPTK_RX_TUNE in the environment is masked to these bits). */
#define PPTK_RX_TUNE_NT_LOADS 0x1
#define PPTK_RX_TUNE_NO_STAGING 0x2
#define PPTK_RX_TUNE_NT_STORES 0x20
#define PPTK_RX_TUNE_SC1_STORES 0x40
#define PPTK_RX_TUNE_BLOCKED 0x100   /* contiguous tiles per wavefront */
#define PPTK_RX_TUNE_PERMIT_PASSES 0x400   /* rate limiter: four launches, not one */
int pptk_rx_set_tuning(struct pptk_rx_ctx *ctx, int variant, int flags);
int pptk_rx_variant_count(void);
/* The kernel variant the last device batch of this context launched (the
 * automatic or forced choice after eligibility checks; -1 before the first
 * batch).  Diagnostics for tests and benchmarks. */
int pptk_rx_last_variant(const struct pptk_rx_ctx *ctx);

/* Autotuning: run the batch (records are written, as by
 * pptk_rx_batch_device) with the automatic kernel variant and the shapes
 * interchangeable with it -- two warm-up rounds, then reps timed rounds of
 * one launch per shape, interleaved so that clock drift falls on all alike
 * -- and let later device batches of the same automatic variant and layout
 * (fixed-stride or offset-described) use the fastest median (another shape
 * must beat the automatic one by 1 % to replace it).  The best shape
 * depends on how expensive the record writes are (which follows where the
 * record buffer sits, see pptk_rx_place_records) and, for
 * offset-described batches, on the length mix (the candidates include the
 * kernel that bins each tile's frames by length into 4-, 8- and 16-lane
 * rounds, fastest on IMIX-like streams of mostly small frames);
 * results never change.  Synchronous; reps 1..100.
 * pptk_rx_set_tuning's forced variant still takes precedence. */
int pptk_rx_autotune(struct pptk_rx_ctx *ctx, const struct pptk_rx_dev_batch *batch, int reps,
                     void *stream);

/* ---- Multi-GPU (RCCL over xGMI) ------------------------------------------
 * Batches shard embarrassingly: GPU r of R runs pptk_rx_batch_device on its
 * own contiguous range of the batch (pptk_rx_shard_range) with d_hash set,
 * and pptk_rx_allgather_hash then gives every GPU the flow hash of every
 * frame (ncclAllGather of u64 over one communicator).  The reference scales
 * with one rx thread per queue (ldp/ldprecvmt.c:174-182); here one context
 * per GPU, driven by one process per GPU (pptk_rx_comm_uid +
 * pptk_rx_comm_create) or by one thread per GPU of a single process
 * (pptk_rx_comm_create_all).  The communicator belongs to its context and is
 * destroyed with it (or by pptk_rx_comm_destroy).
 *
 * Failure containment: the reference's queue threads share nothing, so one
 * failing thread never stalls the others; ranks of a collective do wait for
 * each other.  So no call here waits without a bound: creation gives up
 * after opts.comm_timeout_ms (-ETIMEDOUT, e.g. a rank that never joins),
 * pptk_rx_comm_sync waits for a stream with a deadline and surfaces RCCL's
 * asynchronous errors (a dead peer: -EIO), and pptk_rx_comm_abort lets any
 * thread cancel a communicator other threads are waiting on.  After
 * -ETIMEDOUT / -EIO from a gather or a sync, or an abort, the communicator
 * is dead (calls on it return -ECANCELED): destroy it and create a new one.
 * RCCL is loaded on first use; without it these calls return -ENOSYS. */
#define PPTK_RX_COMM_UID_BYTES 128

/* Number of visible GPUs (>= 0), or -EIO. */
int pptk_rx_device_count(void);

/* A new communicator id: made once by one rank and handed to every rank
 * through the application's own channel (a file, a socket, MPI). */
int pptk_rx_comm_uid(uint8_t uid[PPTK_RX_COMM_UID_BYTES]);

/* Join `ctx` (one context per GPU) to communicator `uid` as rank `rank` of
 * `nranks`.  Collective: blocks until every rank has called it, at most
 * opts.comm_timeout_ms (then -ETIMEDOUT and the context has no
 * communicator, so it may try again with a new uid).  -ECANCELED if
 * pptk_rx_comm_abort was called on the context while this ran, or before
 * it (a pending abort, consumed by this call).  -EAGAIN if kMaxAbandoned
 * (4) earlier creations of this process that gave up are still stuck inside
 * RCCL (a rank that never joined).  -EINVAL if the context already has a
 * communicator or a creation in progress. */
int pptk_rx_comm_create(struct pptk_rx_ctx *ctx, int nranks, int rank,
                        const uint8_t uid[PPTK_RX_COMM_UID_BYTES]);

/* Single process, one thread per GPU: one communicator over ctxs[0..n)
 * (each on a different device), rank i = ctxs[i].  Call from one thread;
 * afterwards each rx thread uses its own context concurrently.  Bounded by
 * ctxs[0]'s opts.comm_timeout_ms; an abort of any of the contexts cancels
 * it (-ECANCELED, as pptk_rx_comm_create); on any failure no context keeps
 * one. */
int pptk_rx_comm_create_all(struct pptk_rx_ctx *const *ctxs, int n);

/* Orderly teardown (flushes enqueued gathers, bounded; an abort if the
 * flush does not finish).  Also drops a pending abort.  The context may then
 * create a new one.  -EBUSY while the context's creation is in progress. */
int pptk_rx_comm_destroy(struct pptk_rx_ctx *ctx);

/* Cancel the context's communicator now, from any thread: RCCL's kernels
 * of pending gathers return (so their streams drain, with wrong gathered
 * data), waits in pptk_rx_comm_sync / pptk_rx_allgather_hash on it return
 * -ECANCELED, and so does every later call on it until
 * pptk_rx_comm_destroy.  A creation still in progress on the context
 * (pptk_rx_comm_create / _create_all) returns -ECANCELED promptly and keeps
 * nothing; on a context with no communicator yet the abort is kept pending
 * and cancels its next creation.  An rx thread that fails calls this on
 * every context of the job, so no sibling waits for a gather -- or a
 * creation -- it will never join (examples/rx_multigpu.c).  0 in every
 * case.  It must not race with pptk_rx_comm_destroy or pptk_rx_ctx_destroy
 * of the same context. */
int pptk_rx_comm_abort(struct pptk_rx_ctx *ctx);

/* Wait until everything enqueued on `stream` (gathers included) is done,
 * for at most timeout_ms (0 = opts.comm_timeout_ms), watching the
 * communicator for RCCL's asynchronous errors.  0: done.  -ETIMEDOUT: the
 * deadline passed (a peer never issued its part); -EIO: RCCL reported an
 * error (a peer died); in both cases the communicator is aborted, so the
 * stream drains.  -ECANCELED: it was aborted (pptk_rx_comm_abort).  Use it
 * instead of hipStreamSynchronize on a stream that carries gathers.
 * Without a communicator: a bounded stream wait (-ETIMEDOUT). */
int pptk_rx_comm_sync(struct pptk_rx_ctx *ctx, void *stream, uint32_t timeout_ms);

/* The context's communicator size and rank; -EINVAL without one. */
int pptk_rx_comm_info(const struct pptk_rx_ctx *ctx, int *nranks, int *rank);

/* Equal-shard policy for a batch of n frames over nranks GPUs: per_rank =
 * ceil(n / nranks); rank r owns frames [first, first + count) with first =
 * min(r * per_rank, n).  Every rank all-gathers per_rank hashes (the last
 * ranks' shards are padded), so the gathered array holds the flow hash of
 * global frame i at index i for every i < n. */
void pptk_rx_shard_range(uint64_t n, int nranks, int rank, uint64_t *first, uint64_t *count,
                         uint64_t *per_rank);

/* d_out[r * n + i] = d_hash[i] of rank r, for every rank r (n u64 per rank,
 * the same n on every rank; d_hash may be d_out + rank * n).  Asynchronous
 * on `stream`; collective: every rank calls it, in the same order relative
 * to its other collectives.  -EIO if an earlier gather failed
 * asynchronously, -ECANCELED on an aborted communicator, -ETIMEDOUT (and
 * the communicator aborted) if RCCL's enqueue -- the connection setup with
 * the peers at the first gather -- does not finish in opts.comm_timeout_ms.
 * Completion: pptk_rx_comm_sync. */
int pptk_rx_allgather_hash(struct pptk_rx_ctx *ctx, const uint64_t *d_hash, uint64_t n,
                           uint64_t *d_out, void *stream);

/* Two streams that split the chip's CUs between the batches and the
 * gather that overlaps them (no reference counterpart: the reference has no
 * device; this belongs with the collective above).  RCCL's all-gather
 * kernel needs a whole CU per block on gfx950 (512 threads, 37 KB of LDS,
 * 248 VGPRs), and the receive grid fills every CU (persistent for
 * fixed-stride batches, oversubscribed for offset-described ones and the
 * small-frame kernel), so at each batch boundary one kernel takes CUs the
 * other was sized for and the two run one after the other (DESIGN.md
 * section 8).  *coll_stream (for
 * pptk_rx_allgather_hash) may use `coll_cus` CUs -- the same number in
 * every shader engine of every XCC -- and *rx_stream (for the batches) the
 * rest; the context sizes its receive grids for the rest from now on, on
 * any stream, and the rate limiter's one-launch path
 * (pptk_rx_permit_keys_device) its grid too; launch only the collective on
 * *coll_stream.  coll_cus: a multiple of 4 x the device's XCC count (32 on an
 * MI355X), below its CU count; -EINVAL otherwise.
 *
 * Order: split first, then create the communicator.  A communicator created
 * on a split context runs at most coll_cus RCCL blocks (channels) per
 * collective (ncclConfig_t.maxCTAs), so that all of them are resident on the
 * CUs left to it at once; that cap is fixed at creation, so a split to a
 * different CU count while the context has a communicator (or a creation in
 * progress) returns -EBUSY.  A split to the count the context already holds
 * returns the same two streams.  coll_cus 0 (streams NULL allowed) gives the
 * context's grids the whole chip again; the streams stay valid.
 *
 * The streams belong to the context: pptk_rx_ctx_destroy destroys them,
 * after its communicator (a gather stream destroyed before the communicator
 * made later device-wide waits or the teardown hang).
 * pptk_rx_stream_destroy returns -EBUSY for a stream its context still holds,
 * 0 (and does nothing) for one its context has destroyed, and destroys any
 * other stream. */
int pptk_rx_stream_split(struct pptk_rx_ctx *ctx, int coll_cus, void **rx_stream,
                         void **coll_stream);
int pptk_rx_stream_destroy(void *stream);

/* Buffer placement.  What the memory charges for the record writes beside
 * the frame-read stream depends on where the frame buffer and the record
 * buffer sit physically: the same C1500 launch, same kernel, same bytes,
 * takes 4.15-4.3 ms or 4.5-5.1 ms depending on the frame buffer, the record
 * buffer, or the pair.  For long-lived rings, set up
 * once: allocate a few candidate buffers (any allocator; spread apart, e.g.
 * with a few GB allocated between them), frame candidates each holding the
 * same representative batch, and let this run the batch on every (frames,
 * records) pair -- `reps` timed launches after one warm-up, pairs
 * interleaved -- and return the fastest pair in *best_frames / *best_recs;
 * keep those, free the others.  The frame candidates replace b->d_frames
 * (offsets in b->d_off are relative to it, so one descriptor array serves
 * all), the record candidates b->d_recs (b->d_recs32 for a compact batch)
 * and receive the batch's records; the rest of `b` is used as given.
 * Synchronous; nframes 1..16, nrecs 1..64, nframes * nrecs <= 256, reps
 * 1..100.  ms (nullable) receives nframes * nrecs median launch times,
 * frames-major.  Freeing the candidates not kept makes the driver scrub that
 * memory in the background (~30 GB/s measured); batches beside the scrub
 * run up to 9 % slower, so a latency-sensitive ring starts after it. */
int pptk_rx_place_buffers(struct pptk_rx_ctx *ctx, const struct pptk_rx_dev_batch *b,
                          const uint8_t *const *d_frames, int nframes, void *const *d_recs,
                          int nrecs, int reps, int *best_frames, int *best_recs, float *ms,
                          void *stream);

/* The record buffer alone (the frames as given in b->d_frames): as
 * pptk_rx_place_buffers with one frame candidate; *best = the record
 * candidate's index, ms = ncand median times. */
int pptk_rx_place_records(struct pptk_rx_ctx *ctx, const struct pptk_rx_dev_batch *b,
                          void *const *d_cands, int ncand, int reps, int *best, float *ms,
                          void *stream);

/* ---- Device rings owned by the library -----------------------------------
 * The default way to get the device frame ring and record ring of a
 * long-lived rx queue (an LDP/netmap ring lives for the process, reference
 * ldp/ldpnetmap.c:163-185): the library allocates frame and record
 * candidates spread apart in HBM, fills every frame candidate with a
 * synthetic batch of the ring's geometry (fixed-stride IPv4/TCP frames of
 * probe_len bytes, as many as fit, at most nrec), runs the receive
 * transform on every (frames, records) pair as pptk_rx_place_buffers does,
 * keeps the fastest pair and frees everything else -- so an application
 * that takes its rings from here gets the placed pair without managing
 * candidates (placement measured: C1500 4.03 ms placed against 4.80 ms on a
 * plain allocation of the same box).  The frame ring's
 * contents after the call are the probe batch: the application writes its
 * frames over it.  Synchronous (uses `stream` for the probe).
 * frame_cands 1..8 (0 = 3), rec_cands 1..16 (0 = 8), reps 1..20 (0 = 3),
 * probe_len 64..1536 (0 = 1500); candidates beyond the first pair are
 * allocated only as far as budget_bytes (0: 60 % of the free device memory)
 * allows.  Calls for one device run one at a time (several rx queues of a
 * GPU, a context each, setting up their rings together: each probe runs
 * alone and sizes its candidates from what the earlier calls kept; give
 * each queue a budget so the first ones do not take the memory the later
 * ones need for their candidates).  Freeing the
 * candidates not kept makes the driver scrub that memory in the background
 * (~20-30 GB/s; batches beside it run up to 9 % slower): with
 * PPTK_RX_RING_SETTLE the call sleeps until it is over (settle_ms), else
 * freed_bytes says how much was freed.  -EINVAL for a bad spec, -ENOMEM if
 * not even one pair fits.  Release with pptk_rx_ring_free. */
#define PPTK_RX_RING_SETTLE 0x1
/* The queue's batches will also write the dense flow hashes (d_hash, the
 * multi-GPU gather's send slice): the probe batches write them too (into a
 * scratch buffer freed with the candidates), so the pair kept is the best
 * for all three write streams, not for the records alone. */
#define PPTK_RX_RING_PROBE_HASH 0x2
struct pptk_rx_ring_spec {
  uint64_t frame_bytes;   /* frame ring bytes (the ring stays readable 64 B past it) */
  uint64_t nrec;          /* records the record ring holds (<= 2^32 - 1) */
  uint32_t rec_bytes;     /* 64 (struct pptk_rx_rec) or 32 (struct pptk_rx_rec32) */
  uint32_t probe_len;     /* probe frame length, 0 = 1500 */
  uint32_t frame_cands;   /* 0 = 3 */
  uint32_t rec_cands;     /* 0 = 8 */
  uint32_t reps;          /* timed probe launches per pair, 0 = 3 */
  uint32_t flags;         /* PPTK_RX_RING_SETTLE | PPTK_RX_RING_PROBE_HASH */
  uint64_t budget_bytes;  /* device memory the call may hold at once (candidates
                             and spacers included), 0 = 60 % of the free memory */
  uint64_t reserved;      /* 0 */
};
struct pptk_rx_ring {
  uint8_t *d_frames;      /* frame_bytes (+ 64 readable) */
  void *d_recs;           /* nrec * rec_bytes */
  uint64_t frame_bytes;
  uint64_t nrec;
  uint32_t rec_bytes;
  int32_t device;         /* the context's device */
  uint32_t frame_cands;   /* candidates actually probed */
  uint32_t rec_cands;
  int32_t chosen_frames;  /* the pair kept (candidate indices) */
  int32_t chosen_recs;
  float chosen_ms;        /* probe median launch time on the pair kept */
  float first_ms;         /* ... on candidate pair (0, 0): a plain allocation */
  uint64_t probe_frames;  /* frames in the probe batch */
  uint64_t freed_bytes;   /* candidates and spacers freed */
  uint32_t settle_ms;     /* slept for the scrub (PPTK_RX_RING_SETTLE) */
  uint32_t reserved;
};
int pptk_rx_ring_alloc(struct pptk_rx_ctx *ctx, const struct pptk_rx_ring_spec *spec,
                       struct pptk_rx_ring *ring, void *stream);
/* Frees both rings (on ring->device; the context need not exist any more)
 * and zeroes *ring.  Every batch using them must have completed. */
int pptk_rx_ring_free(struct pptk_rx_ring *ring);

/* The multi-GPU gather buffers, placed by the library like the rings: the
 * two (double-buffered) destinations of pptk_rx_allgather_hash for this
 * rank, nranks * per_rank u64 each, zeroed.  Where they sit decides what the
 * gather's writes -- the kernel's own hashes into the rank's slice and the
 * (nranks - 1) shards the collective lands while the next batch streams --
 * cost beside the frame stream.  Candidate regions
 * (each holding both buffers) are allocated apart; `b` (this rank's batch:
 * frames, records, geometry; b->d_hash is replaced by each buffer's slice in
 * turn) runs ~300 ms to warm the clocks, then `reps` rounds over the
 * candidates, each launch followed, on a second stream, by a device copy of
 * the bytes the gather would land (beside the next launch, as in an rx loop);
 * the region whose launches have the lowest median kernel time is kept,
 * everything else freed.  Synchronous; uses
 * `stream`.  Call after the rings are placed (the probe runs on them) and
 * after the scrub of what their placement freed is over
 * (PPTK_RX_RING_SETTLE): batches beside the scrub run up to 20 % slower on
 * every candidate alike, which hides the differences the probe looks for.
 * cands 1..16 (0 = 8), reps 1..20 (0 = 5); candidates as far as
 * budget_bytes (0: 50 % of the free memory) allows.  b->n <= per_rank.
 * Release with pptk_rx_gather_free. */
struct pptk_rx_gather_spec {
  uint64_t per_rank;      /* hashes each rank gathers (pptk_rx_shard_range) */
  int32_t nranks;
  int32_t rank;
  uint32_t cands;         /* candidate regions, 0 = 8 */
  uint32_t reps;          /* rounds over the candidates (two timed batches each), 0 = 5 */
  uint32_t flags;         /* PPTK_RX_RING_SETTLE */
  uint32_t reserved;      /* 0 */
  uint64_t budget_bytes;  /* 0 = 50 % of the free memory */
};
struct pptk_rx_gather {
  uint64_t *d_out[2];     /* the two gather buffers; rank r's slice of each
                             starts at d_out[k] + r * per_rank */
  uint64_t per_rank;
  int32_t nranks;
  int32_t rank;
  int32_t device;
  uint32_t cands;         /* candidate regions probed */
  int32_t chosen;         /* the region kept */
  float chosen_ms;        /* median probe kernel ms on the region kept */
  float first_ms;         /* ... on candidate 0: a plain allocation */
  uint32_t settle_ms;
  uint64_t freed_bytes;
  float cand_ms[16];      /* median probe kernel ms of every candidate probed */
};
int pptk_rx_gather_alloc(struct pptk_rx_ctx *ctx, const struct pptk_rx_dev_batch *b,
                         const struct pptk_rx_gather_spec *spec, struct pptk_rx_gather *gather,
                         void *stream);
int pptk_rx_gather_free(struct pptk_rx_gather *gather);

/* Library / build identification for the loaders. */
const char *pptk_rx_version(void);

/* The layout revision of the structs in this header (pptk_rx_opts,
 * pptk_rx_dev_batch, pptk_rx_ring_spec, ...).  It changes whenever one of
 * them changes size or meaning (round 5 added pptk_rx_ring_spec.budget_bytes
 * and .reserved; round 6 is the first revision with this check): a caller
 * compares pptk_rx_abi() with the PPTK_RX_ABI it was compiled against before
 * passing any struct, so a caller built against an older header is detected
 * instead of read past its structs' end. */
#define PPTK_RX_ABI 6
int pptk_rx_abi(void);

#ifdef __cplusplus
}
#endif

#endif /* PPTK_RX_H */
