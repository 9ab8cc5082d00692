// rx_kernel.hip -- the MI355X (gfx950) receive-transform kernels.
//
// One launch turns n Ethernet frames resident in HBM into n 64-byte records
// (include/pptk_rx.h).  Per record it computes exactly what the reference's
// per-packet primitives return for the same bytes:
//   ip_hdr_cksum_calc                 iphdr/ipcksum.c:39-49
//   tcp/udp_cksum_calc                iphdr/ipcksum.c:51-68, :117-134
//   tcp6/udp6_cksum_calc              iphdr/ipcksum.c:74-115, :140-181
//   ipv6_const_proto_hdr_2 (ext walk) iphdr/iphdr.h:804-860
//   siphash_buf (flow hash)           misc/siphash.h:214-229
//   ip_permitted/ipv6_permitted hash  iphash/iphash.c:157-162, :108-120
// composed as DESIGN.md "Record semantics" defines.
//
// Work decomposition (DESIGN.md "Kernel"):
//   * a wavefront owns a tile of 64 frames; lane q owns frame q of the tile
//     for parsing, hashing and the record store;
//   * the byte stream is summed by TEAMS of T lanes: in round r, team g sums
//     frame g*T + r with coalesced 16-byte loads (16*T contiguous bytes per
//     team per load), keeping S chunks per lane in registers; the loads of
//     round r+1 are issued before round r is summed;
//   * the first 128 aligned bytes of each frame are parked in an LDS image
//     (one 144-byte slot per frame) so the header fields never come from
//     HBM twice;
//   * one's-complement partial sums use v_dot2_u32_u16 (both 16-bit halves
//     of a dword in one op), are combined across the team with xor
//     shuffles, and are folded with end-around carry at the end.  The sum is
//     paired on even ABSOLUTE addresses; a region starting at an odd
//     address is corrected by one byte swap of the folded sum (RFC 1071
//     2.(B)), which is bit-exact (DESIGN.md "Checksum invariants").
#include "rx_internal.h"

#include <type_traits>

namespace pptk {

namespace {

constexpr int WAVE = 64;
constexpr int WPB = kWavesPerBlock;   // waves per block (4: 256 threads)
constexpr int IMG_CHUNKS = 8;     // 16-byte chunks parked in LDS per frame
#ifndef PPTK_RX_IMG_STRIDE
#define PPTK_RX_IMG_STRIDE 144
#endif
// LDS bytes per frame slot.  144 = 9 x 16: no b128 bank conflicts when a
// team parks its chunks; an odd dword pitch (148) instead spreads the
// per-frame phase's byte reads (every lane reading the same offset of its
// own frame) over all banks, at the price of parking chunks as dwords:
// measured equal (CMIX 2.717 vs 2.721 ms, C1500 4.161 vs 4.160 ms,
// in-process A/B) -- the per-frame phase is hidden behind the streaming --
// so 144 stays.
constexpr int IMG_STRIDE = PPTK_RX_IMG_STRIDE;
// Offset-described batches: where the team parks a frame's last chunk in the
// frame's slot (rx_kernel); PPTK_RX_TAIL_LDS=0 (A/B) corrects in the round.
#ifndef PPTK_RX_TAIL_LDS
#define PPTK_RX_TAIL_LDS 1
#endif
constexpr bool TAIL_LDS = PPTK_RX_TAIL_LDS;
constexpr int TAIL_OFF = 128;
static_assert(!TAIL_LDS || (IMG_STRIDE >= TAIL_OFF + 16 && IMG_STRIDE % 16 == 0),
              "the parked tail chunk lives past the 128-byte image");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// Explicit address spaces for every pointer the per-frame code dereferences:
// a pointer the compiler cannot place becomes a FLAT access, which counts in
// both vmcnt and lgkmcnt and may complete out of order, so every later wait
// on the streaming loads degrades to vmcnt(0) -- a drain of the prefetch.
#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t dot16(uint32_t w, uint32_t acc) {
  // acc + (w & 0xffff) + (w >> 16) in one VALU op
  return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w), (us2){1, 1}, acc, false);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
  return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

// End-around-carry fold of a 32-bit sum to 16 bits: identical to the
// reference's while (sum >> 16) loop (iphdr/ipcksum.h:17-25).
__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  return s;
}

// ip_cksum_postprocess: ntohs(~fold(sum)).
__device__ __forceinline__ uint32_t finish16(uint32_t s) {
  return bswap16(~fold16(s) & 0xffffu);
}

// 64-bit rotate left by 0 < b < 32 as two v_alignbit_b32 (full-rate 32-bit
// funnel shifts); b == 32 is a register swap.
template <int B>
__device__ __forceinline__ uint64_t rotl64(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if constexpr (B == 32) {
    return (uint64_t)hi | ((uint64_t)lo << 32);
  } else {
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - B);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - B);
    return (uint64_t)nlo | ((uint64_t)nhi << 32);
  }
}

// SipHash-2-4 on uint64_t state: 64-bit adds become one v_lshl_add_u64
// each.  (A variant on 32-bit halves with add/add-carry pairs, which saves
// the v_mov pairs that rotl-by-32 costs on aligned register pairs, measured
// 3 % slower on C64 -- 0.488 vs 0.474 ms, same box, in-process A/B.)
struct Sip {
  uint64_t v0, v1, v2, v3;
  __device__ __forceinline__ Sip(uint64_t k0, uint64_t k1)
      : v0(0x736f6d6570736575ULL ^ k0), v1(0x646f72616e646f6dULL ^ k1),
        v2(0x6c7967656e657261ULL ^ k0), v3(0x7465646279746573ULL ^ k1) {}
  __device__ __forceinline__ void round() {
    v0 += v1; v1 = rotl64<13>(v1); v1 ^= v0; v0 = rotl64<32>(v0);
    v2 += v3; v3 = rotl64<16>(v3); v3 ^= v2;
    v0 += v3; v3 = rotl64<21>(v3); v3 ^= v0;
    v2 += v1; v1 = rotl64<17>(v1); v1 ^= v2; v2 = rotl64<32>(v2);
  }
  // siphash_feed_u64 (misc/siphash.h:42-68), cROUNDS = 2
  __device__ __forceinline__ void block(uint64_t m) {
    v3 ^= m; round(); round(); v0 ^= m;
  }
  // final block (b | inlen << 56) + siphash_get (misc/siphash.h:70-121)
  __device__ __forceinline__ uint64_t finish(uint64_t last) {
    block(last);
    v2 ^= 0xff;
    round(); round(); round(); round();
    return v0 ^ v1 ^ v2 ^ v3;
  }
};

// A value loaded from global memory on a rare path, made ready before the
// paths join: the empty asm consumes it, so its vmcnt wait sits inside the
// rare branch.  Consumed after the join instead, the wait would be a
// vmcnt(0) on the common path -- a drain of the prefetched rounds.
__device__ __forceinline__ uint32_t settle(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// A frame as seen by a lane: bytes [0, lim) from the LDS image (frame byte k
// at img[m + k], image = aligned 16-byte chunks from floor16(frame start)),
// everything else straight from global memory.
struct FrameView {
  const LDS_AS uint8_t *img;
  const GLB_AS uint8_t *g;
  int m;
  int lim;

  __device__ __forceinline__ uint32_t u8(int k) const {
    if (k < lim) return (uint32_t)img[m + k];
    return settle((uint32_t)g[k]);
  }
  __device__ __forceinline__ uint32_t be16(int k) const {
    return (u8(k) << 8) | u8(k + 1);
  }
  // 4 frame bytes at offset k as a little-endian dword (hdr_get32h).
  __device__ __forceinline__ uint32_t le32(int k) const {
    if (k + 4 <= lim) {
      const int a = m + k;
      const LDS_AS uint32_t *p = (const LDS_AS uint32_t *)(img + (a & ~3));
      return __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)(a & 3));
    }
    return settle((uint32_t)g[k] | ((uint32_t)g[k + 1] << 8) | ((uint32_t)g[k + 2] << 16) |
                  ((uint32_t)g[k + 3] << 24));
  }
};

// Structural parse of one frame (the branchy part of DESIGN.md "Record
// semantics"): where L3/L4 are, what they are, and whether the L4 sum
// applies.  IP_OK / L4_OK / UDP_ZERO are decided later by the owning lane.
struct Parse {
  uint32_t flags, l3, ver, et, proto, rs, re;
  uint32_t fho;   // IPv6: offset of the last fragment header from L3 (0: none)
};

__device__ __forceinline__ bool is_v6_ext(uint32_t nh) {
  // is_ipv6_nexthdr, iphdr/iphdr.h:717-727
  return nh == 0 || nh == 60 || nh == 43 || nh == 44 || nh == 51;
}

__device__ __forceinline__ Parse parse_frame(const FrameView &v, uint32_t len) {
  Parse p = {0, 0, 0, 0, 0, 0, 0, 0};
  if (len < 14 || len > 65535) {
    p.flags = PPTK_RX_F_MALFORMED;
    return p;
  }
  uint32_t et = v.be16(12), l3 = 14;             // ether_type, iphdr.h:403
  if (et == 0x8100) {
    p.flags = PPTK_RX_F_VLAN;
    if (len < 18) {
      p.flags |= PPTK_RX_F_MALFORMED;
      return p;
    }
    et = v.be16(16);
    l3 = 18;
  }
  p.et = et;
  p.l3 = l3;
  uint32_t frag = 0;
  if (et == 0x0800) {
    if (len < l3 + 20) {
      p.flags |= PPTK_RX_F_MALFORMED;
      return p;
    }
    const uint32_t b0 = v.u8(l3);
    p.ver = b0 >> 4;                              // ip_version, :435
    const uint32_t ihl = (b0 & 15u) * 4u;         // ip_hdr_len, :876
    const uint32_t tl = v.be16(l3 + 2);           // ip_total_len, :943
    if (p.ver != 4 || ihl < 20 || tl < ihl || l3 + tl > len) {
      p.flags |= PPTK_RX_F_MALFORMED;
      return p;
    }
    p.flags |= PPTK_RX_F_PARSED;
    p.proto = v.u8(l3 + 9);                       // ip_proto, :1171
    frag = (v.be16(l3 + 6) & 0x3fffu) != 0;       // ip_frag_off/ip_more_frags
    p.rs = l3 + ihl;
    p.re = l3 + tl;
  } else if (et == 0x86dd) {
    p.flags |= PPTK_RX_F_IPV6;
    if (len < l3 + 40) {
      p.flags |= PPTK_RX_F_MALFORMED;
      return p;
    }
    p.ver = v.u8(l3) >> 4;
    const uint32_t tlen = v.be16(l3 + 4) + 40u;   // ipv6_payload_len + 40
    if (p.ver != 6 || l3 + tlen > len) {
      p.flags |= PPTK_RX_F_MALFORMED;
      return p;
    }
    // ipv6_const_proto_hdr_2, iphdr/iphdr.h:804-860, restated literally
    // (the length of the header at `off` is derived from the NEXT header's
    // type, as in the reference).
    uint32_t off = 40, nh = v.u8(l3 + 6);
    bool walked = false;
    while (is_v6_ext(nh)) {
      walked = true;
      if (off + 8u > tlen) {
        p.flags |= PPTK_RX_F_MALFORMED;
        p.fho = 0;
        return p;
      }
      if (nh == 44) {
        frag = 1;
        p.fho = off;
        if ((v.be16(l3 + off + 2) & 0xfff8u) > 0)
          break;
      }
      nh = v.u8(l3 + off);
      const uint32_t lf = v.u8(l3 + off + 1);
      const uint32_t extlen = nh == 44 ? 8u : (nh == 51 ? lf * 4u + 8u : lf * 8u + 8u);
      if (off + extlen > tlen) {
        p.flags |= PPTK_RX_F_MALFORMED;
        p.fho = 0;
        return p;
      }
      off = (off + extlen) & 0xffffu;
    }
    if (walked)
      p.flags |= PPTK_RX_F_V6_EXT;
    p.flags |= PPTK_RX_F_PARSED | PPTK_RX_F_IP_OK;
    p.proto = nh;
    p.rs = l3 + off;
    p.re = l3 + tlen;
  } else {
    return p;
  }
  if (frag)
    p.flags |= PPTK_RX_F_FRAGMENT;
  const uint32_t l4len = p.re - p.rs;
  if (!frag && ((p.proto == 6 && l4len >= 20) || (p.proto == 17 && l4len >= 8)))
    p.flags |= PPTK_RX_F_L4;
  return p;
}

// Byte-keep mask for bytes [lo, hi) of a dword (0 <= lo, hi <= 4).
__device__ __forceinline__ uint32_t bmask(int lo, int hi) {
  return (uint32_t)(((1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull));
}

// Sum (absolute-address pairing) the bytes of one aligned 16-byte chunk that
// fall inside the frame region [rs, re); `o` is the chunk's frame-relative
// offset (may be < 0).
__device__ __forceinline__ uint32_t sum_chunk(u32x4 c, int o, int rs, int re, uint32_t acc) {
  if (o >= rs && o + 16 <= re) {
    acc = dot16(c.x, acc);
    acc = dot16(c.y, acc);
    acc = dot16(c.z, acc);
    acc = dot16(c.w, acc);
  } else if (o + 16 > rs && o < re) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int od = o + 4 * d;
      acc = dot16(c[d] & bmask(min(max(rs - od, 0), 4), min(max(re - od, 0), 4)), acc);
    }
  }
  return acc;
}

// Team-round chunk sum: every chunk that starts in [start, len) is summed
// whole -- no byte masking at either end, so every lane runs the same four
// dot2 ops whatever its frame's length.  The chunk holding the frame's last
// byte therefore also adds the bytes [len, end of that chunk), which the
// same round takes off again (tail_past_end on the copy of that chunk the
// team's last lane holds, see load_round).  `o` = frame offset.
//
// MASKED instead masks the bytes past the end inside the chunk (no
// correction needed): the choice for fixed-stride batches, whose frames all
// end in the same one or two chunk slots of a round, so the masking runs on
// few slots -- cheaper there than the per-frame correction, whose extra load
// of the last chunk costs C1500 5 %.
template <bool MASKED = false>
__device__ __forceinline__ uint32_t sum_chunk_from(u32x4 c, int o, int start, int len,
                                                   uint32_t acc) {
  uint32_t t;
  if (!MASKED || o + 16 <= len) {
    t = dot16(c.x, 0);
    t = dot16(c.y, t);
    t = dot16(c.z, t);
    t = dot16(c.w, t);
  } else {
    t = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      t = dot16(c[d] & bmask(0, min(max(len - (o + 4 * d), 0), 4)), t);
  }
  return (o >= start && o < len) ? acc + t : acc;
}

// Frame offset of the aligned 16-byte chunk holding the last byte of a frame
// of `len` bytes that starts at `m` inside its chunk (len >= 1).
__device__ __forceinline__ int last_chunk_off(int m, int len) {
  return ((m + len - 1) & ~15) - m;
}

// What sum_chunk_from over-counted for this frame: the bytes past its end
// in its last chunk `tc`, if that chunk was summed (it starts at or after
// the team start ts); absolute pairing, like the team sums.  Branch-free
// (every lane of a round computes it): the keep-masks of the two 8-byte
// halves are one 64-bit shift each.
__device__ __forceinline__ uint32_t tail_past_end(u32x4 tc, int m, int len, int ts) {
  const uint32_t e8 = 8u * (uint32_t)((m + len) & 15);   // first bit past the end
  const uint64_t lo = e8 >= 64u ? 0ull : ~0ull << (e8 & 63u);
  const uint64_t hi = e8 <= 64u ? ~0ull : ~0ull << ((e8 - 64u) & 63u);
  uint32_t t = dot16(tc.x & (uint32_t)lo, 0u);
  t = dot16(tc.y & (uint32_t)(lo >> 32), t);
  t = dot16(tc.z & (uint32_t)hi, t);
  t = dot16(tc.w & (uint32_t)(hi >> 32), t);
  return (len > 0 && e8 != 0u && last_chunk_off(m, len) >= ts) ? t : 0u;
}

// First chunk boundary (frame offset) at or after byte 18 of a frame whose
// start sits at `m` inside its chunk: the team rounds sum [team_start, len);
// 18 <= team_start <= 33 < 34 <= every L4 start, so the owning lane only
// subtracts the few bytes [team_start, rs).
__device__ __forceinline__ int team_start_of(int m) {
  return (((m + 18 + 15) >> 4) << 4) - m;
}

// Absolute-pairing sum of frame bytes [a, b): image dwords first, bytes past
// the image from global memory (rare: long IPv6 chains, Ethernet padding
// beyond the parked 128 bytes).
__device__ uint32_t sum_abs(const FrameView &v, int a, int b) {
  uint32_t s = 0;
  const int hi_img = min(b, v.lim);
  if (a < hi_img) {
    const int lo_o = v.m + a, hi_o = v.m + hi_img;
    for (int d = lo_o & ~3; d < hi_o; d += 4) {
      const uint32_t w = *(const LDS_AS uint32_t *)(v.img + d);
      s = dot16(w & bmask(min(max(lo_o - d, 0), 4), min(max(hi_o - d, 0), 4)), s);
    }
  }
  for (int k = max(a, v.lim); k < b; ++k)
    s += settle((uint32_t)v.g[k]) << (((v.m + k) & 1) * 8);
  return s;
}

// Frame chunk load; frames are read once, so optionally non-temporal.
template <bool NT>
__device__ __forceinline__ u32x4 ldc(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// Sum over a team of T lanes, complete in every lane of the team.  Teams
// inside a row of 16 lanes by DPP adds (no LDS crossbar traffic): quad_perm
// [1,0,3,2] and [2,3,0,1] (quads), row_half_mirror (lane i <-> 7 - i: the
// two quads of an 8-lane half), row_mirror (i <-> 15 - i: the two halves):
// CMIX T16S6 2.743 -> 2.717 ms, IMIX 1.696 -> 1.653 ms, C1500 T16S6 4.330
// -> 4.312 ms (in-process A/B, profiles/r03/dpp).  Teams of 32 and 64 lanes
// keep xor shuffles for every step (C1500 T32S3 4.184 vs 4.208 ms with the
// row steps as DPP).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
  return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true);
}
template <int T>
__device__ __forceinline__ uint32_t team_sum(uint32_t x) {
  if constexpr (T >= 32) {
#pragma unroll
    for (int d = T / 2; d >= 1; d >>= 1)
      x += __shfl_xor(x, d, T);
    return x;
  }
  if constexpr (T >= 2) x = dpp_add<0xb1>(x);    // quad_perm [1,0,3,2]
  if constexpr (T >= 4) x = dpp_add<0x4e>(x);    // quad_perm [2,3,0,1]
  if constexpr (T >= 8) x = dpp_add<0x141>(x);   // row_half_mirror
  if constexpr (T >= 16) x = dpp_add<0x140>(x);  // row_mirror
  return x;
}

// Per-lane descriptor of the lane's frame in a tile.
struct Desc {
  uint64_t base;
  uint32_t len, idx;
};

// Descriptors come either from arithmetic (FIXED: frame i at i * stride,
// fixed_len bytes, identity order -- no memory traffic, nothing to wait for)
// or from the d_perm / d_off / d_len arrays (GATHER).  The GATHER loads are
// unconditional and their results are combined arithmetically (absent arrays
// and lanes past n read zeros from a.zero, see RxKArgs): a load under a
// branch or feeding a select leaves the compiler an unknown number of loads
// in flight, and it answers with a full vmcnt(0) drain of the streaming
// rounds.  Past-the-end lanes describe frame 0 with idx = ~0 (no record).
template <bool GATHER>
__device__ __forceinline__ uint32_t desc_idx(const RxKArgs &a, uint64_t tile, int lane) {
  const uint64_t i = tile * WAVE + lane;
  const uint32_t bad = 0u - (uint32_t)(i >= a.n);
  if constexpr (GATHER) {
    const uint32_t ic = (uint32_t)i & ~bad;
    const uint32_t v = a.perm_ld[ic & a.perm_msk];
    return (v + (ic & ~a.perm_msk)) | bad;
  } else {
    return (uint32_t)i | bad;
  }
}

template <bool GATHER>
__device__ __forceinline__ Desc desc_fill(const RxKArgs &a, uint32_t idx, uint64_t tile, int lane) {
  Desc d;
  d.idx = idx;
  const uint32_t ic = idx == 0xffffffffu ? 0u : idx;
  if constexpr (GATHER) {
    // descriptors by frame index, or (by_pos) by processing position
    const uint64_t pos = tile * WAVE + lane;
    const uint32_t pc = pos < a.n ? (uint32_t)pos : 0u;
    const uint32_t key = a.by_pos ? pc : ic;
    const uint64_t o = a.off_ld[key & a.off_msk];
    const uint32_t l = a.len_ld[key & a.len_msk];
    d.base = o + (uint64_t)ic * a.stride_g;
    d.len = l + a.fixed_g;
  } else {
    (void)tile;
    (void)lane;
    d.base = (uint64_t)ic * a.stride;
    d.len = a.fixed_len;
  }
  return d;
}

template <bool GATHER>
__device__ __forceinline__ Desc load_desc(const RxKArgs &a, uint64_t tile, int lane) {
  return desc_fill<GATHER>(a, desc_idx<GATHER>(a, tile, lane), tile, lane);
}

// One round's staged chunks for a team: S chunks per lane + the frame.
template <int S>
struct Buf {
  u32x4 v[S];
  uint64_t pb;
  uint32_t pl;
};

// AL = log2 of the chunk-grid alignment: 4 -> chunks on 16-byte boundaries
// of the frame buffer, 7 -> on 128-byte (cache line) boundaries, so a team's
// 16*T contiguous bytes are whole lines (no line split between two loads).
template <int T, int S, int AL, bool NT>
__device__ __forceinline__ Buf<S> load_round(const RxKArgs &a, const Desc &d, int r, int g,
                                             int j) {
  Buf<S> b;
  const int q = g * T + r;
  b.pb = __shfl(d.base, q);
  b.pl = __shfl(d.len, q);
  const int m = (int)(b.pb & ((1u << AL) - 1));
  const u32x4 *c0 = (const u32x4 *)(a.frames + (b.pb - (uint64_t)m));
  const int nch = (m + (int)b.pl + 15) >> 4;
  const int clast = nch > 0 ? nch - 1 : 0;
  // Unconditional loads (chunks past the frame re-read its last chunk):
  // branch-free loads let the compiler count vmcnt precisely, so the D
  // rounds in flight are not drained at every use.
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int c = s * T + j;
    // Non-temporal streaming: the last 8 chunks of the window -- a
    // full-window frame's last line, which the next frame's first chunk
    // shares -- with a temporal load, so that line stays in L2 for the next
    // round instead of being fetched again after the non-temporal load let it
    // go (C1500: 201.2 M -> 197.0 M 128-byte reads per launch, the SOL
    // kernel's 196.6 M; 4.092 -> 4.042 ms, profiles/r04/c1500_tail/); the
    // other lanes of each of the two loads re-read a neighbour's chunk
    // (coalesced in the instruction: no extra traffic)
    if (NT && s == S - 1 && T >= 8) {
      const bool tl = j >= T - 8;
      const int cn = tl ? (S - 1) * T + (T - 9) : c;    // NT instruction: tail lanes -> lane T-9's chunk
      const int ct = tl ? c : (S - 1) * T + (T - 8);    // temporal one: other lanes -> lane T-8's chunk
      const u32x4 a = ldc<true>(c0 + min(cn, clast));
      const u32x4 t = c0[min(ct, clast)];
      b.v[s] = tl ? t : a;
      continue;
    }
    b.v[s] = ldc<NT>(c0 + min(c, clast));   // bytes past the frame are masked at use
  }
  return b;
}

// Tx, in place (offset-described batches; fixed-stride ones run in two
// passes through RxKArgs::txside and tx_apply_kernel): store the checksum
// fields txp[k] (frame offsets, -1 = none) with values txv[k], network byte
// order.  Each field is a 2-byte write into a
// line this wave read long before, so every field costs the memory a whole
// write granule; writing 16/32/64-byte granules around the fields from the
// patched LDS image instead was measured no faster, nor were
// 16-bit stores of the aligned fields (C1500 5.329 vs 5.327 ms, CMIX 3.008
// vs 3.004 ms, tools/ab_tx.py), and non-temporal 16-bit stores were much
// slower (5.90 vs 5.36 ms, 3.63 vs 3.13 ms), so plain byte stores it is.
__device__ __forceinline__ void tx_store(const RxKArgs &a, uint64_t base, const int txp[2],
                                         const uint32_t txv[2]) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (txp[k] < 0) continue;
    uint8_t *fw = a.frames_w + base + txp[k];
    fw[0] = (uint8_t)(txv[k] >> 8);
    fw[1] = (uint8_t)txv[k];
  }
}

// The 16 record words of struct pptk_rx_rec (include/pptk_rx.h) of one frame,
// before the compact projection.
struct LaneRec {
  uint32_t w[16];
  uint64_t fh;
  uint32_t flags;
  u32x4 frag;   // struct pptk_rx_frag (only when RxKArgs::frag is set)
  uint64_t tx;  // two-pass tx: the txside entry (only when RxKArgs::txside is set)
};

constexpr uint64_t kTxNone = 0x0000ffff0000ffffull;   // no field to set

// The txside entry of a frame: (offset, value) of the IPv4 header checksum
// field and of the L4 checksum field, 0xffff offsets for none.
__device__ __forceinline__ uint64_t tx_entry(const int txp[2], const uint32_t txv[2]) {
  uint64_t e = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint64_t f = txp[k] < 0 ? 0xffffull : ((uint64_t)txp[k] | ((uint64_t)txv[k] << 16));
    e |= f << (32 * k);
  }
  return e;
}

// struct pptk_rx_frag (include/pptk_rx.h) of a parsed frame: the IPv4
// fragment fields (ip_id :1093, ip_frag_off :1124, ip_more_frags :1023,
// ip_dont_frag :1040 of iphdr/iphdr.h) or those of the last IPv6 fragment
// header the walk met (ipv6_const_proto_hdr_2's frag_hdr_off and
// proto_hdr_off_from_frag, :804-860; ipv6_frag_off / ipv6_more_frags
// :727-737).
__device__ __forceinline__ u32x4 frag_words(const FrameView &v, const Parse &p) {
  u32x4 r = (u32x4){0u, 0u, 0u, 0u};
  if ((p.flags & (PPTK_RX_F_PARSED | PPTK_RX_F_MALFORMED)) != PPTK_RX_F_PARSED) return r;
  const int l3 = (int)p.l3;
  uint32_t ident, foff, fl, dlen, nh, fho = 0, pofs = 0;
  if (!(p.flags & PPTK_RX_F_IPV6)) {
    const uint32_t fw = v.be16(l3 + 6);
    ident = v.be16(l3 + 4);
    foff = ((fw & 0x1fffu) * 8u) & 0xffffu;
    fl = ((p.flags & PPTK_RX_F_FRAGMENT) ? PPTK_RX_FRAG_IS : 0u) |
         ((fw & 0x2000u) ? PPTK_RX_FRAG_MF : 0u) | ((fw & 0x4000u) ? PPTK_RX_FRAG_DF : 0u);
    dlen = p.re - p.rs;
    nh = p.proto;
  } else {
    if (p.fho == 0) return r;
    fho = p.fho;
    const int fh = l3 + (int)fho;
    const uint32_t fw = v.be16(fh + 2);
    ident = (v.be16(fh + 4) << 16) | v.be16(fh + 6);
    foff = fw & 0xfff8u;
    fl = PPTK_RX_FRAG_IS | PPTK_RX_FRAG_V6 | ((fw & 1u) ? PPTK_RX_FRAG_MF : 0u);
    dlen = (p.re - p.l3) - (fho + 8u);
    nh = v.u8(fh);
    pofs = ((p.rs - p.l3) - fho) & 0xffffu;
  }
  r.x = ident;
  r.y = foff | (dlen << 16);
  r.z = fho | (pofs << 16);
  r.w = nh | (fl << 8);
  return r;
}

// The per-frame part of the transform for a frame in any layout: structural
// parse, IPv4 header checksum, L4 checksum from the team sum `my_sum` of the
// frame bytes [team_start_of(v.m), len), flow hash, bucket hash, and (tx
// batches) the checksum stores.  DESIGN.md "Record semantics" steps 1-9.
// `my_sum` = the team sum of the frame bytes [team_start_of(v.m), end of the
// chunk holding the last byte) when `tailc` is that last chunk (the bytes
// past the end are taken off here), or of exactly [team_start, len) when
// `tailc` is zero.
__device__ __forceinline__ void lane_generic(const RxKArgs &a, const FrameView &v, uint32_t len,
                                             uint64_t base, uint32_t my_sum, u32x4 tailc,
                                             LaneRec &o) {
  const int m = v.m;
  const Parse p = parse_frame(v, len);
  if (a.frag)
    o.frag = frag_words(v, p);
  o.tx = kTxNone;
  uint32_t flags = p.flags;
  const uint32_t l3 = p.l3, rs = p.rs, re = p.re, proto = p.proto;
  uint32_t *w = o.w;
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = 0;
  uint64_t fh = 0;
  if (flags & PPTK_RX_F_MALFORMED) {
    flags &= PPTK_RX_F_MALFORMED | PPTK_RX_F_VLAN | PPTK_RX_F_IPV6;
  } else if (flags & PPTK_RX_F_PARSED) {
    const bool v6 = flags & PPTK_RX_F_IPV6;
    uint32_t s0, s1 = 0, s2 = 0, s3 = 0, d0, d1 = 0, d2 = 0, d3 = 0;
    int txp[2] = {-1, -1};          // tx: frame offsets of the fields to set
    uint32_t txv[2] = {0, 0};
    uint32_t ipc = 0;
    // [ts, rs): the header bytes between the team start (18 <= ts <= 33) and
    // the L4 start (>= 34), absolute pairing; the L4 correction subtracts
    // them, and for IPv4 they are most of the header sum
    const int ts = team_start_of(m);
    const uint32_t s_tr = sum_abs(v, ts, (int)rs);
    if (v6) {
      s0 = v.le32(l3 + 8);  s1 = v.le32(l3 + 12); s2 = v.le32(l3 + 16); s3 = v.le32(l3 + 20);
      d0 = v.le32(l3 + 24); d1 = v.le32(l3 + 28); d2 = v.le32(l3 + 32); d3 = v.le32(l3 + 36);
    } else {
      s0 = v.le32(l3 + 12);
      d0 = v.le32(l3 + 16);
      // ip_hdr_cksum_calc over ihl = rs - l3 bytes: [l3, ts) + [ts, rs), a
      // sum of sums (no subtraction, so exactly 0 only for all-zero bytes);
      // absolute pairing, byte-swapped to the header's own pairing when the
      // header starts at an odd address (RFC 1071 2.(B))
      uint32_t hs = fold16(sum_abs(v, (int)l3, ts) + s_tr);
      if ((m + (int)l3) & 1)
        hs = bswap16(hs);
      ipc = finish16(hs);
      if (ipc == 0)
        flags |= PPTK_RX_F_IP_OK;
      if (a.frames_w) {
        // tx: ip_set_hdr_cksum_calc (iphdr/ipcksum.h:101-111) -- the sum
        // with the field zeroed is hs - field; the version nibble makes
        // it positive, so the mod-0xffff residue is exact
        const uint32_t fld = v.le32((int)l3 + 8) >> 16;
        txp[0] = (int)l3 + 10;
        txv[0] = finish16(fold16(hs) + (0xffffu - fld));
      }
    }
    uint32_t ports = 0, l4c = 0;
    if (flags & PPTK_RX_F_L4) {
      ports = v.le32((int)rs);
      const uint32_t l4len = re - rs;
      uint32_t ps = dot16(s0, 0);
      ps = dot16(s1, ps); ps = dot16(s2, ps); ps = dot16(s3, ps);
      ps = dot16(d0, ps); ps = dot16(d1, ps); ps = dot16(d2, ps); ps = dot16(d3, ps);
      ps += bswap16(proto) + bswap16(l4len);   // > 0: proto is 6 or 17
      // region [rs, re) = [ts, L) - [len, L) - [ts, rs) - [re, len), mod
      // 0xffff, where the team sum covered [ts, L): L = len, or the end of
      // the chunk holding the last byte (tailc: tail_past_end is [len, L))
      uint32_t rsum = fold16(my_sum) + (0xffffu - fold16(tail_past_end(tailc, m, (int)len, ts)));
      rsum += 0xffffu - fold16(s_tr);
      if (re < len)
        rsum += 0xffffu - fold16(sum_abs(v, (int)re, (int)len));
      rsum = fold16(rsum);
      if ((m + (int)rs) & 1)
        rsum = bswap16(rsum);   // region starts at an odd address
      l4c = finish16(ps + rsum);
      if (l4c == 0)
        flags |= PPTK_RX_F_L4_OK;
      if (a.frames_w) {
        // tx: tcp/udp(6)_set_cksum_calc (iphdr/ipcksum.h:127-211) -- the
        // region sum minus the transmitted field (an even offset of the
        // region, so one of its words); the pseudo-header keeps the
        // total positive
        const int f = (int)rs + (proto == 6 ? 16 : 6);
        const uint32_t fld = v.u8(f) | (v.u8(f + 1) << 8);
        txp[1] = f;
        txv[1] = finish16(ps + fold16(rsum + (0xffffu - fld)));
      }
      if (proto == 17 && (v.le32((int)rs + 4) >> 16) == 0)
        flags |= PPTK_RX_F_UDP_ZERO;
    }
    if (a.txside)
      o.tx = tx_entry(txp, txv);
    else if (a.frames_w && !(kDiag && (a.tune & 512u)))   // bit 9: diagnostics, no tx writes
      tx_store(a, base, txp, txv);
    uint32_t bucket = 0;
    if (a.recs || a.recs32 || a.hash) {   // tx batches need no hashes
      Sip sh(a.k0, a.k1);
      sh.block((uint64_t)s0 | ((uint64_t)s1 << 32));
      sh.block((uint64_t)s2 | ((uint64_t)s3 << 32));
      sh.block((uint64_t)d0 | ((uint64_t)d1 << 32));
      sh.block((uint64_t)d2 | ((uint64_t)d3 << 32));
      sh.block((uint64_t)ports | ((uint64_t)proto << 32));
      fh = sh.finish(40ull << 56);
      if (!v6 && a.bucket4) {
        const uint32_t host = __builtin_bswap32(s0) & a.mask4;
        Sip bh(a.k0, a.k1);
        bh.block((uint64_t)host);
        bucket = (uint32_t)bh.finish(8ull << 56) & a.hash_mask;
      } else if (v6 && a.bucket6) {
        Sip bh(a.k0, a.k1);
        bh.block(((uint64_t)s0 | ((uint64_t)s1 << 32)) & a.mask6_0);
        bh.block(((uint64_t)s2 | ((uint64_t)s3 << 32)) & a.mask6_1);
        bucket = (uint32_t)bh.finish(16ull << 56) & a.hash_mask;
      }
    }
    w[0] = (uint32_t)fh;
    w[1] = (uint32_t)(fh >> 32);
    w[2] = s0; w[3] = s1; w[4] = s2; w[5] = s3;
    w[6] = d0; w[7] = d1; w[8] = d2; w[9] = d3;
    w[10] = bswap16(ports & 0xffffu) | (bswap16(ports >> 16) << 16);
    w[11] = ipc | (l4c << 16);
    w[12] = rs | ((re - rs) << 16);
    w[13] = proto << 8;
    w[14] = bucket;
  }
  w[13] |= l3 | (flags << 16);
  w[15] = p.et | (p.ver << 16);
  o.fh = fh;
  o.flags = flags;
}

// The common case parsed from registers: frame bytes 0..63 as little-endian
// dwords d[0..15] (frame start 16-byte aligned, bytes >= len arbitrary), an
// untagged IPv4 frame with a 20-byte header that is not a fragment and lies
// within the frame.  Returns false for every other frame (lane_generic
// handles it); otherwise fills the same words lane_generic would: the fixed
// offsets are Ethernet 14 + IPv4 20, so L4 starts at 34 (an even address:
// no byte swap) and the team-start correction disappears.
__device__ __forceinline__ bool lane_fast(const RxKArgs &a, const uint32_t d[16], uint32_t len,
                                          LaneRec &o) {
  const uint32_t tl = bswap16(d[4] & 0xffffu);            // ip_total_len
  // ethertype 0x0800 (bytes 12-13), version 4 + IHL 5 (byte 14), no MF /
  // offset (bytes 20-21), 20 <= tl, 14 + tl <= len
  if ((d[3] & 0x00ffffffu) != 0x00450008u || (d[5] & 0xff3fu) != 0u || tl < 20u ||
      tl + 14u > len)
    return false;
  const uint32_t proto = d[5] >> 24;
  const uint32_t re = 14u + tl, l4len = tl - 20u;
  uint32_t flags = PPTK_RX_F_PARSED;
  // ip_hdr_cksum_calc over bytes 14..33
  uint32_t hs = dot16(d[3] & 0xffff0000u, 0);
  hs = dot16(d[4], hs); hs = dot16(d[5], hs); hs = dot16(d[6], hs); hs = dot16(d[7], hs);
  hs = dot16(d[8] & 0xffffu, hs);
  const uint32_t ipc = finish16(hs);
  if (ipc == 0) flags |= PPTK_RX_F_IP_OK;
  const uint32_t s0 = __builtin_amdgcn_alignbyte(d[7], d[6], 2u);   // bytes 26..29
  const uint32_t d0 = __builtin_amdgcn_alignbyte(d[8], d[7], 2u);   // bytes 30..33
  uint32_t ports = 0, l4c = 0;
  if ((proto == 6u && l4len >= 20u) || (proto == 17u && l4len >= 8u)) {
    flags |= PPTK_RX_F_L4;
    ports = __builtin_amdgcn_alignbyte(d[9], d[8], 2u);            // bytes 34..37
    uint32_t ps = dot16(s0, 0);
    ps = dot16(d0, ps);
    ps += bswap16(proto) + bswap16(l4len);
    uint32_t rsum;
    if (re >= 64u) {      // region [34, 64)
      rsum = dot16(d[8] & 0xffff0000u, 0);
#pragma unroll
      for (int k = 9; k < 16; ++k) rsum = dot16(d[k], rsum);
    } else {              // Ethernet padding or a shorter frame: [34, re)
      rsum = 0;
#pragma unroll
      for (int k = 8; k < 16; ++k)
        rsum = dot16(d[k] & bmask(min(max(34 - 4 * k, 0), 4), min(max((int)re - 4 * k, 0), 4)),
                     rsum);
    }
    l4c = finish16(ps + rsum);
    if (l4c == 0) flags |= PPTK_RX_F_L4_OK;
    if (proto == 17u && (d[10] & 0xffffu) == 0u) flags |= PPTK_RX_F_UDP_ZERO;
  }
  Sip sh(a.k0, a.k1);
  sh.block((uint64_t)s0);
  sh.block(0);
  sh.block((uint64_t)d0);
  sh.block(0);
  sh.block((uint64_t)ports | ((uint64_t)proto << 32));
  const uint64_t fh = sh.finish(40ull << 56);
  uint32_t bucket = 0;
  if (a.bucket4) {
    Sip bh(a.k0, a.k1);
    bh.block((uint64_t)(__builtin_bswap32(s0) & a.mask4));
    bucket = (uint32_t)bh.finish(8ull << 56) & a.hash_mask;
  }
  uint32_t *w = o.w;
  w[0] = (uint32_t)fh;
  w[1] = (uint32_t)(fh >> 32);
  w[2] = s0; w[3] = 0; w[4] = 0; w[5] = 0;
  w[6] = d0; w[7] = 0; w[8] = 0; w[9] = 0;
  w[10] = bswap16(ports & 0xffffu) | (bswap16(ports >> 16) << 16);
  w[11] = ipc | (l4c << 16);
  w[12] = 34u | (l4len << 16);
  w[13] = 14u | (proto << 8) | (flags << 16);
  w[14] = bucket;
  w[15] = 0x0800u | (4u << 16);
  o.fh = fh;
  o.flags = flags;
  return true;
}

// How the kernel writes the dense flow-hash array (A/B builds: 0 plain
// per-lane stores, 1 non-temporal per-lane stores, 2 staged beside the
// record and stored by flush_records as one run per tile).
#ifndef PPTK_RX_HASH_MODE
#define PPTK_RX_HASH_MODE 2
#endif


// Record of frame `idx`: the optional dense flow-hash word, then the record
// (64 bytes, or the 32-byte compact projection) either parked in the lane's
// LDS slot `st` for flush_records (batch order) or stored directly
// (permuted order: records scatter).
__device__ __forceinline__ void emit_record(const RxKArgs &a, const LaneRec &o, uint32_t idx,
                                            LDS_AS u32x4 *st, bool stage) {
  const uint32_t *w = o.w;
  // The dense flow hash (the all-gather's send slice).  Beside the frame
  // stream, where the memory charges writes by their burst (DESIGN.md 7
  // "Placement"), it goes out like the records: non-temporal, and (batch
  // order) parked in the record slot's spare 16 bytes and stored by the
  // flush as one 512-byte run per tile next to the tile's records.
  if (a.hash) {
    if (PPTK_RX_HASH_MODE == 2 && stage && !a.perm)
      *(LDS_AS uint64_t *)(st + 4) = o.fh;
    else if (PPTK_RX_HASH_MODE >= 1 && (a.tune & 32u))
      __builtin_nontemporal_store(o.fh, (GLB_AS uint64_t *)a.hash + idx);
    else
      a.hash[idx] = o.fh;
  }
  if (a.key)   // rate-limiter key: src_bucket (word 14), IPv6 bit 31; ~0 unparsed
    a.key[idx] = !(o.flags & PPTK_RX_F_PARSED) ? 0xffffffffu
                 : (o.flags & PPTK_RX_F_IPV6)  ? (w[14] | 0x80000000u)
                                               : w[14];
  if (a.frag)
    ((GLB_AS u32x4 *)a.frag)[idx] = o.frag;
  if (!a.recs && !a.recs32)
    return;   // tx batch: no records
  const bool c32 = a.recs32 != nullptr;   // compact 32-byte records
  u32x4 r0, r1, r2, r3;
  if (c32) {   // struct pptk_rx_rec32: a projection of the same words
    const bool v6 = o.flags & PPTK_RX_F_IPV6;
    r0 = (u32x4){w[0], w[1], v6 ? 0u : w[2], v6 ? 0u : w[6]};
    r1 = (u32x4){w[10], (w[13] >> 16) | (((w[13] >> 8) & 0xffu) << 16) | (w[13] << 24),
                 w[12], w[14]};
    r2 = r3 = (u32x4){0u, 0u, 0u, 0u};
  } else {
    r0 = (u32x4){w[0], w[1], w[2], w[3]};
    r1 = (u32x4){w[4], w[5], w[6], w[7]};
    r2 = (u32x4){w[8], w[9], w[10], w[11]};
    r3 = (u32x4){w[12], w[13], w[14], w[15]};
  }
  if (stage) {
    st[0] = r0; st[1] = r1;
    if (!c32) { st[2] = r2; st[3] = r3; }
  } else {
    GLB_AS u32x4 *dst = (GLB_AS u32x4 *)(c32 ? (GLB_AS uint8_t *)a.recs32 + (uint64_t)idx * 32u
                                             : (GLB_AS uint8_t *)a.recs + (uint64_t)idx * 64u);
    dst[0] = r0; dst[1] = r1;
    if (!c32) { dst[2] = r2; dst[3] = r3; }
  }
}

// The tile's 64 records, parked in the wave's LDS at an 80-byte pitch, are
// stored with whole-record runs per instruction.  Batch order: they are one
// contiguous 4 KB run (2 KB compact) in memory, so each store instruction
// writes 1 KB contiguously instead of 64 scattered 16-byte pieces.
// Permuted order (SCATTER: the binned processing order of
// pptk_rx_batch_device_mixed, records land at the frames' own indices):
// 4 (compact: 2) consecutive lanes write one record's 64 (32) bytes, so an
// instruction touches 16 (32) records of whole 64-byte (32-byte) runs
// instead of one 16-byte piece of each of 64 records.  `my_idx` is the
// lane's frame index (~0: no record).
__device__ __forceinline__ void flush_records(const RxKArgs &a, const LDS_AS uint8_t *wimg, uint64_t tile,
                                              int lane, uint32_t my_idx, bool scatter,
                                              LDS_AS u32x4 *stash = nullptr) {
  const bool c32 = a.recs32 != nullptr;
  __builtin_amdgcn_wave_barrier();
  const LDS_AS u32x4 *st = (const LDS_AS u32x4 *)wimg;
  GLB_AS uint8_t *rbase = c32 ? (GLB_AS uint8_t *)a.recs32 : (GLB_AS uint8_t *)a.recs;
  GLB_AS u32x4 *dst = (GLB_AS u32x4 *)(rbase + tile * (uint64_t)WAVE * (c32 ? 32u : 64u));
  const uint64_t nrec = min((uint64_t)WAVE, a.n - tile * WAVE);
  const int lg = c32 ? 1 : 2;                 // log2 16-byte pieces per record
  int kmax = c32 ? 2 : 4;
  if (kDiag && (a.tune & 128u)) kmax >>= 1;   // bit 7: diagnostics, half the bytes
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = k * WAVE + lane;   // 16-byte piece e of the tile's records
    const int r = e >> lg;
    const int piece = e & ((1 << lg) - 1);
    GLB_AS u32x4 *d = dst + e;
    bool live = (uint64_t)r < nrec;
    if (scatter) {
      const uint32_t ridx = __shfl(my_idx, r & (WAVE - 1));
      live = ridx != 0xffffffffu;
      d = (GLB_AS u32x4 *)(rbase + (uint64_t)ridx * (c32 ? 32u : 64u)) + piece;
    }
    if (live && k < kmax) {
      const u32x4 val = st[r * 5 + piece];
      if (stash) {                   // global write phases: held in LDS, stored later
        stash[e] = val;
      } else if (a.tune & 64u) {     // bit 6: write-through, drop from L2 (sc1)
        GLB_AS uint64_t *d8 = (GLB_AS uint64_t *)d;
        __hip_atomic_store(d8, (uint64_t)val.x | ((uint64_t)val.y << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d8 + 1, (uint64_t)val.z | ((uint64_t)val.w << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      } else if (a.tune & 32u) {     // bit 5: non-temporal stores
        asm volatile("" ::: "memory");
        __builtin_nontemporal_store(val, d);
      } else {
        *d = val;
      }
    }
  }
  // the tile's flow hashes (parked in each record slot's spare 16 bytes):
  // lanes 0..31 store two records' hashes each, one 512-byte run
  // (the same condition as emit_record's: !a.perm -- a permuted batch
  // stored its hashes per lane)
  if (PPTK_RX_HASH_MODE == 2 && a.hash && !scatter && !a.perm && lane < WAVE / 2) {
    const uint32_t r0 = 2u * (uint32_t)lane;
    if ((uint64_t)r0 < nrec) {
      const uint64_t h0 = *(const LDS_AS uint64_t *)(st + r0 * 5 + 4);
      GLB_AS uint64_t *hd = (GLB_AS uint64_t *)a.hash + tile * (uint64_t)WAVE + r0;
      if ((uint64_t)r0 + 1 < nrec && ((uintptr_t)hd & 15u) == 0) {
        const uint64_t h1 = *(const LDS_AS uint64_t *)(st + (r0 + 1) * 5 + 4);
        const u64x2 v = {h0, h1};
        if (a.tune & 32u)
          __builtin_nontemporal_store(v, (GLB_AS u64x2 *)hd);
        else
          *(GLB_AS u64x2 *)hd = v;
      } else {
        hd[0] = h0;
        if ((uint64_t)r0 + 1 < nrec) hd[1] = *(const LDS_AS uint64_t *)(st + (r0 + 1) * 5 + 4);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// Global write phases (RxKArgs::phase_ticks != 0).  The record writes beside
// the frame stream cost the memory more than their bytes (DESIGN.md section
// 7 "Placement"), and less when every wave's come together: a tile's record
// run waits in the wave's LDS stash until the chip-wide clock
// (s_memrealtime, 100 MHz, one clock for every CU) passes the next multiple
// of phase_ticks -- checked after every streaming round -- or until the next
// tile's run needs the stash, so the waves' record writes fall in the first
// microseconds of each period instead of each at its own tile end.  The
// host sets the period to ~0.75 of a tile's expected duration (rx_capi.hip
// phase_ticks_for): C1500 4.036 -> 3.954 ms and 4.370 -> 4.102 ms on two
// boxes, CMIX 2.541 -> 2.510 ms (profiles/r05/v, w).
__device__ __forceinline__ uint64_t phase_deadline(uint32_t period) {
  const uint64_t rt = __builtin_amdgcn_s_memrealtime();
  return rt - rt % period + period;
}
__device__ __forceinline__ void flush_stash(const RxKArgs &a, const LDS_AS u32x4 *stash, uint64_t tile,
                                            int lane) {
  const bool c32 = a.recs32 != nullptr;
  GLB_AS uint8_t *rbase = c32 ? (GLB_AS uint8_t *)a.recs32 : (GLB_AS uint8_t *)a.recs;
  GLB_AS u32x4 *dst = (GLB_AS u32x4 *)(rbase + tile * (uint64_t)WAVE * (c32 ? 32u : 64u));
  const uint64_t nrec = min((uint64_t)WAVE, a.n - tile * WAVE);
  const int lg = c32 ? 1 : 2;
  const int kmax = c32 ? 2 : 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = k * WAVE + lane;
    if (k < kmax && (uint64_t)(e >> lg) < nrec) {
      const u32x4 val = stash[e];
      asm volatile("" ::: "memory");
      __builtin_nontemporal_store(val, dst + e);
    }
  }
}

// The tiles of wave `wv` of this block: first, first + step, ... below end.
// Strided over the grid by default; with a tail region (RxKArgs::tail_block)
// the blocks before it stride over the tiles before tail_tile and the ones
// from it on over the rest; with tune bit 8 (experiment) a contiguous run.
struct TileRange {
  uint64_t first, step, end;
};
__device__ __forceinline__ TileRange wave_tiles(const RxKArgs &a, uint64_t ntiles, int wv) {
  const uint64_t wid = (uint64_t)blockIdx.x * WPB + wv;
  const uint64_t nwaves = (uint64_t)gridDim.x * WPB;
  if (a.tune & 256u) {
    const uint64_t per = (ntiles + nwaves - 1) / nwaves;
    return {wid * per, 1, min(ntiles, (wid + 1) * per)};
  }
  if (a.tail_block == 0) return {wid, nwaves, ntiles};
  if (blockIdx.x < a.tail_block) return {wid, (uint64_t)a.tail_block * WPB, min(a.tail_tile, ntiles)};
  return {a.tail_tile + (uint64_t)(blockIdx.x - a.tail_block) * WPB + wv,
          (uint64_t)(gridDim.x - a.tail_block) * WPB, ntiles};
}
// A tile to prefetch descriptors or frames for: past the wave's range it
// is no tile (ntiles: past-the-end lanes, which read frame 0 / the batch's
// last chunk from cache), not a tile of another region.
__device__ __forceinline__ uint64_t pf_tile(const TileRange &r, uint64_t ntiles, uint64_t t) {
  return t < r.end ? t : ntiles;
}

// Waves per SIMD the register allocator must leave room for: the streaming
// variants keep D = 3 rounds of S chunks in registers (D * S * 4 VGPRs) and
// need 2 waves/SIMD; the small-frame variants 4.
template <int T, int S>
constexpr int min_waves_per_simd() { return S * T >= 32 ? 2 : 4; }
#ifndef PPTK_RX_D1_WAVES
#define PPTK_RX_D1_WAVES 3
#endif
template <int T, int S, int D>
constexpr int min_waves() { return D == 1 && S * T >= 32 ? PPTK_RX_D1_WAVES : min_waves_per_simd<T, S>(); }

// D = rounds in flight; (D + 1) must divide T so that the prefetch ring is
// back in its starting registers at the tile boundary (no moves of in-flight
// load destinations, which would force vmcnt waits).
// Length-group launch (pptk_rx_batch_device_mixed): this launch owns
// positions [*range_lo, *range_hi) of the binned order, known on the device
// only.  Returns false when the launch has nothing to do.
__device__ __forceinline__ bool group_range(RxKArgs &a) {
  if (a.range_lo && a.plan && !(*a.plan & 1u)) {
    // the binning found the batch not worth binning: the launch of the
    // group the plan names runs every frame in batch order from the
    // caller's own descriptors (records in whole 4 KB runs), the others
    // nothing
    if (((*a.plan >> 8) & 0xffu) != a.plan_group) return false;
    a.perm = nullptr;
    a.perm_ld = (const uint32_t *)a.zero;
    a.perm_msk = 0u;
    a.off_ld = a.off0 ? a.off0 : (const uint64_t *)a.zero;
    a.off_msk = a.off0 ? ~0u : 0u;
    a.stride_g = a.off0 ? 0u : a.stride;
    a.len_ld = a.len0;
    a.len_msk = ~0u;
    a.by_pos = 0;
  } else if (a.range_lo) {
    const uint32_t lo = *a.range_lo, hi = *a.range_hi;
    a.perm_ld += lo;
    if (a.by_pos) {
      a.off_ld += lo;
      a.len_ld += lo;
    }
    a.n = hi > lo ? hi - lo : 0;
    // an empty group: perm_ld points one past the permutation, and even
    // the clamped descriptor loads below would read it
    if (a.n == 0) return false;
  }
  return true;
}

template <int T, int S, int D, int AL, bool NT, bool GATHER>
__global__ __launch_bounds__(WAVE * WPB, (min_waves<T, S, D>())) void rx_kernel(RxKArgs a) {
  if constexpr (GATHER) {
    if (!group_range(a)) return;
  }
  __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * WAVE * IMG_STRIDE];
  constexpr int IMGC = (S * T < IMG_CHUNKS) ? S * T : IMG_CHUNKS;  // chunks parked
  constexpr uint32_t ALM = (1u << AL) - 1;
  static_assert(T % (D + 1) == 0, "prefetch ring must wrap at the tile boundary");
  // the streaming shapes up to 1536-byte frames hold a tile's records for
  // the write phases (the small-frame shapes, four waves per SIMD, have no
  // LDS to spare; the jumbo shape T64S2 measured slower with them: JMIX
  // 3.832 -> 3.939 ms, profiles/r05/x)
  constexpr bool PHASED = S * T >= 32 && T <= 32;
  __shared__ __attribute__((aligned(16))) u32x4 stash_lds[PHASED ? WPB * 4 * WAVE : 1];
  const bool phased = PHASED && a.phase_ticks != 0;
  uint64_t st_tile = ~0ull;     // the tile whose records wait in the stash
  uint64_t st_deadline = 0;
  constexpr bool UNROLL = T <= 32;   // tail chunks summed in the lane phase
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = threadIdx.x / WAVE;
  const int g = lane / T, j = lane % T;
  LDS_AS uint8_t *wimg = (LDS_AS uint8_t *)lds + wv * WAVE * IMG_STRIDE;
  LDS_AS u32x4 *stash = (LDS_AS u32x4 *)stash_lds + (PHASED ? wv * 4 * WAVE : 0);
  const uint64_t ntiles = (a.n + WAVE - 1) / WAVE;
  // Tile order (wave_tiles): strided over the grid (default), or, with tune
  // bit 8 (experiment), a contiguous block of tiles per wave, so that one
  // wave's successive record flushes are adjacent in memory.
  const TileRange tr = wave_tiles(a, ntiles, wv);
  const uint64_t step = tr.step, tend = tr.end;

  uint64_t tile = tr.first;
#ifdef PPTK_RX_WAVE_TIMES
  const uint64_t wid = (uint64_t)blockIdx.x * WPB + wv;
  const uint64_t wt_start = __builtin_amdgcn_s_memrealtime();
#endif
  Desc dc = load_desc<GATHER>(a, pf_tile(tr, ntiles, tile), lane);
  Desc dn = load_desc<GATHER>(a, pf_tile(tr, ntiles, tile + step), lane);
  uint32_t idx2 = desc_idx<GATHER>(a, pf_tile(tr, ntiles, tile + 2 * step), lane);
  // prologue: the first D rounds of the first tile, in slots 0 .. D-1
  Buf<S> b[D + 1];
  // (issued strictly in slot order: the loop-header wait is computed from
  // the older of the entry and back-edge states, and a reordered prologue
  // would turn it into a full drain)
#pragma unroll
  for (int k = 0; k < D; ++k) {
    b[k] = load_round<T, S, AL, NT>(a, dc, k, g, j);
    __builtin_amdgcn_sched_barrier(0);
  }

  while (tile < tend) {
    uint32_t my_sum = 0;
    // Descriptors run ahead in two stages so that no wait on them ever has
    // to drain the chunk loads in flight: the index (perm) of tile + 3 nwaves
    // is loaded here, the dependent offset/length of tile + 2 nwaves (whose
    // index arrived during the previous tile) before the last round group.
    const uint32_t idx3 = desc_idx<GATHER>(a, pf_tile(tr, ntiles, tile + 3 * step), lane);
    // ---- streaming rounds: team g sums frame g*T + r over [team_start, len).
    // Fixed-slot ring of D + 1 rounds: round r lives in slot r % (D + 1); a
    // group of D + 1 rounds is unrolled so every slot index is a constant and
    // no register of an in-flight load is ever copied.
    auto group = [&](const int r0) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u <= D; ++u) {
        const int r = r0 + u;
        {  // keep D rounds in flight: round r + D (of this or the next tile)
          const int rr = r + D;
          const Desc &dd = rr < T ? dc : dn;
          b[(u + D) % (D + 1)] = load_round<T, S, AL, NT>(a, dd, rr < T ? rr : rr - T, g, j);
        }
        const Buf<S> &cb = b[u];
        const int q = g * T + r;
        const int m = (int)(cb.pb & ALM);       // frame start inside its first chunk row
        const int c_img = m >> 4;                  // first chunk holding frame bytes
        const int nch = (m + (int)cb.pl + 15) >> 4;
        LDS_AS uint8_t *img = wimg + q * IMG_STRIDE;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if (s * T < IMGC + (int)(ALM >> 4)) {
            const int ci = s * T + j - c_img;      // image = 16-byte chunks from floor16(frame)
            if (ci >= 0 && ci < IMGC) {
              if constexpr (IMG_STRIDE % 16 == 0) {
                *(LDS_AS u32x4 *)(img + 16 * ci) = cb.v[s];
              } else {
                LDS_AS uint32_t *w = (LDS_AS uint32_t *)(img + 16 * ci);
                w[0] = cb.v[s].x;
                w[1] = cb.v[s].y;
                w[2] = cb.v[s].z;
                w[3] = cb.v[s].w;
              }
            }
          }
        }
        uint32_t acc = 0;
        const int ts = team_start_of(m & 15);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int c = s * T + j;
          acc = sum_chunk_from<!GATHER>(cb.v[s], 16 * c - m, ts, (int)cb.pl, acc);
        }
        if (!UNROLL && nch > S * T) {  // frames longer than the staged chunks (masked)
          const u32x4 *c0 = (const u32x4 *)(a.frames + (cb.pb - (uint64_t)m));
          for (int c = S * T + j; c < nch; c += T)
            acc = sum_chunk_from<true>(ldc<NT>(c0 + c), 16 * c - m, ts, (int)cb.pl, acc);
        }
        if constexpr (GATHER) {
          // The unmasked sums added the bytes past the frame's end in its
          // last chunk.  The team's last lane holds that chunk in its last
          // slot whenever the frame fits the round (its loads are clamped to
          // the last chunk, load_round): it parks it in the frame's image
          // slot (bytes 128..143), where the owning lane takes those bytes
          // off in the lane phase -- no second read of the chunk from
          // memory, one LDS store per round.  (TAIL_LDS 0, A/B: the same
          // correction here, every lane computing it, every round; a lane's
          // partial may wrap below zero, the team's u32 total cannot.)
          if constexpr (TAIL_LDS) {
            if (j == T - 1) *(LDS_AS u32x4 *)(img + TAIL_OFF) = cb.v[S - 1];
          } else {
            const uint32_t corr = tail_past_end(cb.v[S - 1], m, (int)cb.pl, ts);
            acc -= (j == T - 1 && nch <= S * T) ? corr : 0u;
          }
        }
        acc = team_sum<T>(acc);
        if (j == r)
          my_sum = acc;
        // the write-phase check after every round of the group (the last
        // one's follows the group): the finer the check, the closer the
        // waves' writes fall together (C1500 T16S6 4.150 -> 4.123 ms, CMIX
        // 2.551 -> 2.542, against checks between groups only,
        // profiles/r05/ag/)
        if (PHASED && u < D && st_tile != ~0ull && __builtin_amdgcn_s_memrealtime() >= st_deadline) {
          flush_stash(a, stash, st_tile, lane);
          st_tile = ~0ull;
        }
      }
    };
#ifdef PPTK_RX_FULL_UNROLL
#pragma unroll(T <= 16 ? T : 1)
#else
#pragma unroll 1
#endif
    for (int r0 = 0; r0 < T - (D + 1); r0 += D + 1) {
      group(r0);
      if (PHASED && st_tile != ~0ull && __builtin_amdgcn_s_memrealtime() >= st_deadline) {
        flush_stash(a, stash, st_tile, lane);
        st_tile = ~0ull;
      }
    }
    // the descriptors two tiles ahead are loaded BEFORE the last group issues
    // the next tile's first D rounds: the copies dc <- dn <- d2 at the tile
    // boundary then wait only for these loads, not for the rounds in flight
    const Desc d2 = desc_fill<GATHER>(a, idx2, pf_tile(tr, ntiles, tile + 2 * step), lane);
    __builtin_amdgcn_sched_barrier(0);
    group(T - (D + 1));

    // ---- lane phase: frame `lane` -> record (parsed once per frame)
    const bool stage = !(a.tune & 2u);
    const bool scatter = GATHER && a.perm;
    // tune bit 4 (diagnostics only, output invalid): skip the lane phase
    if (dc.idx != 0xffffffffu && !(kDiag && (a.tune & 16u))) {
      const int m = (int)(dc.base & 15);
      const int ma = (int)(dc.base & ALM);
      const int nch = (ma + (int)dc.len + 15) >> 4;
      // the frame's last chunk as its team parked it (frames that fit the
      // round; longer ones were summed masked)
      u32x4 tailc = (u32x4){0u, 0u, 0u, 0u};
      if constexpr (GATHER && TAIL_LDS) {
        const u32x4 t = *(const LDS_AS u32x4 *)(wimg + lane * IMG_STRIDE + TAIL_OFF);
        const bool fits = nch <= S * T;
        tailc = (u32x4){fits ? t.x : 0u, fits ? t.y : 0u, fits ? t.z : 0u, fits ? t.w : 0u};
      }
      if (UNROLL) {  // unrolled variants: chunks past the staged S*T, summed here (rare)
        if (nch > S * T) {
          const u32x4 *c0 = (const u32x4 *)(a.frames + (dc.base - (uint64_t)ma));
          for (int c = S * T; c < nch; ++c)   // (masked: the last one ends the frame)
            my_sum = settle(sum_chunk_from<true>(ldc<NT>(c0 + c), 16 * c - ma, 0, (int)dc.len,
                                                 my_sum));
        }
      }
      const FrameView v = {wimg + lane * IMG_STRIDE, (const GLB_AS uint8_t *)a.frames + dc.base, m,
                           16 * IMGC - m};
      LaneRec o;
      lane_generic(a, v, dc.len, dc.base, my_sum, tailc, o);
      if (a.txside)
        a.txside[dc.idx] = o.tx;   // two-pass tx: 8 B per frame, coalesced in batch order
      // park the record in LDS (every lane's image reads are behind us in
      // program order) for the coalesced store below
      emit_record(a, o, dc.idx, (LDS_AS u32x4 *)wimg + lane * 5, stage);
    }
    if (stage && !(kDiag && (a.tune & 8u)) && (a.recs || a.recs32)) {  // tune bit 3: diagnostics, no stores
      if (PHASED && phased && !scatter) {
        if (st_tile != ~0ull) flush_stash(a, stash, st_tile, lane);   // the stash is needed
        flush_records(a, wimg, tile, lane, dc.idx, scatter, stash);
        st_tile = tile;
        st_deadline = phase_deadline(a.phase_ticks);
      } else {
        flush_records(a, wimg, tile, lane, dc.idx, scatter);
      }
    }
    tile += step;
    dc = dn;
    dn = d2;
    idx2 = idx3;
  }
  if (PHASED && st_tile != ~0ull) flush_stash(a, stash, st_tile, lane);
#ifdef PPTK_RX_WAVE_TIMES
  // probe build (tools/wave_times.py): when each wave started and finished
  if (a.wave_times && lane == 0) {
    a.wave_times[2 * wid] = wt_start;
    a.wave_times[2 * wid + 1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// ---- Mixed-shape kernel (RX_M6): lanes binned by length inside each tile.
//
// rx_kernel gives every frame of a tile a team round sized for the longest
// frame the batch may hold (T16S6: 4 frames per round, 6 chunk loads per
// lane), so a 64-byte frame of an IMIX tile costs as many load and sum
// instructions as a 1500-byte one.  Here each tile's 64 frames are binned by
// their chunk count into three classes, each run with rounds of the same
// register shape -- 6 chunk loads per lane -- but a different team width:
//   class 0: <= 24 chunks (<= 384-byte span), teams of 4 lanes, 16 frames/round
//   class 1: <= 48 chunks (<= 768 bytes),     teams of 8 lanes,  8 frames/round
//   class 2: anything longer,                 teams of 16 lanes, 4 frames/round
// (longer than 96 chunks: the rest is summed in the lane phase, as the
// unrolled team variants do).  The binning is a ballot per class and a
// rank by mbcnt: the tile's frame lanes are listed round by round in LDS
// (m_schedule; no global permutation, no extra HBM traffic); round r of the
// tile runs frames of one class.  Every round issues the same six
// loads, so the prefetch ring of rx_kernel carries over unchanged: D rounds
// in flight in fixed register slots, the round count padded to a multiple
// of D + 1 with empty rounds, and the next tile's schedule (built from
// its descriptors, which run a tile ahead) known before the last round
// group issues that tile's first rounds.  A round's team sum goes to the
// frame's LDS slot (bytes 128..131 of its image), where the owning lane
// reads it in the lane phase.  Frame i's record stays at its own index,
// written in the tile's 4 KB run.  IMIX (7:4:1 of 64/576/1500 B) needs ~8
// rounds per tile instead of 16.
constexpr int M_S = 6;        // chunk loads per lane per round
// Rounds in flight and waves per SIMD: one round in flight at 3 waves/SIMD
// (141 VGPRs) beat three at 2 waves/SIMD (195) and two at 2 or 3 (168):
// IMIX 1.537 / 1.475 / 1.451 ms for D = 3 / 2 / 1, CMIX 2.891 / 2.864 /
// 2.865 ms (in-process A/B, profiles/r03/m6/m6d_ab_*.json).
#ifndef PPTK_RX_M_D
#define PPTK_RX_M_D 1
#endif
#ifndef PPTK_RX_M_WAVES
#define PPTK_RX_M_WAVES 3
#endif
constexpr int M_D = PPTK_RX_M_D;   // rounds in flight
constexpr int M_SUM = 128;    // byte offset of a frame's team sum in its image slot
static_assert(IMG_STRIDE >= M_SUM + 4, "the team sum lives past the 128-byte image");

// A tile's schedule (wave-uniform): frames per class, and the round
// boundaries -- class 0 runs rounds [0, e0), class 1 [e0, e1), class 2
// [e1, e2), rounds [e2, P) are empty.
struct MSched {
  uint32_t n0, n1, n2, e0, e1, e2;
};

__device__ __forceinline__ uint32_t m_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Bin the tile's frames (descriptor d per lane) and list them round by
// round in `list`: row r (16 bytes) holds the lanes of the frames round r's
// teams sum, 0xff for an empty team, so a round finds its team's frame with
// one LDS byte load and no per-class arithmetic.  Lanes past the batch are
// not listed.  (Listing whole descriptors, 16 bytes each, read by one
// broadcast LDS load per round instead of the lane index plus three
// shuffles, measured slower: IMIX 1.62 vs 1.54 ms, CMIX +11 % vs +1.5 %
// against the team kernel.)
constexpr int M_RMAX = 24;   // list rows (a tile needs at most 20: 1 + 1 + 16 rounds, padded)
__device__ __forceinline__ MSched m_schedule(const Desc &d, int lane, LDS_AS uint8_t *list) {
  const bool valid = d.idx != 0xffffffffu;
  const uint32_t nch = ((uint32_t)(d.base & 15u) + d.len + 15u) >> 4;
  const uint64_t b0 = __ballot(valid && nch <= 24u);
  const uint64_t b1 = __ballot(valid && nch > 24u && nch <= 48u);
  const uint64_t b2 = __ballot(valid && nch > 48u);
  MSched s;
  s.n0 = (uint32_t)__popcll(b0);
  s.n1 = (uint32_t)__popcll(b1);
  s.n2 = (uint32_t)__popcll(b2);
  s.e0 = (s.n0 + 15u) >> 4;
  s.e1 = s.e0 + ((s.n1 + 7u) >> 3);
  s.e2 = s.e1 + ((s.n2 + 3u) >> 2);
  LDS_AS uint32_t *lw = (LDS_AS uint32_t *)list;   // every row empty first
  lw[lane] = 0xffffffffu;
  if (lane < M_RMAX * 4 - WAVE) lw[WAVE + lane] = 0xffffffffu;
  // class c: rows from its first round on, 16 >> c frames per row
  const uint32_t c = nch <= 24u ? 0u : nch <= 48u ? 1u : 2u;
  const uint32_t rho = c == 0u ? m_rank(b0) : c == 1u ? m_rank(b1) : m_rank(b2);
  const uint32_t er = c == 0u ? 0u : c == 1u ? s.e0 : s.e1;
  const uint32_t sh = 4u - c;
  if (valid) list[(er + (rho >> sh)) * 16u + (rho & ((1u << sh) - 1u))] = (uint8_t)lane;
  return s;
}

// Rounds the tile runs: the schedule's, padded to whole groups of D + 1,
// and at least two groups -- the group loop then runs at least once, so the
// compiler has no zero-trip path on which it would copy the ring's in-flight
// registers (a vmcnt(0) drain at every such tile).
__device__ __forceinline__ uint32_t m_rounds(const MSched &s) {
  constexpr uint32_t G = M_D + 1;
  return s.e2 <= 2 * G ? 2 * G : (s.e2 + G - 1) / G * G;
}

// log2 of the team width of round r (wave-uniform).
__device__ __forceinline__ int m_tl(const MSched &s, uint32_t r) {
  return r < s.e0 ? 2 : r < s.e1 ? 3 : 4;
}

// Team sum of a round, complete in the team's LAST lane (lane T - 1 of the
// team), by DPP adds inside each row of 16 lanes -- no LDS crossbar traffic:
// quad_perm [1,0,3,2] and [2,3,0,1] sum each quad (every lane of it), then
// row_shr:4 and row_shr:8 fold the quads of an 8- or 16-lane team into its
// last lane (lanes whose source lies outside the row add 0).
template <int CTRL>
__device__ __forceinline__ uint32_t m_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t m_team_sum(uint32_t x, int tl) {
  x += m_dpp<0xb1>(x);   // quad_perm [1,0,3,2]
  x += m_dpp<0x4e>(x);   // quad_perm [2,3,0,1]
  const uint32_t x8 = x + m_dpp<0x114>(x);    // row_shr:4
  x = tl >= 3 ? x8 : x;
  const uint32_t x16 = x + m_dpp<0x118>(x);   // row_shr:8
  return tl >= 4 ? x16 : x;
}

struct MBuf {
  u32x4 v[M_S];
  // packed: bits 0-7 the frame's lane in the tile (0xff: no frame, an empty
  // team), 8-11 the frame start inside its chunk, 16-31 the frame length
  uint32_t qml;
};

template <bool NT>
__device__ __forceinline__ MBuf m_load_round(const RxKArgs &a, const Desc &d, const MSched &s,
                                             const LDS_AS uint8_t *list, uint32_t r, int lane) {
  const int tl = m_tl(s, r);
  const uint32_t e = list[r * 16u + ((uint32_t)lane >> tl)];
  const bool real = e != 0xffu;
  // (an empty team reads lane 63's frame: every lane describes a valid
  // frame, lanes past the batch frame 0)
  const uint32_t q = e & (WAVE - 1);
  MBuf b;
  // both shuffles unconditional: a ds_bpermute executed under a lane mask
  // reads 0 from every source lane outside the mask
  const uint64_t pb = __shfl(d.base, (int)q);
  const uint32_t pl = __shfl(d.len, (int)q) & (0u - (uint32_t)real);
  const int m = (int)(pb & 15u);
  b.qml = (real ? q : 0xffu) | ((uint32_t)m << 8) | (pl << 16);
  const u32x4 *c0 = (const u32x4 *)(a.frames + (pb - (uint64_t)m));
  const int nch = (m + (int)pl + 15) >> 4;
  const int clast = nch > 0 ? nch - 1 : 0;
  const int j = lane & ((1 << tl) - 1);
#pragma unroll
  for (int i = 0; i < M_S; ++i)
    b.v[i] = ldc<NT>(c0 + min((i << tl) + j, clast));   // unconditional (see load_round)
  return b;
}

template <bool NT, bool GATHER>
__global__ __launch_bounds__(WAVE * WPB, PPTK_RX_M_WAVES) void rx_kernel_mixed(RxKArgs a) {
  if constexpr (GATHER) {
    if (!group_range(a)) return;
  }
  __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * WAVE * IMG_STRIDE];
  __shared__ __attribute__((aligned(16))) uint8_t lists[WPB][2][M_RMAX * 16];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = threadIdx.x / WAVE;
  LDS_AS uint8_t *wimg = (LDS_AS uint8_t *)lds + wv * WAVE * IMG_STRIDE;
  LDS_AS uint8_t *lst[2] = {(LDS_AS uint8_t *)lists[wv][0], (LDS_AS uint8_t *)lists[wv][1]};
  const uint64_t ntiles = (a.n + WAVE - 1) / WAVE;
  const TileRange tr = wave_tiles(a, ntiles, wv);
  const uint64_t step = tr.step, tend = tr.end;

  uint64_t tile = tr.first;
  Desc dc = load_desc<GATHER>(a, pf_tile(tr, ntiles, tile), lane);
  Desc dn = load_desc<GATHER>(a, pf_tile(tr, ntiles, tile + step), lane);
  uint32_t idx2 = desc_idx<GATHER>(a, pf_tile(tr, ntiles, tile + 2 * step), lane);
  int cur = 0;
  MSched sc = m_schedule(dc, lane, lst[0]);
  MBuf b[M_D + 1];
#pragma unroll
  for (int k = 0; k < M_D; ++k) {
    b[k] = m_load_round<NT>(a, dc, sc, lst[0], (uint32_t)k, lane);
    __builtin_amdgcn_sched_barrier(0);
  }

  while (tile < tend) {
    const uint32_t idx3 = desc_idx<GATHER>(a, pf_tile(tr, ntiles, tile + 3 * step), lane);
    // the next tile's schedule, into the other list (the previous tile's,
    // whose rounds are all consumed)
    const MSched sn = m_schedule(dn, lane, lst[cur ^ 1]);
    const uint32_t P = m_rounds(sc);
    // Round r lives in slot r % (D + 1); P is a multiple of D + 1, so the
    // ring is back in slot 0 at every tile boundary.  LAST: the group's
    // prefetches past this tile issue the next tile's first D rounds.
    auto group = [&](const uint32_t r0, auto last_tag) __attribute__((always_inline)) {
      constexpr bool LAST = decltype(last_tag)::value;
#pragma unroll
      for (int u = 0; u <= M_D; ++u) {
        const uint32_t r = r0 + (uint32_t)u;
        if (LAST && u > 0)
          b[(u + M_D) % (M_D + 1)] =
              m_load_round<NT>(a, dn, sn, lst[cur ^ 1], (uint32_t)(u - 1), lane);
        else
          b[(u + M_D) % (M_D + 1)] = m_load_round<NT>(a, dc, sc, lst[cur], r + M_D, lane);
        const MBuf &cb = b[u];
        const int tl = m_tl(sc, r);
        const int j = lane & ((1 << tl) - 1);
        const uint32_t q = cb.qml & 0xffu;
        const bool real = q != 0xffu;
        const int m = (int)((cb.qml >> 8) & 15u);
        const int pl = (int)(cb.qml >> 16);
        LDS_AS uint8_t *img = wimg + (q & (WAVE - 1)) * IMG_STRIDE;
        // the image: chunks 0..7 of the frame (every team width is >= 4,
        // so only the first two load slots can hold them)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int c = (i << tl) + j;
          if (real && c < IMG_CHUNKS) *(LDS_AS u32x4 *)(img + 16 * c) = cb.v[i];
        }
        uint32_t acc = 0;
        const int ts = team_start_of(m);
        if constexpr (GATHER) {
          // unmasked sums of the chunks c in [c_lo, nch): o = 16c - m >= ts
          // and o < len; one unsigned compare per chunk
          const int c_lo = (ts + m + 15) >> 4;
          const uint32_t span = (uint32_t)max(((m + pl + 15) >> 4) - c_lo, 0);
          const uint32_t jc = (uint32_t)(j - c_lo);
#pragma unroll
          for (int i = 0; i < M_S; ++i) {
            uint32_t t = dot16(cb.v[i].x, 0);
            t = dot16(cb.v[i].y, t);
            t = dot16(cb.v[i].z, t);
            t = dot16(cb.v[i].w, t);
            acc += jc + ((uint32_t)i << tl) < span ? t : 0u;
          }
        } else {
#pragma unroll
          for (int i = 0; i < M_S; ++i)
            acc = sum_chunk_from<true>(cb.v[i], 16 * ((i << tl) + j) - m, ts, pl, acc);
        }
        acc = m_team_sum(acc, tl);
        if constexpr (GATHER) {
          // the bytes past the frame's end in its last chunk, which the
          // unmasked sums added: the team's last lane (which holds the team
          // total) holds that chunk in its last slot when the frame fits the
          // round (loads clamped to the last chunk, m_load_round)
          const uint32_t corr = tail_past_end(cb.v[M_S - 1], m, pl, ts);
          acc -= ((m + pl + 15) >> 4) <= (M_S << tl) ? corr : 0u;
        }
        if (real && j == (1 << tl) - 1) *(LDS_AS uint32_t *)(img + M_SUM) = acc;
      }
    };
    uint32_t r0 = 0;
#pragma unroll 1
    do {   // P >= 2 (D + 1): at least once
      group(r0, std::false_type{});
      r0 += M_D + 1;
    } while (r0 < P - (M_D + 1));
    const Desc d2 = desc_fill<GATHER>(a, idx2, pf_tile(tr, ntiles, tile + 2 * step), lane);
    __builtin_amdgcn_sched_barrier(0);
    group(P - (M_D + 1), std::true_type{});

    // ---- lane phase: frame `lane` -> record
    __builtin_amdgcn_wave_barrier();
    const bool stage = !(a.tune & 2u);
    const bool scatter = GATHER && a.perm;
    if (dc.idx != 0xffffffffu && !(kDiag && (a.tune & 16u))) {
      const int m = (int)(dc.base & 15);
      uint32_t my_sum = *(const LDS_AS uint32_t *)(wimg + lane * IMG_STRIDE + M_SUM);
      const int nch = (m + (int)dc.len + 15) >> 4;
      if (nch > 16 * M_S) {   // longer than a 16-lane round holds (jumbo): rare
        const u32x4 *c0 = (const u32x4 *)(a.frames + (dc.base - (uint64_t)m));
        for (int c = 16 * M_S; c < nch; ++c)   // (masked: the last one ends the frame)
          my_sum = settle(sum_chunk_from<true>(ldc<NT>(c0 + c), 16 * c - m, 0, (int)dc.len,
                                               my_sum));
      }
      const FrameView v = {wimg + lane * IMG_STRIDE, (const GLB_AS uint8_t *)a.frames + dc.base, m,
                           16 * IMG_CHUNKS - m};
      LaneRec o;
      lane_generic(a, v, dc.len, dc.base, my_sum, (u32x4){0u, 0u, 0u, 0u}, o);
      if (a.txside)
        a.txside[dc.idx] = o.tx;
      emit_record(a, o, dc.idx, (LDS_AS u32x4 *)wimg + lane * 5, stage);
    }
    if (stage && !(kDiag && (a.tune & 8u)) && (a.recs || a.recs32))
      flush_records(a, wimg, tile, lane, dc.idx, scatter);
    tile += step;
    dc = dn;
    dn = d2;
    idx2 = idx3;
    sc = sn;
    cur ^= 1;
  }
}

// Lane kernel (RX_L4): frames of at most 64 bytes at a fixed stride, every
// frame start 16-byte aligned (the host checks the buffer address and the
// stride).  Small frames need no team streaming: lane q loads its own frame
// as four 16-byte chunks (a wave's four loads cover the tile's 4 KB exactly;
// each line is fetched once and served to its lanes from the caches), the
// common IPv4 case is parsed from registers at fixed offsets (lane_fast),
// anything else goes through the LDS image and lane_generic.  The next tile's
// chunks are in flight while a tile is processed (two register sets used in
// turn, so no in-flight load destination is ever copied).
constexpr int LSLOT = 80;   // LDS bytes per lane: 64-byte frame image, then the record

// Coalesced tiles (PPTK_RX_LANE_COAL): when the frames are packed at a
// 64-byte stride and every frame spans four chunks, the tile is one
// contiguous 4 KB run and load s of lane q takes its chunk 64 s + q (each
// instruction reads 1 KB contiguously, as the speed-of-light kernel does,
// instead of 16 bytes of each of 64 frames); the chunks then go through the
// LDS slots to the lane of their frame (lane_chunks).  With non-temporal
// loads (the automatic policy for such batches): C64 0.3815 -> 0.3723 ms,
// compact records 0.3178 -> 0.3151 (in-process A/B, profiles/r06/lane/);
// with temporal loads it is slower (0.3885), as the per-frame loads are
// with non-temporal ones (0.4662).

template <bool NT>
__device__ __forceinline__ void lane_load(const RxKArgs &a, uint64_t tile, int lane, uint32_t nch,
                                          bool coal, u32x4 c[4]) {
  uint64_t i = tile * WAVE + lane;
  i = i < a.n ? i : a.n - 1;   // past-the-end lanes re-read the last frame (no record)
  const u32x4 *p = (const u32x4 *)(a.frames + i * a.stride);
  const u32x4 *t = (const u32x4 *)a.frames;
  const uint64_t last = 4 * a.n - 1;   // (coalesced: the batch's last chunk)
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint64_t k = min(tile * (4 * WAVE) + (uint64_t)(s * WAVE + lane), last);
    c[s] = ldc<NT>(coal ? t + k : p + min((uint32_t)s, nch ? nch - 1 : 0u));   // past the frame: masked at use
  }
}

// The lane's own four chunks from a coalesced tile's loads: chunk 64 s + q
// belongs to frame 16 s + q / 4, piece q % 4; parked in that frame's LDS slot
// and read back by its lane.  (The 80-byte slot pitch keeps both the stores
// and the 16-lane read groups free of bank conflicts.)
__device__ __forceinline__ void lane_chunks(LDS_AS uint8_t *wimg, int lane, u32x4 c[4]) {
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int s = 0; s < 4; ++s)
    *(LDS_AS u32x4 *)(wimg + (16 * s + (lane >> 2)) * LSLOT + (lane & 3) * 16) = c[s];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int s = 0; s < 4; ++s) c[s] = *(const LDS_AS u32x4 *)(wimg + lane * LSLOT + s * 16);
  __builtin_amdgcn_wave_barrier();
}

template <bool NT>
__device__ __forceinline__ void lane_tile(const RxKArgs &a, uint64_t tile, int lane, uint32_t nch,
                                          bool coal, const u32x4 cl[4], LDS_AS uint8_t *wimg) {
  const uint64_t i = tile * WAVE + lane;
  LDS_AS uint8_t *slot = wimg + lane * LSLOT;
  u32x4 c[4] = {cl[0], cl[1], cl[2], cl[3]};
  if (coal) lane_chunks(wimg, lane, c);
  if (i < a.n && !(kDiag && (a.tune & 16u))) {
    const uint32_t len = a.fixed_len;
    uint32_t d[16];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bool in = (uint32_t)s < nch;
      d[4 * s + 0] = in ? c[s].x : 0u;
      d[4 * s + 1] = in ? c[s].y : 0u;
      d[4 * s + 2] = in ? c[s].z : 0u;
      d[4 * s + 3] = in ? c[s].w : 0u;
    }
    LaneRec o;
    if (!lane_fast(a, d, len, o)) {
      LDS_AS u32x4 *img = (LDS_AS u32x4 *)slot;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        img[s] = (u32x4){d[4 * s], d[4 * s + 1], d[4 * s + 2], d[4 * s + 3]};
      // team-round equivalent: the sum of [team_start_of(0) = 32, len)
      uint32_t ms = sum_chunk_from<true>(img[2], 32, 32, (int)len, 0u);
      ms = sum_chunk_from<true>(img[3], 48, 32, (int)len, ms);
      const FrameView v = {slot, (const GLB_AS uint8_t *)a.frames + i * a.stride, 0, 64};
      lane_generic(a, v, len, i * a.stride, ms, (u32x4){0u, 0u, 0u, 0u}, o);
    }
    emit_record(a, o, (uint32_t)i, (LDS_AS u32x4 *)slot, true);
  }
  if (!(kDiag && (a.tune & 8u)) && (a.recs || a.recs32))
    flush_records(a, wimg, tile, lane, 0u, false);
}

// (A/B: PPTK_RX_LANE_WAVES waves per SIMD the registers must allow;
// PPTK_RX_LANE_PREFETCH 0 loads each tile at its start instead of one tile
// ahead, for more waves in the same registers)
#ifndef PPTK_RX_LANE_WAVES
#define PPTK_RX_LANE_WAVES 4
#endif
#ifndef PPTK_RX_LANE_PREFETCH
#define PPTK_RX_LANE_PREFETCH 1
#endif
template <bool NT>
__global__ __launch_bounds__(WAVE * WPB, PPTK_RX_LANE_WAVES) void rx_kernel_lane(RxKArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * WAVE * LSLOT];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = threadIdx.x / WAVE;
  LDS_AS uint8_t *wimg = (LDS_AS uint8_t *)lds + wv * WAVE * LSLOT;
  const uint64_t ntiles = (a.n + WAVE - 1) / WAVE;
  const TileRange tr = wave_tiles(a, ntiles, wv);
  const uint64_t step = tr.step;
  const uint32_t nch = (a.fixed_len + 15u) >> 4;   // 1..4, uniform
  // (uniform: the batch is one contiguous run of 64-byte frame slots)
  const bool coal = lane_coalesced(a.stride, a.fixed_len);
  uint64_t tile = tr.first;
#if PPTK_RX_LANE_PREFETCH
  u32x4 c0[4], c1[4];
  lane_load<NT>(a, pf_tile(tr, ntiles, tile), lane, nch, coal, c0);
  while (tile < tr.end) {
    lane_load<NT>(a, pf_tile(tr, ntiles, tile + step), lane, nch, coal, c1);
    lane_tile<NT>(a, tile, lane, nch, coal, c0, wimg);
    tile += step;
#pragma unroll
    for (int s = 0; s < 4; ++s) c0[s] = c1[s];
  }
#else
  while (tile < tr.end) {
    u32x4 c0[4];
    lane_load<NT>(a, tile, lane, nch, coal, c0);
    lane_tile<NT>(a, tile, lane, nch, coal, c0, wimg);
    tile += step;
  }
#endif
}

// Header rewrite with incremental checksum updates (pptk_tx_rewrite_device,
// reference iphdr/ipcksum.h:213-393).  Only the first 128 bytes of a frame
// matter (Ethernet, the IPv4 header, the first 18 bytes of TCP/UDP), so one
// lane per frame loads its frame's first eight aligned chunks (clamped to
// the frame) into its LDS slot, parses it exactly as the receive transform
// does, folds the requested changes into the transmitted checksums with
// RFC 1624 updates, and stores the changed fields.
__device__ __forceinline__ uint32_t upd16(uint32_t ck, uint32_t o, uint32_t nw) {
  // ip_update_cksum16 (iphdr/ipcksum.h:213-226)
  uint32_t s = (~ck & 0xffffu) + (~o & 0xffffu) + nw;
  s = fold16(s);
  return ~s & 0xffffu;
}
__device__ __forceinline__ uint32_t upd32(uint32_t ck, uint32_t o, uint32_t nw) {
  // ip_update_cksum32 (:228-236): high halves, then low halves
  return upd16(upd16(ck, o >> 16, nw >> 16), o & 0xffffu, nw & 0xffffu);
}

// Field writes of one frame: patched into the lane's LDS image (and marked
// in `touched`) where the image holds the byte, stored directly otherwise;
// flush() then writes back every image chunk that lies inside the frame
// whole -- whole 16-byte chunks instead of a dozen scattered byte stores per
// frame: C64 0.77 -> 0.58 ms, C1500 1.47 -> 1.24 ms, CMIX 1.28 -> 1.15 ms
// (in-process A/B, tools/ab_rewrite.py) -- and only the touched bytes of
// chunks that reach outside it (those bytes may be a neighbour's).
template <int SLOT>
struct FieldWriter {
  LDS_AS uint8_t *img;
  GLB_AS uint8_t *f;     // frame start
  int m;
  uint64_t touched = 0;  // image byte positions patched

  __device__ __forceinline__ void put(int k, uint32_t v, int nbytes) {
    for (int b = 0; b < nbytes; ++b) {
      const uint8_t x = (uint8_t)(v >> (8 * (nbytes - 1 - b)));
      const int pos = m + k + b;
      if (pos < SLOT) {
        img[pos] = x;
        touched |= 1ull << pos;
      } else {
        f[k + b] = x;
      }
    }
  }
  __device__ __forceinline__ void flush(uint32_t len) {
    if (!touched) return;
    GLB_AS uint8_t *row = f - m;
#pragma unroll
    for (int c = 0; c < SLOT / 16; ++c) {
      const int fo = 16 * c - m;                    // frame offset of the chunk
      // only chunks holding a changed byte (writing back the untouched ones
      // as well cost C64 0.526 vs 0.463 ms, C1500 1.300 vs 1.220 ms)
      if (!((touched >> (16 * c)) & 0xffffu)) continue;
      if (fo >= 0 && fo + 16 <= (int)len) {
        const LDS_AS uint32_t *w = (const LDS_AS uint32_t *)img + 4 * c;
        *(GLB_AS u32x4 *)(row + 16 * c) = (u32x4){w[0], w[1], w[2], w[3]};
      } else {
        uint32_t t = (uint32_t)(touched >> (16 * c)) & 0xffffu;
        while (t) {
          const int b = __builtin_ctz(t);
          row[16 * c + b] = img[16 * c + b];
          t &= t - 1;
        }
      }
    }
  }
};

// The lane's image holds the frame's first four aligned chunks, 64 - m
// frame bytes: every field of an IPv4 frame with a 20-byte header lies in
// the first 52 bytes (56 behind a VLAN tag), so the image covers it when the
// frame starts at most 12 (8) bytes into its chunk; fields past the image
// come from global memory through the FrameView rare path.
constexpr int RW_SLOT = 64;

// Lane slots of the header kernels sit an odd number of dwords apart (slot
// + 4 bytes): the per-frame parse reads the same frame offset in every
// lane's slot, which at a 64- or 128-byte pitch falls into one or two LDS
// banks (a 32- to 64-way conflict on every byte read: SQ_ACTIVE_INST_LDS
// ~15x SQ_INSTS_LDS); at an odd dword pitch the lanes spread over all 32
// banks.  The slots are then only 4-byte aligned, so chunks are parked and
// read back as dwords.
template <int SLOT>
__device__ __forceinline__ void park_chunks(LDS_AS uint8_t *slot, const u32x4 *c0, int nch) {
  LDS_AS uint32_t *w = (LDS_AS uint32_t *)slot;
#pragma unroll
  for (int c = 0; c < SLOT / 16; ++c) {
    const u32x4 v = c0[min(c, nch - 1)];
    w[4 * c] = v.x;
    w[4 * c + 1] = v.y;
    w[4 * c + 2] = v.z;
    w[4 * c + 3] = v.w;
  }
}

__global__ __launch_bounds__(256) void rx_rewrite_kernel(RxKArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[256 * (RW_SLOT + 4)];
  LDS_AS uint8_t *slot = (LDS_AS uint8_t *)lds + threadIdx.x * (RW_SLOT + 4);
  const uint64_t step = (uint64_t)gridDim.x * 256u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += step) {
    const uint64_t base = a.off ? a.off[i] : i * a.stride;
    const uint32_t len = a.len ? a.len[i] : a.fixed_len;
    const int m = (int)(base & 15);
    const int nch = max((m + (int)len + 15) >> 4, 1);
    park_chunks<RW_SLOT>(slot, (const u32x4 *)(a.frames + (base - (uint64_t)m)), nch);
    const FrameView v = {slot, (const GLB_AS uint8_t *)a.frames + base, m, RW_SLOT - m};
    const Parse p = parse_frame(v, len);
    uint32_t st = 0;
    if ((p.flags & (PPTK_RX_F_PARSED | PPTK_RX_F_MALFORMED | PPTK_RX_F_IPV6)) == PPTK_RX_F_PARSED) {
      const pptk_rewrite w = a.rw[a.rw_one ? 0 : i];
      const int l3 = (int)p.l3, l4 = (int)p.rs;
      const bool l4ok = p.flags & PPTK_RX_F_L4;
      const uint32_t proto = p.proto;
      uint32_t ttl = v.u8(l3 + 8);
      if ((w.ops & PPTK_RW_DECR_TTL) && ttl == 0) {
        st = PPTK_RW_ST_TTL_ZERO;   // the reference abort()s (:382-385)
      } else {
        st = PPTK_RW_ST_IP | (l4ok ? PPTK_RW_ST_L4 : 0u);
        FieldWriter<RW_SLOT> fw{slot, (GLB_AS uint8_t *)a.frames_w + base, m};
        const int cko = proto == 6 ? 16 : 6;          // TCP / UDP checksum field
        uint32_t ipc = v.be16(l3 + 10);
        uint32_t l4c = l4ok ? v.be16(l4 + cko) : 0u;
        bool l4c_w = false;
        if (w.ops & PPTK_RW_DECR_TTL) {   // ip_decr_ttl_cksum_update (:374-393)
          ipc = upd16(ipc, (ttl << 8) | proto, ((ttl - 1) << 8) | proto);
          ttl -= 1;
          fw.put(l3 + 8, ttl, 1);
          if (ttl == 0) st |= PPTK_RW_ST_EXPIRED;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {    // ip_set_src/dst_cksum_update (:238-261, :349-372)
          const uint32_t op = k == 0 ? PPTK_RW_SRC : PPTK_RW_DST;
          if (!(w.ops & op)) continue;
          const uint32_t nw = k == 0 ? w.src : w.dst;
          const uint32_t old = __builtin_bswap32(v.le32(l3 + 12 + 4 * k));
          ipc = upd32(ipc, old, nw);
          if (l4ok && (proto == 6 || l4c != 0)) {   // UDP: a 0 checksum stays 0
            l4c = upd32(l4c, old, nw);
            l4c_w = true;
          }
          fw.put(l3 + 12 + 4 * k, nw, 4);
        }
        if (l4ok) {
#pragma unroll
          for (int k = 0; k < 2; ++k) {  // tcp/udp_set_src/dst_port_cksum_update (:263-347)
            const uint32_t op = k == 0 ? PPTK_RW_SPORT : PPTK_RW_DPORT;
            if (!(w.ops & op)) continue;
            const uint32_t nw = k == 0 ? w.sport : w.dport;
            if (proto == 6 || l4c != 0) {
              l4c = upd16(l4c, v.be16(l4 + 2 * k), nw);
              l4c_w = true;
            }
            fw.put(l4 + 2 * k, nw, 2);
          }
        }
        if ((w.ops & PPTK_RW_ICMP_ID) && proto == 1 && !(p.flags & PPTK_RX_F_FRAGMENT) &&
            p.re - p.rs >= 8u) {
          // icmp_set_echo_identifier_cksum_update (:283-291) on an echo
          // request / reply; the ICMP checksum has no pseudo-header, so the
          // address changes above leave it alone
          const uint32_t type = v.u8(l4);
          if (type == 8 || type == 0) {
            fw.put(l4 + 2, upd16(v.be16(l4 + 2), v.be16(l4 + 4), w.sport), 2);
            fw.put(l4 + 4, w.sport, 2);
            st |= PPTK_RW_ST_ICMP;
          }
        }
        if (w.ops & (PPTK_RW_DECR_TTL | PPTK_RW_SRC | PPTK_RW_DST))
          fw.put(l3 + 10, ipc, 2);
        if (l4c_w)
          fw.put(l4 + cko, l4c, 2);
        fw.flush(len);
      }
    }
    if (a.rw_status) a.rw_status[i] = (uint8_t)st;
  }
}

// TCP MSS clamping (pptk_tcp_mss_clamp_device): one lane per frame, the
// frame's first eight aligned chunks in the lane's LDS slot (Ethernet, IPv4
// or IPv6 with a VLAN tag and a 20-byte IP header leave the TCP options in
// it; longer headers reach the rest through the FrameView rare path), the
// receive transform's parse, tcp_parse_options (iphdr/iphdr.c:4-132) over
// the options, and tcp_set_mss_cksum_update (iphdr/ipcksum.h:466-489) when
// the MSS option exceeds the clamp.  Only clamped frames are written (four
// bytes: the option value and the checksum).
constexpr int MSS_SLOT = 128;

__global__ __launch_bounds__(256) void rx_mss_kernel(RxKArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[256 * (MSS_SLOT + 4)];
  LDS_AS uint8_t *slot = (LDS_AS uint8_t *)lds + threadIdx.x * (MSS_SLOT + 4);
  const uint64_t step = (uint64_t)gridDim.x * 256u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += step) {
    const uint64_t base = a.off ? a.off[i] : i * a.stride;
    const uint32_t len = a.len ? a.len[i] : a.fixed_len;
    const int m = (int)(base & 15);
    const int nch = max((m + (int)len + 15) >> 4, 1);
    park_chunks<MSS_SLOT>(slot, (const u32x4 *)(a.frames + (base - (uint64_t)m)), nch);
    const FrameView v = {slot, (const GLB_AS uint8_t *)a.frames + base, m, MSS_SLOT - m};
    const Parse p = parse_frame(v, len);
    uint32_t st = 0;
    if ((p.flags & (PPTK_RX_F_PARSED | PPTK_RX_F_MALFORMED | PPTK_RX_F_L4)) ==
            (PPTK_RX_F_PARSED | PPTK_RX_F_L4) &&
        p.proto == 6) {
      const int t = (int)p.rs;   // TCP header
      if (!(a.mss_flags & PPTK_MSS_SYN_ONLY) || (v.u8(t + 13) & 2u)) {
        st = PPTK_MSS_ST_TCP;
        const int end = (int)(v.u8(t + 12) >> 4) * 4;   // tcp_data_offset
        if (t + end > (int)p.re) {
          st |= PPTK_MSS_ST_BADOPT;   // options past the segment
        } else {
          // tcp_parse_options: kind 0 ends the list, kind 1 is a NOP, any
          // other option is min(length byte, bytes left) long (the bytes
          // left when its length byte is past the options) and the list is
          // malformed below 2; the last 4-byte MSS option counts
          int off = 20, mssoff = 0;
          uint32_t mssv = 536u;
          bool valid = true;
          // one exit branch per option: the kind, length and MSS bytes are
          // read unconditionally (a length byte past the options is not
          // used) and combined arithmetically
          auto walk = [&](auto rd) __attribute__((always_inline)) {
            while (off < end) {
              const uint32_t kind = rd(t + off), lb = rd(t + off + 1);
              const uint32_t mv = (rd(t + off + 2) << 8) | rd(t + off + 3);
              int L = off + 1 < end ? min(end - off, (int)lb) : 1;
              L = kind == 1 ? 1 : L;
              const bool bad = kind > 1 && L < 2;
              const bool is_mss = kind == 2 && L == 4;
              mssv = is_mss ? mv : mssv;
              mssoff = is_mss ? off : mssoff;
              if (kind == 0 || bad) {
                valid = !bad;
                break;
              }
              off += L;
            }
          };
          if (m + t + end <= MSS_SLOT) {
            // the whole option list (and 3 bytes past it, in the slot or
            // its 4 pad bytes) is in the LDS image: plain LDS reads
            const LDS_AS uint8_t *img = v.img + m;
            walk([&](int k) __attribute__((always_inline)) { return (uint32_t)img[k]; });
          } else {
            // long headers (IPv6 extension chains): reads past the image
            // come from global memory, clamped to the frame
            walk([&](int k) __attribute__((always_inline)) {
              return v.u8(min(k, (int)len - 1));
            });
          }
          if (!valid) {
            st |= PPTK_MSS_ST_BADOPT;
          } else if (mssoff) {
            st |= PPTK_MSS_ST_FOUND;
            if (mssv > a.mss) {
              // tcp_set_mss_cksum_update: a value at an even TCP offset is
              // one checksum word; at an odd offset it straddles two, each
              // updated with its other byte unchanged (that byte cancels in
              // the RFC 1624 sum, so a byte past the frame is taken as 0)
              const int f = t + mssoff + 2;
              uint32_t ck = v.be16(t + 16);
              if (!(mssoff & 1)) {
                ck = upd16(ck, mssv, a.mss);
              } else {
                const uint32_t x1 = v.u8(f - 1);
                const uint32_t x2 = f + 2 < (int)len ? v.u8(f + 2) : 0u;
                ck = upd16(ck, (x1 << 8) | (mssv >> 8), (x1 << 8) | (a.mss >> 8));
                ck = upd16(ck, ((mssv & 0xffu) << 8) | x2, ((a.mss & 0xffu) << 8) | x2);
              }
              GLB_AS uint8_t *fw = (GLB_AS uint8_t *)a.frames_w + base;
              // each field as one 16-bit store where its address is even.
              // The stores dominate this kernel: loading, parking, parsing
              // and walking 16 M SYNs takes 0.29 ms, the four byte stores
              // per frame added 0.35 ms; two 16-bit stores cut the total
              // 0.639 -> 0.577 ms; writing back the patched 16-byte image
              // chunks instead measured the same (0.575), non-temporal
              // 16-bit stores 2 % slower (tools/ab_mss.py, one box each)
              const uintptr_t fa = (uintptr_t)(fw + f), ca = (uintptr_t)(fw + t + 16);
              if (!(fa & 1)) {
                *(GLB_AS uint16_t *)(fw + f) = (uint16_t)bswap16(a.mss);
              } else {
                fw[f] = (uint8_t)(a.mss >> 8);
                fw[f + 1] = (uint8_t)a.mss;
              }
              if (!(ca & 1)) {
                *(GLB_AS uint16_t *)(fw + t + 16) = (uint16_t)bswap16(ck);
              } else {
                fw[t + 16] = (uint8_t)(ck >> 8);
                fw[t + 17] = (uint8_t)ck;
              }
              st |= PPTK_MSS_ST_CLAMPED;
            }
          }
        }
      }
    }
    if (a.rw_status) a.rw_status[i] = (uint8_t)st;
  }
}

// Descriptor sources of an offset-described (GATHER) launch: absent arrays
// read the context's zeroed stand-in buffer (RxKArgs::zero).
void gather_args(RxKArgs &a) {
  a.perm_ld = a.perm ? a.perm : (const uint32_t *)a.zero;
  a.perm_msk = a.perm ? ~0u : 0u;
  a.off_ld = a.off ? a.off : (const uint64_t *)a.zero;
  a.off_msk = a.off ? ~0u : 0u;
  a.stride_g = a.off ? 0u : a.stride;
  a.len_ld = a.len ? a.len : (const uint16_t *)a.zero;
  a.len_msk = a.len ? ~0u : 0u;
  a.fixed_g = a.len ? 0u : a.fixed_len;
}

template <int T, int S, int D, int AL>
hipError_t launch_variant(const RxKArgs &a0, int grid, hipStream_t s) {
  const dim3 gd(grid), bd(WAVE * WPB);
  RxKArgs a = a0;
  const bool nt = a.tune & 1u;
  const bool gather = a.off || a.len || a.perm;
  if (gather) {
    gather_args(a);
    if (nt) hipLaunchKernelGGL((rx_kernel<T, S, D, AL, true, true>), gd, bd, 0, s, a);
    else hipLaunchKernelGGL((rx_kernel<T, S, D, AL, false, true>), gd, bd, 0, s, a);
  } else {
    if (nt) hipLaunchKernelGGL((rx_kernel<T, S, D, AL, true, false>), gd, bd, 0, s, a);
    else hipLaunchKernelGGL((rx_kernel<T, S, D, AL, false, false>), gd, bd, 0, s, a);
  }
  return hipGetLastError();
}

template <int T, int S, int D, int AL>
int blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel<T, S, D, AL, true, true>,
                                                   WAVE * WPB, 0) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}

// variant table: T, S, D, AL
#define PPTK_RX_VARIANTS(X)       \
  X(RX_T4S1, 4, 1, 3, 4)          \
  X(RX_T4S2, 4, 2, 3, 4)          \
  X(RX_T16S2, 16, 2, 3, 4)        \
  X(RX_T16S6, 16, 6, 3, 4)        \
  X(RX_T32S3, 32, 3, 3, 4)        \
  X(RX_T64S2, 64, 2, 1, 4)        \
  X(RX_T16S7L, 16, 7, 1, 7)       \
  X(RX_T32S4L, 32, 4, 3, 7)       \
  X(RX_T32S3D7, 32, 3, 7, 4)      \
  X(RX_T16S6D1, 16, 6, 1, 4)       \
  X(RX_T8S2, 8, 2, 3, 4)          \
  X(RX_T16S4, 16, 4, 3, 4)

}  // namespace

// Two-pass tx, second pass: one thread per frame writes the (at most two)
// checksum fields the streaming pass left in txside -- the only writes of
// the operation, issued without a read stream beside them.
__global__ __launch_bounds__(256) void tx_apply_kernel(const uint64_t *__restrict__ side,
                                                       uint8_t *__restrict__ frames,
                                                       const uint64_t *__restrict__ off,
                                                       uint64_t stride, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = side[i];
    const uint64_t base = off ? off[i] : i * stride;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t f = (uint32_t)(e >> (32 * k));
      const uint32_t o = f & 0xffffu;
      if (o == 0xffffu) continue;
      uint8_t *p = frames + base + o;
      if (((uintptr_t)p & 1u) == 0) {
        *(uint16_t *)p = (uint16_t)bswap16(f >> 16);   // network order
      } else {
        p[0] = (uint8_t)(f >> 24);
        p[1] = (uint8_t)(f >> 16);
      }
    }
  }
}

hipError_t launch_tx_apply(const uint64_t *txside, uint8_t *frames, const uint64_t *off,
                           uint64_t stride, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(tx_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, txside, frames,
                     off, stride, n);
  return hipGetLastError();
}

hipError_t launch_rx(int variant, const RxKArgs &a, int grid, hipStream_t s) {
  if (variant == RX_M6) {
    const dim3 gd(grid), bd(WAVE * WPB);
    RxKArgs m = a;
    const bool nt = m.tune & 1u;
    if (m.off || m.len || m.perm) {
      gather_args(m);
      if (nt) hipLaunchKernelGGL((rx_kernel_mixed<true, true>), gd, bd, 0, s, m);
      else hipLaunchKernelGGL((rx_kernel_mixed<false, true>), gd, bd, 0, s, m);
    } else {
      if (nt) hipLaunchKernelGGL((rx_kernel_mixed<true, false>), gd, bd, 0, s, m);
      else hipLaunchKernelGGL((rx_kernel_mixed<false, false>), gd, bd, 0, s, m);
    }
    return hipGetLastError();
  }
  if (variant == RX_L4) {
    const dim3 gd(grid), bd(WAVE * WPB);
    if (a.tune & 1u) hipLaunchKernelGGL(rx_kernel_lane<true>, gd, bd, 0, s, a);
    else hipLaunchKernelGGL(rx_kernel_lane<false>, gd, bd, 0, s, a);
    return hipGetLastError();
  }
  switch (variant) {
#define X(name, T, S, D, AL) \
  case name: return launch_variant<T, S, D, AL>(a, grid, s);
    PPTK_RX_VARIANTS(X)
#undef X
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_rewrite(const RxKArgs &a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(rx_rewrite_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_mss_clamp(const RxKArgs &a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(rx_mss_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

bool rx_variant_phased(int variant) {
  switch (variant) {
#define X(name, T, S, D, AL) \
  case name: return S * T >= 32 && T <= 32;
    PPTK_RX_VARIANTS(X)
#undef X
    default: return false;   // M6, L4: no stash
  }
}

int rx_variant_blocks_per_cu(int variant) {
  if (variant == RX_M6) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel_mixed<false, true>, WAVE * WPB,
                                                     0) != hipSuccess)
      return 1;
    return nb > 0 ? nb : 1;
  }
  if (variant == RX_L4) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel_lane<false>, WAVE * WPB, 0) !=
        hipSuccess)
      return 1;
    return nb > 0 ? nb : 1;
  }
  switch (variant) {
#define X(name, T, S, D, AL) \
  case name: return blocks_per_cu<T, S, D, AL>();
    PPTK_RX_VARIANTS(X)
#undef X
    default: return 1;
  }
}

}  // namespace pptk
