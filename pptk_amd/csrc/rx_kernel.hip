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

namespace pptk {

namespace {

constexpr int WAVE = 64;
constexpr int WPB = 4;            // waves per block (256 threads)
constexpr int IMG_CHUNKS = 8;     // 16-byte chunks parked in LDS per frame
constexpr int IMG_STRIDE = 144;   // LDS bytes per frame slot (9 x 16: no b128 bank conflicts)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int b) {
  return (x << b) | (x >> (64 - b));
}

struct Sip {
  uint64_t v0, v1, v2, v3;
  __device__ __forceinline__ Sip(uint64_t k0, uint64_t k1)
      : v0(0x736f6d6570736575ULL ^ k0), v1(0x646f72616e646f6dULL ^ k1),
        v2(0x6c7967656e657261ULL ^ k0), v3(0x7465646279746573ULL ^ k1) {}
  __device__ __forceinline__ void round() {
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);
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

// A frame as seen by a lane: bytes [0, lim) from the LDS image (frame byte k
// at img[m + k], image = aligned 16-byte chunks from floor16(frame start)),
// everything else straight from global memory.
struct FrameView {
  const uint8_t *img;
  const uint8_t *g;
  int m;
  int lim;

  __device__ __forceinline__ uint32_t u8(int k) const {
    return k < lim ? (uint32_t)img[m + k] : (uint32_t)g[k];
  }
  __device__ __forceinline__ uint32_t be16(int k) const {
    return (u8(k) << 8) | u8(k + 1);
  }
  // 4 frame bytes at offset k as a little-endian dword (hdr_get32h).
  __device__ __forceinline__ uint32_t le32(int k) const {
    if (k + 4 <= lim) {
      const int a = m + k;
      const uint32_t *p = (const uint32_t *)(img + (a & ~3));
      return __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)(a & 3));
    }
    return (uint32_t)g[k] | ((uint32_t)g[k + 1] << 8) | ((uint32_t)g[k + 2] << 16) |
           ((uint32_t)g[k + 3] << 24);
  }
};

// Structural parse of one frame (the branchy part of DESIGN.md "Record
// semantics"): where L3/L4 are, what they are, and whether the L4 sum
// applies.  IP_OK / L4_OK / UDP_ZERO are decided later by the owning lane.
struct Parse {
  uint32_t flags, l3, ver, et, proto, rs, re;
};

__device__ __forceinline__ bool is_v6_ext(uint32_t nh) {
  // is_ipv6_nexthdr, iphdr/iphdr.h:717-727
  return nh == 0 || nh == 60 || nh == 43 || nh == 44 || nh == 51;
}

__device__ Parse parse_frame(const FrameView &v, uint32_t len) {
  Parse p = {0, 0, 0, 0, 0, 0, 0};
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
        return p;
      }
      if (nh == 44) {
        frag = 1;
        if ((v.be16(l3 + off + 2) & 0xfff8u) > 0)
          break;
      }
      nh = v.u8(l3 + off);
      const uint32_t lf = v.u8(l3 + off + 1);
      const uint32_t extlen = nh == 44 ? 8u : (nh == 51 ? lf * 4u + 8u : lf * 8u + 8u);
      if (off + extlen > tlen) {
        p.flags |= PPTK_RX_F_MALFORMED;
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

// Sum the bytes of one aligned 16-byte chunk that fall inside the frame
// region [rs, re); `o` is the chunk's frame-relative offset (may be < 0).
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
      const int lo = min(max(rs - od, 0), 4);
      const int hi = min(max(re - od, 0), 4);
      const uint32_t mk = (uint32_t)(((1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull));
      acc = dot16(c[d] & mk, acc);
    }
  }
  return acc;
}

template <int T>
__device__ __forceinline__ uint32_t team_sum(uint32_t x) {
#pragma unroll
  for (int d = T / 2; d >= 1; d >>= 1)
    x += __shfl_xor(x, d, T);
  return x;
}

template <int T, int S>
__global__ __launch_bounds__(WAVE * WPB) void rx_kernel(RxKArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * WAVE * IMG_STRIDE];
  constexpr int IMGC = (S * T < IMG_CHUNKS) ? S * T : IMG_CHUNKS;  // chunks parked
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = threadIdx.x / WAVE;
  const int g = lane / T, j = lane % T;
  uint8_t *wimg = lds + wv * WAVE * IMG_STRIDE;
  const uint64_t ntiles = (a.n + WAVE - 1) / WAVE;
  const uint64_t nwaves = (uint64_t)gridDim.x * WPB;

  for (uint64_t tile = (uint64_t)blockIdx.x * WPB + wv; tile < ntiles; tile += nwaves) {
    // ---- the lane's own frame
    const uint64_t i = tile * WAVE + lane;
    const bool valid = i < a.n;
    const uint32_t idx = valid ? (a.perm ? a.perm[i] : (uint32_t)i) : 0u;
    const uint64_t base = valid ? (a.off ? a.off[idx] : (uint64_t)idx * a.stride) : 0ull;
    const uint32_t flen = valid ? (a.len ? (uint32_t)a.len[idx] : a.fixed_len) : 0u;

    uint32_t my_sum = 0, my_p0 = 0, my_p1 = 0, my_p2 = 0;

    // ---- streaming rounds: team g sums frame g*T + r
    u32x4 cur[S];
    uint64_t cb;
    uint32_t cl;
    {
      const int q = g * T;
      cb = __shfl(base, q);
      cl = __shfl(flen, q);
      const int m = (int)(cb & 15);
      const u32x4 *c0 = (const u32x4 *)(a.frames + (cb - (uint64_t)m));
      const int nch = (m + (int)cl + 15) >> 4;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int c = s * T + j;
        cur[s] = c < nch ? c0[c] : (u32x4){0, 0, 0, 0};
      }
    }
#pragma unroll 1
    for (int r = 0; r < T; ++r) {
      const int q = g * T + r;
      const uint64_t pb = cb;
      const uint32_t pl = cl;
      // issue the next round's loads first
      u32x4 nxt[S];
      if (r + 1 < T) {
        cb = __shfl(base, q + 1);
        cl = __shfl(flen, q + 1);
        const int mn = (int)(cb & 15);
        const u32x4 *c0n = (const u32x4 *)(a.frames + (cb - (uint64_t)mn));
        const int nchn = (mn + (int)cl + 15) >> 4;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int c = s * T + j;
          nxt[s] = c < nchn ? c0n[c] : (u32x4){0, 0, 0, 0};
        }
      }
      const int m = (int)(pb & 15);
      const int nch = (m + (int)pl + 15) >> 4;
      uint8_t *img = wimg + q * IMG_STRIDE;
      // park the first IMGC chunks of the frame in LDS
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s * T < IMGC) {
          const int c = s * T + j;
          if (c < IMGC)
            *(u32x4 *)(img + 16 * c) = cur[s];
        }
      }
      __builtin_amdgcn_wave_barrier();
      const uint8_t *gf = a.frames + pb;
      const FrameView v = {img, gf, m, 16 * IMGC - m};
      const Parse p = parse_frame(v, pl);
      int rs = 0, re = 0;
      if (p.flags & PPTK_RX_F_L4) {
        rs = (int)p.rs;
        re = (int)p.re;
      }
      uint32_t acc = 0;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int c = s * T + j;
        if (c < nch)
          acc = sum_chunk(cur[s], 16 * c - m, rs, re, acc);
      }
      if (nch > S * T) {  // long frames: unbuffered tail
        const u32x4 *c0 = (const u32x4 *)(a.frames + (pb - (uint64_t)m));
        for (int c = S * T + j; c < nch; c += T)
          acc = sum_chunk(c0[c], 16 * c - m, rs, re, acc);
      }
      acc = team_sum<T>(acc);
      if (j == r) {
        my_sum = acc;
        my_p0 = p.flags | (p.l3 << 16) | (p.ver << 24);
        my_p1 = p.rs | (p.re << 16);
        my_p2 = p.et | (p.proto << 16);
      }
      if (r + 1 < T) {
#pragma unroll
        for (int s = 0; s < S; ++s)
          cur[s] = nxt[s];
      }
      __builtin_amdgcn_wave_barrier();
    }

    // ---- lane phase: frame `lane` -> record
    if (!valid)
      continue;
    uint32_t flags = my_p0 & 0xffffu;
    const uint32_t l3 = (my_p0 >> 16) & 0xffu, ver = my_p0 >> 24;
    const uint32_t rs = my_p1 & 0xffffu, re = my_p1 >> 16;
    const uint32_t et = my_p2 & 0xffffu, proto = my_p2 >> 16;
    const int m = (int)(base & 15);
    const FrameView v = {wimg + lane * IMG_STRIDE, a.frames + base, m, 16 * IMGC - m};

    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = 0;
    uint64_t fh = 0;
    if (flags & PPTK_RX_F_MALFORMED) {
      flags &= PPTK_RX_F_MALFORMED | PPTK_RX_F_VLAN | PPTK_RX_F_IPV6;
    } else if (flags & PPTK_RX_F_PARSED) {
      const bool v6 = flags & PPTK_RX_F_IPV6;
      uint32_t s0, s1 = 0, s2 = 0, s3 = 0, d0, d1 = 0, d2 = 0, d3 = 0;
      uint32_t ipc = 0;
      if (v6) {
        s0 = v.le32(l3 + 8);  s1 = v.le32(l3 + 12); s2 = v.le32(l3 + 16); s3 = v.le32(l3 + 20);
        d0 = v.le32(l3 + 24); d1 = v.le32(l3 + 28); d2 = v.le32(l3 + 32); d3 = v.le32(l3 + 36);
      } else {
        s0 = v.le32(l3 + 12);
        d0 = v.le32(l3 + 16);
        // ip_hdr_cksum_calc over ihl = rs - l3 bytes
        uint32_t hs = 0;
        for (uint32_t k = l3; k < rs; k += 4)
          hs = dot16(v.le32((int)k), hs);
        ipc = finish16(hs);
        if (ipc == 0)
          flags |= PPTK_RX_F_IP_OK;
      }
      uint32_t ports = 0, l4c = 0;
      if (flags & PPTK_RX_F_L4) {
        ports = v.le32((int)rs);
        const uint32_t l4len = re - rs;
        uint32_t ps = dot16(s0, 0);
        ps = dot16(s1, ps); ps = dot16(s2, ps); ps = dot16(s3, ps);
        ps = dot16(d0, ps); ps = dot16(d1, ps); ps = dot16(d2, ps); ps = dot16(d3, ps);
        ps += bswap16(proto) + bswap16(l4len);
        uint32_t rsum = fold16(my_sum);
        if ((m + (int)rs) & 1)
          rsum = bswap16(rsum);
        l4c = finish16(ps + rsum);
        if (l4c == 0)
          flags |= PPTK_RX_F_L4_OK;
        if (proto == 17 && (v.le32((int)rs + 4) >> 16) == 0)
          flags |= PPTK_RX_F_UDP_ZERO;
      }
      Sip sh(a.k0, a.k1);
      sh.block((uint64_t)s0 | ((uint64_t)s1 << 32));
      sh.block((uint64_t)s2 | ((uint64_t)s3 << 32));
      sh.block((uint64_t)d0 | ((uint64_t)d1 << 32));
      sh.block((uint64_t)d2 | ((uint64_t)d3 << 32));
      sh.block((uint64_t)ports | ((uint64_t)proto << 32));
      fh = sh.finish(40ull << 56);
      uint32_t bucket = 0;
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
    if (a.hash)
      a.hash[idx] = fh;
    w[13] |= l3 | (flags << 16);
    w[15] = et | (ver << 16);
    u32x4 *dst = (u32x4 *)((uint8_t *)a.recs + (uint64_t)idx * 64u);
    dst[0] = (u32x4){w[0], w[1], w[2], w[3]};
    dst[1] = (u32x4){w[4], w[5], w[6], w[7]};
    dst[2] = (u32x4){w[8], w[9], w[10], w[11]};
    dst[3] = (u32x4){w[12], w[13], w[14], w[15]};
  }
}

template <int T, int S>
hipError_t launch_variant(const RxKArgs &a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((rx_kernel<T, S>), dim3(grid), dim3(WAVE * WPB), 0, s, a);
  return hipGetLastError();
}

template <int T, int S>
int blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel<T, S>, WAVE * WPB, 0) !=
      hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}

}  // namespace

hipError_t launch_rx(int variant, const RxKArgs &a, int grid, hipStream_t s) {
  switch (variant) {
    case RX_T4S1: return launch_variant<4, 1>(a, grid, s);
    case RX_T4S2: return launch_variant<4, 2>(a, grid, s);
    case RX_T16S2: return launch_variant<16, 2>(a, grid, s);
    case RX_T16S6: return launch_variant<16, 6>(a, grid, s);
    case RX_T64S2: return launch_variant<64, 2>(a, grid, s);
    default: return hipErrorInvalidValue;
  }
}

int rx_variant_blocks_per_cu(int variant) {
  switch (variant) {
    case RX_T4S1: return blocks_per_cu<4, 1>();
    case RX_T4S2: return blocks_per_cu<4, 2>();
    case RX_T16S2: return blocks_per_cu<16, 2>();
    case RX_T16S6: return blocks_per_cu<16, 6>();
    case RX_T64S2: return blocks_per_cu<64, 2>();
    default: return 1;
  }
}

}  // namespace pptk
