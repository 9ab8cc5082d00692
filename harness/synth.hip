// synth.hip -- BENCH/TEST TOOLING (not part of libpptkrx.so).
//
// Writes synthetic Ethernet frames straight into HBM, one thread per frame,
// following SURVEY.md 8(d) and the reference's frame recipe
// (ldp/ldpsend.c:141-168: Eth + IPv4 DF TTL 64 + L4, checksums filled):
//   C64   64 B IPv4/UDP, 22 B random payload
//   C1500 1500 B IPv4/TCP (doff 5), 1446 B random payload
//   CMIX  64..1500 B, 70 % IPv4 / 30 % IPv6, 50/50 TCP/UDP, 25 % 802.1Q,
//         5 % IPv4 with IHL > 5, 2 % IPv6 with one hop-by-hop header
//   IMIX  the classic 7:4:1 mix of 64 / 576 / 1500 B frames, otherwise as
//         CMIX (a short frame grows to its headers' minimum, <= 102 B)
//   JMIX  CMIX with 2 % of the frames 9000-byte jumbo frames
// Checksums are computed here by a plain per-thread big-endian word sum
// (independent of the product kernel).  About 1 % of frames are corrupted
// (half in the IPv4 header, half in the L4 bytes); `expect` receives, per
// frame, bit0 = IP checksum should verify, bit1 = L4 checksum should verify.
// Everything derives from (seed, global frame index), so any shard of a
// multi-GPU run regenerates exactly its part of the global batch.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t s;
  __device__ uint64_t next() { s = mix64(s); return s; }
  __device__ uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * n >> 32); }
  __device__ bool chance(uint32_t per_mille) { return below(1000) < per_mille; }
};

struct Writer {
  uint8_t *f;
  __device__ void b8(int k, uint32_t v) { f[k] = (uint8_t)v; }
  __device__ void be16(int k, uint32_t v) { f[k] = (uint8_t)(v >> 8); f[k + 1] = (uint8_t)v; }
  __device__ uint32_t get_be16(int k) const { return ((uint32_t)f[k] << 8) | f[k + 1]; }
};

__device__ uint32_t fold(uint64_t s) {
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint32_t)s;
}

// big-endian word sum of f[a, b) (odd tail padded with zero)
__device__ uint64_t be_sum(const Writer &w, int a, int b) {
  uint64_t s = 0;
  int k = a;
  for (; k + 1 < b; k += 2) s += w.get_be16(k);
  if (k < b) s += (uint32_t)w.f[k] << 8;
  return s;
}

enum { CFG_C64 = 0, CFG_C1500 = 1, CFG_CMIX = 2, CFG_IMIX = 3, CFG_JMIX = 4 };

// Shape of frame `gi`: everything that determines its length.
struct Shape {
  uint32_t total, proto, ihl;
  bool v6, vlan, hbh;
};

__device__ Shape shape_of(int cfg, uint64_t seed, uint64_t gi) {
  Shape sh = {64, 17, 20, false, false, false};
  if (cfg == CFG_C1500) {
    sh.total = 1500;
    sh.proto = 6;
  } else if (cfg == CFG_CMIX || cfg == CFG_IMIX || cfg == CFG_JMIX) {
    Rng r{mix64(seed ^ (gi * 0xd1b54a32d192ed03ULL)) ^ 0x51e5};
    uint32_t size = 64 + r.below(1437);
    if (cfg == CFG_IMIX) {
      const uint32_t u = size % 12;   // (the same draw, reused)
      size = u < 7 ? 64 : u < 11 ? 576 : 1500;
    } else if (cfg == CFG_JMIX && size % 50 == 7) {   // (the same draw: 2 %)
      size = 9000;
    }
    sh.proto = r.chance(500) ? 6 : 17;
    sh.vlan = r.chance(250);
    sh.v6 = r.chance(300);
    if (!sh.v6 && r.chance(50)) sh.ihl = 4 * (6 + r.below(10));
    if (sh.v6 && r.chance(20)) sh.hbh = true;
    const uint32_t minsz = (sh.vlan ? 18 : 14) + (sh.v6 ? 40 + (sh.hbh ? 8 : 0) : sh.ihl) +
                           (sh.proto == 6 ? 20 : 8);
    sh.total = size < minsz ? minsz : size;
  }
  return sh;
}

__global__ void sizes_kernel(int cfg, uint64_t seed, uint64_t first, uint64_t n, uint16_t *len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) len[i] = (uint16_t)shape_of(cfg, seed, first + i).total;
}

__global__ void gen_kernel(int cfg, uint64_t seed, uint64_t first, uint64_t n, uint8_t *buf,
                           const uint64_t *off, uint64_t stride, uint8_t *expect) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t gi = first + i;
  const Shape sh = shape_of(cfg, seed, gi);
  Writer w{buf + (off ? off[i] : i * stride)};
  Rng r{mix64(seed * 0x2545F4914F6CDD1DULL + gi)};
  const bool v6 = sh.v6, vlan = sh.vlan, hbh = sh.hbh;
  const uint32_t proto = sh.proto, ihl = sh.ihl, total = sh.total;
  // Ethernet
  const uint64_t mac = r.next();
  for (int k = 0; k < 6; ++k) { w.b8(k, 0x02 + (k == 0 ? 0 : (uint32_t)(mac >> (8 * k)))); }
  for (int k = 6; k < 12; ++k) w.b8(k, (uint32_t)(mac >> (8 * (k - 6))) | (k == 6 ? 2 : 0));
  int l3 = 14;
  if (vlan) {
    w.be16(12, 0x8100);
    w.be16(14, 1 + r.below(4094));
    l3 = 18;
  }
  w.be16(l3 - 2, v6 ? 0x86dd : 0x0800);
  const uint32_t l4min = proto == 6 ? 20 : 8;
  int l4;
  uint32_t l4len;
  uint64_t pseudo;
  if (!v6) {
    l4 = l3 + ihl;
    l4len = total - l4;
    w.b8(l3, 0x40 | (ihl / 4));
    w.b8(l3 + 1, 0);
    w.be16(l3 + 2, ihl + l4len);
    w.be16(l3 + 4, (uint32_t)r.below(65536));
    w.be16(l3 + 6, 0x4000);                 // DF
    w.b8(l3 + 8, 64);
    w.b8(l3 + 9, proto);
    w.be16(l3 + 10, 0);
    const uint32_t src = 0x0a000000u | r.below(1u << 24);
    const uint32_t dst = 0xc0a80000u | r.below(1u << 16);
    w.be16(l3 + 12, src >> 16); w.be16(l3 + 14, src & 0xffff);
    w.be16(l3 + 16, dst >> 16); w.be16(l3 + 18, dst & 0xffff);
    for (int k = l3 + 20; k < l4; ++k) w.b8(k, (uint32_t)r.next());   // options
    w.be16(l3 + 10, ~fold(be_sum(w, l3, l3 + ihl)) & 0xffff);
    pseudo = (src >> 16) + (src & 0xffff) + (dst >> 16) + (dst & 0xffff) + proto + l4len;
  } else {
    const int ext = hbh ? 8 : 0;
    l4 = l3 + 40 + ext;
    l4len = total - l4;
    w.b8(l3, 0x60); w.b8(l3 + 1, 0); w.be16(l3 + 2, 0);
    w.be16(l3 + 4, ext + l4len);
    w.b8(l3 + 6, hbh ? 0 : proto);
    w.b8(l3 + 7, 64);
    const uint64_t a = r.next(), b = r.next(), c = r.next();
    for (int k = 0; k < 16; ++k) w.b8(l3 + 8 + k, k < 2 ? (k ? 0x01 : 0x20) : (uint32_t)(a >> (8 * (k & 7))) ^ (uint32_t)(b >> (8 * (k >> 1))));
    for (int k = 0; k < 16; ++k) w.b8(l3 + 24 + k, k == 0 ? 0xfd : (uint32_t)(c >> (8 * (k & 7))) + k);
    if (hbh) {
      const int h = l3 + 40;
      w.b8(h, proto); w.b8(h + 1, 0); w.b8(h + 2, 1); w.b8(h + 3, 4);
      for (int k = 4; k < 8; ++k) w.b8(h + k, 0);
    }
    pseudo = be_sum(w, l3 + 8, l3 + 40) + (l4len >> 16) + (l4len & 0xffff) + proto;
  }
  // L4 header + payload
  const uint32_t sp = r.below(65536), dp = r.below(65536);
  w.be16(l4, sp);
  w.be16(l4 + 2, dp);
  int ck;
  if (proto == 6) {
    const uint64_t sq = r.next();
    w.be16(l4 + 4, (uint32_t)(sq >> 16)); w.be16(l4 + 6, (uint32_t)sq);
    w.be16(l4 + 8, 0); w.be16(l4 + 10, 0);
    w.b8(l4 + 12, 0x50); w.b8(l4 + 13, 0x18);
    w.be16(l4 + 14, 8192);
    w.be16(l4 + 18, 0);
    ck = l4 + 16;
  } else {
    w.be16(l4 + 4, l4len);
    ck = l4 + 6;
  }
  w.be16(ck, 0);
  uint64_t s = pseudo;
  for (int k = l4; k < l4 + (int)l4min; k += 2) s += w.get_be16(k);
  // payload: 8 random bytes per draw, summed as they are written
  int k = l4 + (int)l4min;
  const int end = l4 + (int)l4len;
  while (k < end) {
    const uint64_t v = r.next();
    for (int t = 0; t < 8 && k < end; ++t, ++k) {
      const uint32_t byte = (uint32_t)(v >> (8 * t)) & 0xff;
      w.b8(k, byte);
      s += ((k - l4) & 1) ? byte : byte << 8;
    }
  }
  uint32_t c = ~fold(s) & 0xffff;
  if (proto == 17 && c == 0) c = 0xffff;
  w.be16(ck, c);
  // corruption: ~0.5 % IPv4 header, ~0.5 % L4 bytes
  uint8_t ex = 3;
  const uint32_t u = r.below(1000);
  if (u < 5 && !v6) {
    w.b8(l3 + 4, w.f[l3 + 4] ^ 0x01);
    ex &= ~1;
  } else if (u < 10) {
    const int pos = l4 + (int)r.below(l4len);
    w.b8(pos, w.f[pos] ^ 0xff);
    ex &= ~2;
  }
  if (expect) expect[i] = ex;
}

}  // namespace

extern "C" {

// lengths of frames [first, first + n) of config cfg
int synth_sizes(int cfg, uint64_t seed, uint64_t first, uint64_t n, uint16_t *d_len, void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(sizes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cfg, seed, first, n, d_len);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// frames [first, first + n): at d_off[i] (or i * stride when d_off is NULL)
int synth_frames(int cfg, uint64_t seed, uint64_t first, uint64_t n, uint8_t *d_buf,
                 const uint64_t *d_off, uint64_t stride, uint8_t *d_expect, void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gen_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cfg, seed, first, n, d_buf, d_off, stride, d_expect);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
