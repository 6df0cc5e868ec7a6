// kingdb_amd/csrc/crc_device.h -- CRC32C on a wavefront (crc32c::Extend,
// /root/reference/algorithm/crc32c.cc:296-340: reflected Castagnoli, register
// pre/post-inverted), for the write path (put.hip) and the read path (get.hip).
//
// One message per wave: the message is seen as 64 equal lane chunks of 2^lg
// bytes after zero padding at the FRONT (zero bytes leave a raw CRC register
// of 0 unchanged); each lane runs the byte-table loop over its chunk from a 0
// register, and six tree levels combine neighbours with GF(2) "advance over
// 2^k zero bytes" matrices: raw(A||B) = shift(raw(A), |B|) ^ raw(B).  The
// initial value enters as shift(init ^ ~0, n).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_device.h"

namespace kdb_lz4 {
namespace crc {

struct Tables {
  uint32_t t[256];
  uint32_t shift[32][32];   // column b of the matrix advancing a register over 2^k zero bytes
};
constexpr Tables make_tables() {
  Tables c{};
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t v = i;
    for (int k = 0; k < 8; k++) v = (v >> 1) ^ (0x82F63B78u & (0u - (v & 1u)));
    c.t[i] = v;
  }
  for (int b = 0; b < 32; b++) {
    const uint32_t v = 1u << b;
    c.shift[0][b] = c.t[v & 0xffu] ^ (v >> 8);
  }
  for (int k = 1; k < 32; k++)
    for (int b = 0; b < 32; b++) {
      uint32_t v = c.shift[k - 1][b], r = 0;
      for (int j = 0; j < 32; j++)
        if ((v >> j) & 1u) r ^= c.shift[k - 1][j];
      c.shift[k][b] = r;
    }
  return c;
}
static __constant__ Tables kTab = make_tables();

__device__ __forceinline__ uint32_t shift_pow2(uint32_t c, uint32_t k) {   // advance over 2^k zero bytes
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 32; b++) r ^= ((c >> b) & 1u) ? kTab.shift[k][b] : 0u;
  return r;
}
__device__ __forceinline__ uint32_t shift_n(uint32_t c, uint64_t n) {       // advance over n zero bytes
  for (uint32_t k = 0; n; k++, n >>= 1)
    if (n & 1u) c = shift_pow2(c, k);
  return c;
}

// The 256-entry table staged in LDS by the calling block.
__device__ __forceinline__ void stage_table(uint32_t* s_t) {
  for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) s_t[i] = kTab.t[i];
}

// crc32c::Extend(init, msg[0 .. n)).  Msg::feed(a, b, c, s_t) runs the
// byte-table loop over message bytes [a, b) on register c and returns it.
template <class Msg>
__device__ uint32_t extend_wave(uint32_t init, uint64_t n, const Msg& msg, const uint32_t* s_t) {
  const uint32_t lane = lane_id();
  uint32_t lg = 0;
  while ((64ull << lg) < n) lg++;
  const uint64_t L = 1ull << lg, z = 64ull * L - n;
  uint32_t c = 0;
  const uint64_t a = (uint64_t)lane * L, b = a + L;
  if (b > z) c = msg.feed(a > z ? a - z : 0u, b - z, 0u, s_t);
#pragma unroll
  for (uint32_t s = 0; s < 6; s++) {
    const uint32_t other = (uint32_t)__shfl_xor((int)c, 1 << s);
    if ((lane & (1u << s)) == 0) c = shift_pow2(c, lg + s) ^ other;
  }
  const uint32_t raw = uni(c);
  return raw ^ shift_n(init ^ 0xFFFFFFFFu, n) ^ 0xFFFFFFFFu;
}

__device__ __forceinline__ uint32_t step(uint32_t c, uint32_t byte, const uint32_t* s_t) {
  return s_t[(c ^ byte) & 0xffu] ^ (c >> 8);
}

// Slice-by-4: t[k][i] is the register after byte i and k zero bytes, so four
// message bytes (one little-endian dword) take four independent lookups
// instead of four dependent ones.
struct Tables4 {
  uint32_t t[4][256];
};
constexpr Tables4 make_tables4() {
  Tables4 s{};
  const Tables b = make_tables();
  for (uint32_t i = 0; i < 256; i++) s.t[0][i] = b.t[i];
  for (int k = 1; k < 4; k++)
    for (uint32_t i = 0; i < 256; i++) s.t[k][i] = (s.t[k - 1][i] >> 8) ^ s.t[0][s.t[k - 1][i] & 0xffu];
  return s;
}
static __constant__ Tables4 kTab4 = make_tables4();

// The four 256-entry tables (4 KiB) staged in LDS by the calling block.
__device__ __forceinline__ void stage_table4(uint32_t* s4) {
  for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) s4[i] = kTab4.t[i >> 8][i & 0xffu];
}
// the register after the four bytes of w (byte 0 first)
__device__ __forceinline__ uint32_t step4(uint32_t c, uint32_t w, const uint32_t* s4) {
  c ^= w;
  return s4[768u + (c & 0xffu)] ^ s4[512u + ((c >> 8) & 0xffu)] ^ s4[256u + ((c >> 16) & 0xffu)] ^ s4[c >> 24];
}

}  // namespace crc
}  // namespace kdb_lz4
