// kingdb_amd/csrc/datagen.hip -- synthetic benchmark values on the device.
//
// G1 = db_bench's value generator (/root/reference/doc/bench/db_bench_kingdb.cc:
// 113-142): LevelDB Random(301) (Park-Miller, A = 16807, M = 2^31 - 1) feeding
// test::CompressibleString(ratio 0.5, len 100) = 50 chars ' ' + Uniform(95),
// repeated to 100 bytes.  Each piece consumes exactly 50 draws, so piece j
// starts from x0 * A^(50 j) mod M: pieces are generated independently (one
// thread each) by jump-ahead, giving the same bytes as the sequential
// generator for a pool of any length ("G1-long").
#include <hip/hip_runtime.h>

#include <cstdint>

namespace kdb_lz4 {

namespace {
constexpr uint64_t kM = 2147483647ull;

__device__ __forceinline__ uint64_t mulmod(uint64_t a, uint64_t b) {
  uint64_t p = a * b;
  uint64_t r = (p >> 31) + (p & kM);
  while (r >= kM) r -= kM;
  return r;
}

__device__ __forceinline__ uint64_t powmod(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mulmod(r, a);
    a = mulmod(a, a);
    e >>= 1;
  }
  return r;
}

__global__ __launch_bounds__(256) void gen_g1_kernel(uint8_t* __restrict__ dst, uint64_t first_piece,
                                                     uint64_t npieces, uint32_t seed0) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= npieces) return;
  const uint64_t piece = first_piece + j;
  uint64_t s = seed0 & 0x7fffffffu;
  if (s == 0 || s == kM) s = 1;
  s = mulmod(s, powmod(16807u, (50ull * piece) % (kM - 1)));  // ord(A) divides M-1
  uint32_t words[25];
#pragma unroll
  for (int w = 0; w < 25; ++w) words[w] = 0;
#pragma unroll
  for (int i = 0; i < 50; ++i) {
    s = mulmod(s, 16807u);
    words[i >> 1] |= (uint32_t)(' ' + (uint32_t)(s % 95u)) << (8 * (i & 1));
  }
  // piece = raw(50) raw(50): assemble 100 bytes as 25 dwords
  uint8_t* o = dst + j * 100u;
  uint32_t out[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int idx = (4 * k + b) % 50;
      const uint32_t byte = (words[idx >> 1] >> (8 * (idx & 1))) & 0xffu;
      v |= byte << (8 * b);
    }
    out[k] = v;
  }
  if ((reinterpret_cast<uintptr_t>(o) & 3u) == 0) {
    uint32_t* o4 = reinterpret_cast<uint32_t*>(o);
#pragma unroll
    for (int k = 0; k < 25; ++k) o4[k] = out[k];
  } else {
#pragma unroll
    for (int k = 0; k < 100; ++k) o[k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
  }
}
}  // namespace

hipError_t launch_gen_g1(uint8_t* dst, uint64_t first_piece, uint64_t npieces, uint32_t seed,
                         hipStream_t st) {
  if (npieces == 0) return hipSuccess;
  const uint64_t blocks = (npieces + 255) / 256;
  hipLaunchKernelGGL(gen_g1_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, dst, first_piece, npieces,
                     seed);
  return hipGetLastError();
}

}  // namespace kdb_lz4
