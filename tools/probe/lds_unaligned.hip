// tools/probe/lds_unaligned.hip -- does gfx950 LDS serve a ds_read_b32 /
// ds_read_u16 at a byte address that is not a multiple of 4 / 2 with the
// bytes at that address (unaligned access mode), or with the aligned word
// around it?  The parse reads 4 bytes at arbitrary byte positions; today that
// is ds_read2_b32 of the two aligned words + v_alignbyte.
//   A  ds_read_b32 at byte a = 4*t + lane (t = trial) -> compare with bytes a..a+3
//   B  ds_read_b32 at byte a = 4*t + 3*lane + 1
//   C  ds_read_u16 at odd bytes
// Build: hipcc --offload-arch=gfx950 -O2 -o lds_unaligned lds_unaligned.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(uint32_t* outA, uint32_t* outB, uint32_t* outC) {
  __shared__ uint8_t b[1024];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 1024; i += 64) b[i] = (uint8_t)(i * 7u + 3u);
  __syncthreads();
  for (uint32_t t = 0; t < 8; t++) {
    uint32_t a = 4u * t + lane, ra, rb, rc;
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)b;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(ra) : "v"(base + a) : "memory");
    const uint32_t a2 = 4u * t + 3u * lane + 1u;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(rb) : "v"(base + a2) : "memory");
    const uint32_t a3 = 2u * (t + lane) + 1u;
    asm volatile("ds_read_u16 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(rc) : "v"(base + a3) : "memory");
    outA[t * 64 + lane] = ra;
    outB[t * 64 + lane] = rb;
    outC[t * 64 + lane] = rc;
  }
}

int main() {
  uint32_t *dA, *dB, *dC;
  hipMalloc(&dA, 8 * 64 * 4);
  hipMalloc(&dB, 8 * 64 * 4);
  hipMalloc(&dC, 8 * 64 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  std::vector<uint32_t> A(512), B(512), C(512);
  hipMemcpy(A.data(), dA, 2048, hipMemcpyDeviceToHost);
  hipMemcpy(B.data(), dB, 2048, hipMemcpyDeviceToHost);
  hipMemcpy(C.data(), dC, 2048, hipMemcpyDeviceToHost);
  auto byte = [](uint32_t i) { return (uint32_t)(uint8_t)(i * 7u + 3u); };
  auto w4 = [&](uint32_t a) { return byte(a) | byte(a + 1) << 8 | byte(a + 2) << 16 | byte(a + 3) << 24; };
  int exA = 0, alA = 0, exB = 0, alB = 0, exC = 0, alC = 0;
  for (uint32_t t = 0; t < 8; t++)
    for (uint32_t l = 0; l < 64; l++) {
      const uint32_t a = 4 * t + l, a2 = 4 * t + 3 * l + 1, a3 = 2 * (t + l) + 1;
      exA += A[t * 64 + l] == w4(a);
      alA += A[t * 64 + l] == w4(a & ~3u);
      exB += B[t * 64 + l] == w4(a2);
      alB += B[t * 64 + l] == w4(a2 & ~3u);
      exC += C[t * 64 + l] == (w4(a3) & 0xffffu);
      alC += C[t * 64 + l] == (w4(a3 & ~1u) & 0xffffu);
    }
  printf("{\"b32_exact\": %d, \"b32_aligned\": %d, \"b32b_exact\": %d, \"b32b_aligned\": %d, "
         "\"u16_exact\": %d, \"u16_aligned\": %d, \"of\": 512}\n", exA, alA, exB, alB, exC, alC);
  return 0;
}
