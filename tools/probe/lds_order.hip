// tools/probe/lds_order.hip -- probes how gfx950 LDS resolves several lanes of
// ONE wave instruction hitting the same address (the compressor's same-slot
// grouping could lean on it).  Per trial: 64 lanes draw random slots in [0, K);
// checks, against a host model of "lanes processed in ascending order":
//   A  ds_write_b8: the surviving byte is the highest lane's
//   B  ds_or_rtn_b64: lane i gets the OR of the lower same-slot lanes' bits
//   C  ds_mskor_b32 (nibble field per slot): the surviving nibble is the highest lane's
//   D  ds_max_rtn_u32 with increasing values: lane i gets the max of lower lanes
// Build: hipcc --offload-arch=gfx950 -O2 -o lds_order lds_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(const uint32_t* slots, uint32_t trials, uint32_t* outA, uint64_t* outB, uint32_t* outC,
                      uint32_t* outD) {
  __shared__ uint8_t b8[256];
  __shared__ uint64_t b64[64];
  __shared__ uint32_t w32[64];
  __shared__ uint32_t m32[64];
  const uint32_t lane = threadIdx.x;
  for (uint32_t t = 0; t < trials; t++) {
    const uint32_t s = slots[t * 64 + lane];
    if (lane < 64) { b64[lane] = 0; w32[lane] = 0; m32[lane] = 0; }
    for (uint32_t i = lane; i < 256; i += 64) b8[i] = 0xff;
    __syncthreads();
    b8[s] = (uint8_t)lane;                                                      // A
    const uint64_t r = __hip_atomic_fetch_or(&b64[s], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // B
    const uint32_t sh = 0;
    // C: masked or of a 6-bit field (lane) at bits [0,6) of word s
    {
      uint32_t mask = 63u << sh, data = lane << sh;
      typedef __attribute__((address_space(3))) uint32_t lds_u32;
      const uint32_t a = (uint32_t)(uintptr_t)(lds_u32*)&w32[s];   // LDS byte offset
      asm volatile("ds_mskor_b32 %0, %1, %2\n s_waitcnt lgkmcnt(0)" :: "v"(a), "v"(mask), "v"(data) : "memory");
    }
    const uint32_t d = __hip_atomic_fetch_max(&m32[s], lane + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // D
    __syncthreads();
    outB[t * 64 + lane] = r;
    outD[t * 64 + lane] = d;
    outA[t * 64 + lane] = b8[s];
    outC[t * 64 + lane] = w32[s];
    __syncthreads();
  }
}

int main() {
  const uint32_t trials = 2000;
  std::vector<uint32_t> slots(trials * 64);
  srand(7);
  for (uint32_t t = 0; t < trials; t++) {
    const uint32_t K = 1 + (t % 64);                       // 1..64 distinct slots: heavy to light sharing
    for (int l = 0; l < 64; l++) slots[t * 64 + l] = rand() % K;
  }
  uint32_t *dS, *dA, *dC, *dD;
  uint64_t* dB;
  hipMalloc(&dS, slots.size() * 4);
  hipMalloc(&dA, slots.size() * 4);
  hipMalloc(&dC, slots.size() * 4);
  hipMalloc(&dD, slots.size() * 4);
  hipMalloc(&dB, slots.size() * 8);
  hipMemcpy(dS, slots.data(), slots.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dS, trials, dA, dB, dC, dD);
  std::vector<uint32_t> A(slots.size()), C(slots.size()), D(slots.size());
  std::vector<uint64_t> B(slots.size());
  hipMemcpy(A.data(), dA, A.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(B.data(), dB, B.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  long bad[4] = {0, 0, 0, 0}, badrev[4] = {0, 0, 0, 0};
  for (uint32_t t = 0; t < trials; t++) {
    for (int l = 0; l < 64; l++) {
      const uint32_t s = slots[t * 64 + l];
      int hi = -1, lo = -1;
      uint64_t lower = 0, upper = 0;
      uint32_t mx = 0, mxr = 0;
      for (int j = 0; j < 64; j++) {
        if (slots[t * 64 + j] != s) continue;
        if (lo < 0) lo = j;
        hi = j;
        if (j < l) { lower |= 1ull << j; mx = j + 1; }
        if (j > l) { upper |= 1ull << j; if (!mxr || (uint32_t)j + 1 > mxr) mxr = j + 1; }
      }
      const uint32_t i = t * 64 + l;
      bad[0] += A[i] != (uint32_t)hi;  badrev[0] += A[i] != (uint32_t)lo;
      bad[1] += B[i] != lower;         badrev[1] += B[i] != upper;
      bad[2] += C[i] != (uint32_t)hi;  badrev[2] += C[i] != (uint32_t)lo;
      bad[3] += D[i] != mx;            badrev[3] += D[i] != mxr;
    }
  }
  printf("lanes checked: %u\n", trials * 64);
  printf("A ds_write_b8 same addr   : highest-lane-wins mismatches %ld, lowest-lane-wins mismatches %ld\n", bad[0], badrev[0]);
  printf("B ds_or_rtn_b64           : ascending-order mismatches %ld, descending %ld\n", bad[1], badrev[1]);
  printf("C ds_mskor_b32            : highest-lane-wins mismatches %ld, lowest %ld\n", bad[2], badrev[2]);
  printf("D ds_max_rtn_u32          : ascending-order mismatches %ld, descending %ld\n", bad[3], badrev[3]);
  return 0;
}
