// Workgroups of one wave resident per CU for a given LDS size, measured: each
// workgroup holds its LDS for ~200 us, so a grid of W workgroups takes one
// 200 us round per ceil(W / resident) -- the answer the hardware gives, which
// hipOccupancyMaxActiveBlocksPerMultiprocessor only predicts.
//   lds_occupancy <lds bytes> <workgroups>...
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(64) void hold(uint32_t* sink, uint64_t ticks) {
  extern __shared__ uint32_t lds[];
  lds[threadIdx.x] = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (lds[threadIdx.x] == 12345u) sink[0] = 1u;   // keeps the LDS live
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s <lds bytes> <workgroups>...\n", argv[0]); return 2; }
  const size_t lds = strtoul(argv[1], nullptr, 0);
  int rate = 0;
  if (hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0) != hipSuccess || rate <= 0) rate = 100000;
  const uint64_t ticks = (uint64_t)rate / 5u;   // 200 us (rate in kHz)
  uint32_t* sink = nullptr;
  if (hipMalloc(&sink, 4) != hipSuccess) return 1;
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hold, 64, lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 2; i < argc; ++i) {
    const unsigned w = (unsigned)strtoul(argv[i], nullptr, 0);
    float best = 1e9f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(hold, dim3(w), dim3(64), lds, 0, sink, ticks);
      (void)hipEventRecord(b, 0);
      if (hipEventSynchronize(b) != hipSuccess) return 1;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("lds=%zu predicted_per_cu=%d workgroups=%u ms=%.3f rounds=%.2f\n", lds, per_cu, w, best, best / 0.2f);
  }
  return 0;
}
