// kingdb_amd/csrc/selftest.hip -- run-time guard for the one hardware
// behaviour the compressor's byte identity rests on (lz4_compress.hip,
// Table12/Table16/Table32::xchg): the lanes of ONE ds_mskor_rtn_b32 that hit
// the same LDS dword are applied in ascending lane order, and each lane gets
// the dword as the lower lanes left it.  That was measured once
// (tools/probe/lds_order.hip); HIP promises nothing about it, so every device
// the library compresses on runs this test first (kdb_lz4_set_device, and the
// first launch_compress on a device).  A device that fails it gets
// hipErrorNotSupported from launch_compress (KDB_LZ4_EUNSUPPORTED at the C ABI):
// never a frame that differs from the reference's.
//
// Each trial draws, per lane, a dword among K (1..8: heavy to light sharing),
// a field width (the table planes' 4, 8, 16 and 32 bits), a field and an
// on/off flag (an off lane passes mask 0 and data 0 and still reads, like the
// exchange's lanes past the chunk).  Every lane replays the lower lanes'
// updates of its dword through cross-lane reads and compares what it got; the
// dwords' final values are compared too.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace kdb_lz4 {

namespace {

constexpr uint32_t kTrials = 256, kBlocks = 512;

__device__ __forceinline__ uint32_t xs32(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

__global__ void __launch_bounds__(64) lds_order_selftest_kernel(uint32_t* bad, uint32_t force_fail) {
  __shared__ uint32_t words[8];
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  const uint32_t lane = threadIdx.x;
  uint32_t errs = 0;
  for (uint32_t t = 0; t < kTrials; ++t) {
    uint32_t r = xs32(0x9e3779b9u ^ (blockIdx.x * 0x85ebca6bu) ^ (t * 0xc2b2ae35u) ^ ((lane + 1u) * 0x27d4eb2fu));
    r = xs32(r);
    const uint32_t k = 1u + (t & 7u);
    const uint32_t wsel = (t >> 3) & 3u;                  // 8, 4, 16, 32-bit fields: the planes' widths
    const uint32_t width = wsel == 0 ? 8u : wsel == 1 ? 4u : wsel == 2 ? 16u : 32u;
    const uint32_t d = r % k;
    const uint32_t sh = ((r >> 8) % (32u / width)) * width;
    const uint32_t field = width == 32u ? 0xffffffffu : ((1u << width) - 1u) << sh;
    const bool on = ((r >> 16) & 7u) != 0u;
    const uint32_t m = on ? field : 0u;
    const uint32_t v = (on ? (xs32(r) << sh) & field : 0u);
    if (lane < 8u) words[lane] = xs32(r ^ 0x5bd1e995u);   // a random initial dword each
    __syncthreads();
    const uint32_t init = words[d];
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)(lds_u32*)&words[d];
    uint32_t got;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=&v"(got) : "v"(a), "v"(m), "v"(v)
                 : "memory");
    __syncthreads();
    // replay: the lower lanes of the same dword, in ascending order, then the rest
    uint32_t want = init, fin = init;
    for (uint32_t j = 0; j < 64u; ++j) {
      const uint32_t dj = __shfl(d, (int)j), mj = __shfl(m, (int)j), vj = __shfl(v, (int)j);
      if (dj == d) {
        if (j < lane) want = (want & ~mj) | vj;
        fin = (fin & ~mj) | vj;
      }
    }
    errs += (got != want ? 1u : 0u) + (words[d] != fin ? 1u : 0u);
    __syncthreads();
  }
  if (force_fail && blockIdx.x == 0 && lane == 0) errs += 1u;
  if (errs) atomicAdd(bad, errs);
}

struct DevState {
  int state = 0;   // 0 not run, 1 passed, -1 failed
  uint32_t bad = 0;
};
std::mutex g_mu;
std::unordered_map<int, DevState> g_state;

}  // namespace

// Runs the test on the current device once; later calls return the cached
// verdict.  hipSuccess if the lane order holds, hipErrorNotSupported if not,
// or the HIP error that kept the test from running (then it runs again next time).
hipError_t lane_order_check() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> l(g_mu);
  DevState& s = g_state[dev];
  if (s.state) return s.state > 0 ? hipSuccess : hipErrorNotSupported;
  const char* ff = getenv("KDB_LZ4_SELFTEST_FORCE_FAIL");   // test knob: the failure path
  const uint32_t force = ff && *ff && *ff != '0' ? 1u : 0u;
  hipStream_t st = nullptr;
  uint32_t* dbad = nullptr;
  uint32_t bad = 0;
  if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) == hipSuccess &&
      (e = hipMalloc(&dbad, sizeof(uint32_t))) == hipSuccess &&
      (e = hipMemsetAsync(dbad, 0, sizeof(uint32_t), st)) == hipSuccess) {
    hipLaunchKernelGGL(lds_order_selftest_kernel, dim3(kBlocks), dim3(64), 0, st, dbad, force);
    if ((e = hipGetLastError()) == hipSuccess &&
        (e = hipMemcpyAsync(&bad, dbad, sizeof(uint32_t), hipMemcpyDeviceToHost, st)) == hipSuccess)
      e = hipStreamSynchronize(st);
  }
  if (dbad) (void)hipFree(dbad);
  if (st) (void)hipStreamDestroy(st);
  if (e != hipSuccess) return e;
  s.bad = bad;
  s.state = bad == 0 ? 1 : -1;
  return bad == 0 ? hipSuccess : hipErrorNotSupported;
}

// verdict for `dev` without running anything: 0 not run, 1 passed, -1 failed
int lane_order_state(int dev, uint32_t* bad) {
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_state.find(dev);
  if (it == g_state.end()) return 0;
  if (bad) *bad = it->second.bad;
  return it->second.state;
}

}  // namespace kdb_lz4
