// tools/probe/bar_probe.hip -- where should a resident service's mailbox live?
//
// Ping-pong between a host thread and one resident wave, N round trips, in
// three layouts:
//   A  host memory (pinned, coherent, mapped) for both directions -- today's
//      SvcBox: the wave polls host memory across PCIe;
//   B  the doorbell in device memory the host writes through the large BAR
//      (hipExtMallocWithFlags(hipDeviceMallocUncached)), the answer in host
//      memory: the wave polls its own HBM;
//   C  as B with fine-grained device memory (hipDeviceMallocFinegrained).
// The wave answers each ring (value v) by storing v to host memory with a
// system-scope store; the host spins on it.  Prints the median and p99 round
// trip in microseconds.  Every wave exits: after N rounds or 2 s of wall clock.
//
//   bar_probe [rounds]
#include <hip/hip_runtime.h>

#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void pong(const uint32_t* ring, uint32_t* answer, uint32_t rounds, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  uint32_t seen = 0;
  while (seen < rounds) {
    const uint32_t v = __hip_atomic_load(ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != seen) {
      seen = v;
      __hip_atomic_store(answer, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (wall_clock64() - t0 > max_ticks) {
      break;
    }
  }
}

// D/E: each ring carries `bytes` of input the wave must see whole: the host
// writes dword j of round i as i * 0x9E3779B1 + j, then the doorbell; the wave
// reads it all (16 B per lane) and answers i, or i | 0x80000000 on a mismatch.
__global__ void pong_data(const uint32_t* ring, const uint4* data, uint32_t bytes, uint32_t* answer, uint32_t rounds,
                          uint64_t max_ticks) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  uint32_t seen = 0;
  const uint32_t chunks = bytes / 16u;
  while (seen < rounds) {
    const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    if (v != seen) {
      seen = v;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      bool bad = false;
      for (uint32_t c = lane; c < chunks; c += 64u) {
        const uint4 x = data[c];
        const uint32_t b = v * 0x9E3779B1u + 4u * c;
        bad |= x.x != b || x.y != b + 1u || x.z != b + 2u || x.w != b + 3u;
      }
      const bool any = __builtin_amdgcn_ballot_w64(bad) != 0;
      if (lane == 0) __hip_atomic_store(answer, any ? (v | 0x80000000u) : v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (wall_clock64() - t0 > max_ticks) {
      break;
    }
  }
}

static void run_data(const char* name, uint32_t* ring_host_view, const uint32_t* ring_dev, uint32_t* data_host_view,
                     const uint32_t* data_dev, uint32_t bytes, uint32_t* ans_host, uint32_t* ans_dev, uint32_t rounds,
                     uint64_t max_ticks) {
  __atomic_store_n(ring_host_view, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(ans_host, 0u, __ATOMIC_SEQ_CST);
  __builtin_ia32_sfence();
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return;
  hipLaunchKernelGGL(pong_data, dim3(1), dim3(64), 0, st, ring_dev, (const uint4*)data_dev, bytes, ans_dev, rounds,
                     max_ticks);
  std::vector<double> us;
  us.reserve(rounds);
  bool lost = false;
  uint32_t bad = 0;
  std::vector<uint32_t> buf(bytes / 4u);
  for (uint32_t i = 1; i <= rounds && !lost; i++) {
    for (uint32_t j = 0; j < bytes / 4u; j++) buf[j] = i * 0x9E3779B1u + j;
    const auto a = std::chrono::steady_clock::now();
    memcpy(data_host_view, buf.data(), bytes);
    __builtin_ia32_sfence();
    __atomic_store_n(ring_host_view, i, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    uint32_t got;
    while (((got = __atomic_load_n(ans_host, __ATOMIC_ACQUIRE)) & 0x7fffffffu) != i) {
      if (std::chrono::steady_clock::now() - a > std::chrono::milliseconds(500)) {
        lost = true;
        break;
      }
    }
    bad += (got & 0x80000000u) != 0;
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
  }
  hipStreamSynchronize(st);
  hipStreamDestroy(st);
  if (lost) {
    printf("%s: no answer within 500 ms after %zu rounds\n", name, us.size());
    return;
  }
  std::sort(us.begin() + 10, us.end());
  const size_t n = us.size() - 10;
  printf("%s: %u B, %u rounds, round trip median %.2f us, p10 %.2f, p99 %.2f, %u torn\n", name, bytes, rounds,
         us[10 + n / 2], us[10 + n / 10], us[10 + n * 99 / 100], bad);
}

static void run(const char* name, uint32_t* ring_host_view, const uint32_t* ring_dev, uint32_t* ans_host,
                uint32_t* ans_dev, uint32_t rounds, uint64_t max_ticks) {
  __atomic_store_n(ring_host_view, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(ans_host, 0u, __ATOMIC_SEQ_CST);
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return;
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, st, ring_dev, ans_dev, rounds, max_ticks);
  std::vector<double> us;
  us.reserve(rounds);
  bool lost = false;
  for (uint32_t i = 1; i <= rounds && !lost; i++) {
    const auto a = std::chrono::steady_clock::now();
    __atomic_store_n(ring_host_view, i, __ATOMIC_RELEASE);
    // a BAR mapping is write-combining: the store leaves the core's WC buffer
    // at a fence (harmless for host memory)
    __builtin_ia32_sfence();
    while (__atomic_load_n(ans_host, __ATOMIC_ACQUIRE) != i) {
      if (std::chrono::steady_clock::now() - a > std::chrono::milliseconds(500)) {
        lost = true;
        break;
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
  }
  hipStreamSynchronize(st);
  hipStreamDestroy(st);
  if (lost) {
    printf("%s: no answer within 500 ms after %zu rounds\n", name, us.size());
    return;
  }
  std::sort(us.begin() + 10, us.end());   // the first rounds include the launch
  const size_t n = us.size() - 10;
  printf("%s: %u rounds, round trip median %.2f us, p10 %.2f, p99 %.2f\n", name, rounds, us[10 + n / 2],
         us[10 + n / 10], us[10 + n * 99 / 100]);
}

// a host access to a device pointer the CPU cannot reach faults: caught here
static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }
static bool host_can_write(uint32_t* p) {
  struct sigaction sa {}, old{};
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  bool ok = false;
  if (sigsetjmp(g_jb, 1) == 0) {
    __atomic_store_n(p, 0x12345678u, __ATOMIC_SEQ_CST);
    ok = __atomic_load_n(p, __ATOMIC_SEQ_CST) == 0x12345678u;
  }
  sigaction(SIGSEGV, &old, nullptr);
  sigaction(SIGBUS, &old, nullptr);
  return ok;
}

int main(int argc, char** argv) {
  const uint32_t rounds = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000;
  int large_bar = 0, rate_khz = 0;
  hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0);
  hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  printf("large BAR: %d, wall clock %d kHz\n", large_bar, rate_khz);
  const uint64_t max_ticks = 2000ull * (uint64_t)rate_khz;   // 2 s
  uint32_t* h = nullptr;
  if (hipHostMalloc((void**)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
  uint32_t* hd = nullptr;
  hipHostGetDevicePointer((void**)&hd, h, 0);
  run("A host ring, host answer", h, hd, h + 32, hd + 32, rounds, max_ticks);
  if (!large_bar) {
    printf("B/C skipped: no large BAR\n");
    return 0;
  }
  const unsigned flags[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
  const char* names[2] = {"B device ring (uncached), host answer", "C device ring (fine-grained), host answer"};
  for (int k = 0; k < 2; k++) {
    uint32_t* d = nullptr;
    if (hipExtMallocWithFlags((void**)&d, 4096, flags[k]) != hipSuccess) {
      printf("%s: allocation failed\n", names[k]);
      continue;
    }
    hipPointerAttribute_t at{};
    hipPointerGetAttributes(&at, d);
    uint32_t* hv = at.hostPointer ? (uint32_t*)at.hostPointer : d;   // large BAR: the same address
    const bool ok = host_can_write(hv);
    printf("%s: host pointer %p, device %p, host writes %s\n", names[k], at.hostPointer, (void*)d,
           ok ? "work" : "fault");
    if (ok) run(names[k], hv, d, h + 64, hd + 64, rounds, max_ticks);
    hipFree(d);
  }
  // D / E: 2 400 bytes of input with each ring, in host memory (E: as today's
  // slot.in) or fine-grained device memory written through the BAR (D)
  uint32_t* hin = nullptr;
  if (hipHostMalloc((void**)&hin, 65536, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
  uint32_t* hind = nullptr;
  hipHostGetDevicePointer((void**)&hind, hin, 0);
  for (uint32_t bytes : {112u, 2400u, 8192u}) {
    run_data("E host ring + host input", h, hd, hin, hind, bytes, h + 96, hd + 96, rounds / 4, max_ticks);
    uint32_t* d = nullptr;
    if (hipExtMallocWithFlags((void**)&d, 65536, hipDeviceMallocFinegrained) != hipSuccess) continue;
    if (host_can_write(d))
      run_data("D device ring + device input", d, d, d + 64, d + 64, bytes, h + 96, hd + 96, rounds / 4, max_ticks);
    hipFree(d);
  }
  return 0;
}
