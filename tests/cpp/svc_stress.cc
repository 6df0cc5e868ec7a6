// tests/cpp/svc_stress.cc -- TEST INFRASTRUCTURE: many host threads calling the
// per-call decode and compress entry points (the resident services,
// kingdb_amd/csrc/service.h) at once, on values shaped like oracle/hook_mt.cc's
// (runs of a small alphabet, some with incompressible tails, 1 B - 8 KiB).
// Blocks come from the oracle (oracle/liblz4_oracle.so, pinned to the
// reference); every decoded value and every compressed block is checked, and
// the first mismatches are described (thread, slot size, first differing byte).
//
// With `busy` set, a background thread keeps batch compressions running on
// the device meanwhile (other kernels' dirty lines in L2), and the callers
// pause now and then past the services' idle time (waves leave and are
// relaunched): the conditions under which a done word once overtook the result
// bytes (tests/test_service_isa.py).
//
//   svc_stress <threads> <calls per thread> [seed [busy]]      exit 0: all equal
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kdb_lz4.h"

typedef int (*orc_compress_fn)(const uint8_t*, uint8_t*, int, int);
typedef int (*orc_bound_fn)(int);

static std::string value_of(std::mt19937_64& r) {
  size_t n;
  switch (r() % 4) {
    case 0: n = 1 + r() % 400; break;
    case 1: n = 2000 + r() % 6193; break;
    case 2: n = 100; break;
    default: n = 4000 + r() % 4000; break;
  }
  std::string v(n, '\0');
  for (size_t j = 0; j < n;) {
    const size_t run = 1 + r() % 30;
    const char c = (char)('a' + r() % 12);
    for (size_t k = 0; k < run && j < n; k++, j++) v[j] = c;
  }
  if (r() % 4 == 0)
    for (size_t j = r() % n; j < n; j++) v[j] = (char)r();
  return v;
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 8, N = argc > 2 ? atoi(argv[2]) : 500;
  const uint64_t seed = argc > 3 ? strtoull(argv[3], nullptr, 0) : 1;
  const bool busy = argc > 4 && atoi(argv[4]) != 0;
  void* h = dlopen(getenv("KDB_ORACLE_SO") ? getenv("KDB_ORACLE_SO") : "oracle/liblz4_oracle.so", RTLD_NOW);
  if (!h) {
    fprintf(stderr, "oracle: %s\n", dlerror());
    return 2;
  }
  auto ocomp = (orc_compress_fn)dlsym(h, "orc_compress_limited");
  auto obound = (orc_bound_fn)dlsym(h, "orc_compress_bound");
  if (!ocomp || !obound || kdb_lz4_set_device(0) != KDB_LZ4_OK) return 2;
  // the values and their reference blocks, made up front
  std::mt19937_64 r(seed);
  std::vector<std::string> vals(256), blocks(256);
  for (size_t i = 0; i < vals.size(); i++) {
    vals[i] = value_of(r);
    std::string b((size_t)obound((int)vals[i].size()), '\0');
    const int c = ocomp((const uint8_t*)vals[i].data(), (uint8_t*)&b[0], (int)vals[i].size(), (int)b.size());
    b.resize((size_t)c);
    blocks[i] = b;
  }
  std::atomic<int> bad{0};
  std::atomic<bool> stop{false};
  std::thread bg;
  if (busy)
    bg = std::thread([&] {
      // 16 Mi of G1 data in 4 KiB values, compressed over and over on the device
      kdb_lz4_set_device(0);
      const uint32_t n = 4096, len = 4096;
      void *src = nullptr, *dst = nullptr, *meta = nullptr, *st = nullptr;
      if (kdb_lz4_malloc(&src, (uint64_t)n * len) || kdb_lz4_malloc(&dst, (uint64_t)n * 4200) ||
          kdb_lz4_malloc(&meta, (uint64_t)n * 32) || kdb_lz4_stream_create(&st)) {
        bad++;
        return;
      }
      std::vector<uint64_t> so(n), doff(n);
      std::vector<uint32_t> sl(n, len), cap(n, 4200);
      for (uint32_t i = 0; i < n; i++) so[i] = (uint64_t)i * len, doff[i] = (uint64_t)i * 4200;
      uint8_t* m = static_cast<uint8_t*>(meta);
      kdb_lz4_gen_g1(static_cast<uint8_t*>(src), 0, (uint64_t)n * len / 100, 301, st);
      kdb_lz4_memcpy_h2d(m, so.data(), 8ull * n, st);
      kdb_lz4_memcpy_h2d(m + 8ull * n, doff.data(), 8ull * n, st);
      kdb_lz4_memcpy_h2d(m + 16ull * n, sl.data(), 4ull * n, st);
      kdb_lz4_memcpy_h2d(m + 20ull * n, cap.data(), 4ull * n, st);
      while (!stop.load()) {
        if (kdb_lz4_compress_blocks_batch(st, static_cast<uint8_t*>(src), (uint64_t*)m, (uint32_t*)(m + 16ull * n), n,
                                          len, static_cast<uint8_t*>(dst), (uint64_t*)(m + 8ull * n),
                                          (uint32_t*)(m + 20ull * n), (int32_t*)(m + 24ull * n)) ||
            kdb_lz4_stream_sync(st)) {
          bad++;
          break;
        }
      }
      kdb_lz4_stream_destroy(st);
      kdb_lz4_free(src);
      kdb_lz4_free(dst);
      kdb_lz4_free(meta);
    });
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      kdb_lz4_set_device(0);
      std::mt19937_64 rr(seed * 131 + t);
      std::string out(9000, '\0');
      for (int i = 0; i < N; i++) {
        if (busy && rr() % 16 == 0) std::this_thread::sleep_for(std::chrono::microseconds(2500));   // past the idle time
        const size_t k = rr() % vals.size();
        const std::string& v = vals[k];
        const std::string& b = blocks[k];
        const int d = kdb_lz4_decompress_safe_partial(b.data(), &out[0], (int)b.size(), (int)v.size(), (int)v.size());
        if (d != (int)v.size() || memcmp(out.data(), v.data(), v.size()) != 0) {
          if (bad++ < 10) {
            size_t at = 0;
            while (d > 0 && at < v.size() && out[at] == v[at]) at++;
            fprintf(stderr, "decode t%d call %d value %zu: size %zu block %zu -> ret %d, first diff at %zu\n", t, i,
                    k, v.size(), b.size(), d, at);
          }
        }
        if (rr() % 4 == 0) {
          std::string c((size_t)obound((int)v.size()), '\0');
          const int n = kdb_lz4_compress_limitedOutput(v.data(), &c[0], (int)v.size(), (int)c.size());
          if (n != (int)b.size() || memcmp(c.data(), b.data(), b.size()) != 0) {
            if (bad++ < 10)
              fprintf(stderr, "compress t%d call %d value %zu: size %zu -> %d, reference %zu\n", t, i, k, v.size(), n,
                      b.size());
          }
        }
      }
    });
  for (auto& x : th) x.join();
  stop = true;
  if (bg.joinable()) bg.join();
  if (bad) {
    fprintf(stderr, "%d mismatches\n", bad.load());
    return 1;
  }
  printf("ok: %d threads x %d calls\n", T, N);
  return 0;
}
