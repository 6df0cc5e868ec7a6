// tests/cpp/bench_compressor.cc -- per-call latency of kdb::CompressorLZ4, the
// way KingDB calls it: one Compress per put (interface/database.cc:185-189),
// one Uncompress per frame (interface/multipart.h:98-103), new[] buffers owned
// by the caller.  Written against the class API only, so oracle/Makefile
// `kingdb` builds it twice from the same source: against the reference codec
// (_ref/kingdb_ref/bench_compressor) and against the drop-in
// (_ref/kingdb_dropin/bench_compressor, every LZ4 block on the GPU).
//
//   bench_compressor <value_bytes> <calls>
// prints one JSON line: microseconds per Compress / Uncompress call (median of
// 5 passes over <calls> values, after one warm-up pass).
#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "algorithm/compressor.h"

// G1: LevelDB Random(301) + CompressibleString(0.5) pieces of 100 bytes
// (doc/bench/db_bench_kingdb.cc:113-142), the BASELINE data.
struct Rnd {
  uint32_t s;
  explicit Rnd(uint32_t x) : s(x & 0x7fffffffu) {
    if (s == 0 || s == 2147483647u) s = 1;
  }
  uint32_t next() {
    const uint64_t p = (uint64_t)s * 16807u;
    s = (uint32_t)((p >> 31) + (p & 2147483647u));
    if (s > 2147483647u) s -= 2147483647u;
    return s;
  }
};

static std::string g1_pool(size_t bytes) {
  Rnd r(301);
  std::string pool;
  while (pool.size() < bytes) {
    std::string raw;
    for (int i = 0; i < 50; i++) raw += (char)(' ' + r.next() % 95);
    std::string piece;
    while (piece.size() < 100) piece += raw;
    pool += piece.substr(0, 100);
  }
  return pool;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const uint64_t size = argc > 1 ? strtoull(argv[1], nullptr, 0) : 100;
  const int calls = argc > 2 ? atoi(argv[2]) : 2000;
  // KDB_BENCH_NOVERIFY=1: timing-only library builds (attribution variants
  // whose output is wrong by design) skip the byte check
  const bool verify = !getenv("KDB_BENCH_NOVERIFY");
  const std::string pool = g1_pool(size * (uint64_t)calls + 1);
  kdb::CompressorLZ4 lz4;
  std::vector<char*> frames(calls, nullptr);
  std::vector<uint64_t> flen(calls, 0);
  std::vector<double> tc, td;
  uint64_t bytes_out = 0;
  for (int pass = 0; pass < 6; pass++) {
    double t0 = now_us();
    for (int i = 0; i < calls; i++) {
      delete[] frames[i];
      kdb::Status s = lz4.Compress(const_cast<char*>(pool.data()) + size * i, size, &frames[i], &flen[i]);
      if (!s.IsOK()) {
        fprintf(stderr, "Compress failed: %s\n", s.ToString().c_str());
        return 1;
      }
    }
    double t1 = now_us();
    bytes_out = 0;
    for (int i = 0; i < calls; i++) {
      lz4.ResetThreadLocalStorage();
      char *out = nullptr, *frame = nullptr;
      uint64_t n = 0, fn = 0;
      kdb::Status s = lz4.Uncompress(frames[i], flen[i], &out, &n, &frame, &fn);
      if (!s.IsOK() || (verify && (n != size || memcmp(out, pool.data() + size * i, size) != 0))) {
        fprintf(stderr, "Uncompress failed or differs at %d\n", i);
        return 1;
      }
      bytes_out += flen[i];
      delete[] out;
    }
    double t2 = now_us();
    if (pass) {
      tc.push_back((t1 - t0) / calls);
      td.push_back((t2 - t1) / calls);
    }
  }
  for (char* f : frames) delete[] f;
  std::sort(tc.begin(), tc.end());
  std::sort(td.begin(), td.end());
  printf("{\"value_bytes\": %" PRIu64 ", \"calls\": %d, \"compress_us\": %.3f, \"uncompress_us\": %.3f, "
         "\"frame_bytes\": %" PRIu64 "}\n",
         size, calls, tc[tc.size() / 2], td[td.size() / 2], bytes_out);
  return 0;
}
