// tests/cpp/test_hstable_tsan.cc -- the host-side HSTable writer
// (kingdb_amd/csrc/hstable.cc) under ThreadSanitizer: a CPU-only build
// (tests/cpp/Makefile `tsan`, g++ -fsanitize=thread) of the writer's parallel
// paths -- append_fast's multi-threaded copies and the worker pool that
// encodes and checksums large offset arrays -- driven from several host
// threads at once, one writer each.
//
// Checks: no data race reported (TSan exits 66 on a report), and every
// writer's files are identical to a writer fed the same entries one at a time
// (the serial append_loop path), which in turn must be deterministic.
//
//   test_hstable_tsan [threads [entries]]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kdb_put.h"

namespace {

struct Batch {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off, hashed;
  std::vector<uint32_t> len, kind;
  std::vector<int32_t> status;
};

Batch make_batch(uint32_t n) {
  Batch b;
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto rnd = [&x] {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  uint64_t o = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t l = 40 + (uint32_t)(rnd() % 160);
    b.off.push_back(o);
    b.len.push_back(l);
    b.hashed.push_back(rnd());
    b.kind.push_back(KDB_PUT_SELF_CONTAINED);
    b.status.push_back(0);
    for (uint32_t k = 0; k < l; k++) b.bytes.push_back((uint8_t)rnd());
    o += l;
  }
  return b;
}

typedef std::vector<std::pair<uint32_t, std::string>> Files;

bool files_of(kdb_hstable_writer* w, Files* out) {
  uint32_t c = 0;
  if (kdb_hstable_writer_close(w) || kdb_hstable_writer_file_count(w, &c)) return false;
  for (uint32_t i = 0; i < c; i++) {
    uint32_t id;
    const uint8_t* d;
    uint64_t sz;
    if (kdb_hstable_writer_file(w, i, &id, &d, &sz)) return false;
    out->emplace_back(id, std::string(reinterpret_cast<const char*>(d), sz));
  }
  return true;
}

// step entries per append() call
bool write_all(const Batch& b, uint32_t step, uint64_t hstable_size, Files* out) {
  kdb_hstable_writer* w = nullptr;
  if (kdb_hstable_writer_create(hstable_size, 1, &w)) return false;
  const uint32_t n = (uint32_t)b.len.size();
  bool ok = true;
  for (uint32_t i = 0; i < n && ok; i += step) {
    const uint32_t m = std::min(step, n - i);
    ok = kdb_hstable_writer_append(w, b.bytes.data(), &b.off[i], &b.len[i], &b.hashed[i], &b.kind[i],
                                   &b.status[i], m) == KDB_PUT_OK;
  }
  ok = ok && files_of(w, out);
  kdb_hstable_writer_destroy(w);
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 400000;
  const uint64_t hs = 32ull << 20;   // several files, offset arrays above the pool's 2 MiB threshold
  const Batch b = make_batch(n);

  Files serial, serial2;
  if (!write_all(b, 1, hs, &serial) || !write_all(b, 1, hs, &serial2)) {
    fprintf(stderr, "serial writer failed\n");
    return 1;
  }
  if (serial != serial2) {
    fprintf(stderr, "serial writer not deterministic\n");
    return 1;
  }
  std::vector<Files> got(threads);
  std::vector<int> ok(threads, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] { ok[t] = write_all(b, t % 2 ? n : 65536u, hs, &got[t]); });
  for (auto& x : th) x.join();
  size_t bytes = 0;
  for (auto& f : serial) bytes += f.second.size();
  for (int t = 0; t < threads; t++) {
    if (!ok[t]) {
      fprintf(stderr, "writer %d failed\n", t);
      return 1;
    }
    if (got[t] != serial) {
      fprintf(stderr, "writer %d: files differ from the serial writer\n", t);
      return 1;
    }
  }
  printf("ok: %d writers x %u entries, %zu files, %zu bytes each\n", threads, n, serial.size(), bytes);
  return 0;
}
