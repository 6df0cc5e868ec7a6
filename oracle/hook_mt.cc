// oracle/hook_mt.cc -- TEST INFRASTRUCTURE ONLY (built by `make -C oracle` into
// oracle/_ref/<build>/hook_mt against the reference's own objects, compiled in
// place; nothing of the reference is copied here).
//
// Several client threads write through KingDB's Database::PutPart at once --
// single-part values of every size class, 64 KiB network-style parts,
// ragged parts, values over 1 MiB that Database::PutPart splits itself
// (interface/database.cc:98-124), incompressible stretches that fire the
// disable rule -- then the database is closed, reopened and read back by as
// many threads: Database::Get (values up to the multipart threshold),
// MultipartReader for every key, and one full iteration with GetValue.
// Every value must come back byte for byte.  The flush hook's per-thread
// state (kingdb_amd/csrc/flush_hook.cc) and the read hooks see concurrent
// callers here; tests/test_sanitizers.py runs it under ThreadSanitizer and
// AddressSanitizer, tests/test_kingdb_dropin.py on the GPU.
//
//   hook_mt <dbdir> <threads> <values per thread> [seed]
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "interface/database.h"
#include "util/byte_array.h"
#include "util/status.h"

namespace {

uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

std::string key_of(int t, int i) {
  char b[32];
  snprintf(b, sizeof(b), "t%02d-%08d", t, i);
  return b;
}

// value i of thread t: its size class, then compressible text (runs of a
// small alphabet) with, for some values, an incompressible tail
std::string value_of(uint64_t seed, int t, int i) {
  uint64_t r = mix(seed ^ ((uint64_t)t << 40) ^ (uint64_t)i);
  size_t n;
  switch (r % 10) {
    case 0: n = 0; break;
    case 1: case 2: case 3: n = 1 + (r >> 8) % 400; break;
    case 4: case 5: n = 2000 + (r >> 8) % 6000; break;
    case 6: case 7: n = 60000 + (r >> 8) % 200000; break;
    case 8: n = 1000000 + (r >> 8) % 1200000; break;
    default: n = 100; break;
  }
  std::string v(n, '\0');
  uint64_t s = r;
  for (size_t j = 0; j < n;) {
    s = mix(s + 1);
    const size_t run = 1 + s % 30;
    const char c = (char)('a' + (s >> 8) % 12);
    for (size_t k = 0; k < run && j < n; k++, j++) v[j] = c;
  }
  if (n && (r >> 20) % 4 == 0) {
    for (size_t j = (r >> 24) % n; j < n; j++) {
      s = mix(s + j);
      v[j] = (char)s;
    }
  }
  return v;
}

// how value i is sent: one Put, 64 KiB parts, or ragged parts
std::vector<size_t> parts_of(uint64_t seed, int t, int i, size_t n) {
  const uint64_t r = mix(seed * 7 + ((uint64_t)t << 32) + (uint64_t)i);
  std::vector<size_t> p;
  if (n == 0 || r % 3 == 0) return {n};
  if (r % 3 == 1) {
    for (size_t o = 0; o < n; o += 65536) p.push_back(n - o < 65536 ? n - o : 65536);
    return p;
  }
  size_t o = 0;
  uint64_t s = r;
  while (o < n) {
    s = mix(s + 3);
    size_t c = 1 + s % 150000;
    if (c > n - o) c = n - o;
    p.push_back(c);
    o += c;
  }
  return p;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: hook_mt <dbdir> <threads> <values per thread> [seed]\n");
    return 2;
  }
  kdb::Logger::set_current_level("emerg");
  const int T = atoi(argv[2]), N = atoi(argv[3]);
  const uint64_t seed = argc > 4 ? strtoull(argv[4], nullptr, 0) : 1;
  kdb::DatabaseOptions options;
  options.compression = kdb::kLZ4Compression;
  std::atomic<int> errors{0};
  {
    kdb::Database db(options, argv[1]);
    if (!db.Open().IsOK()) return 1;
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        kdb::WriteOptions wo;
        for (int i = 0; i < N; i++) {
          const std::string k = key_of(t, i), v = value_of(seed, t, i);
          uint64_t off = 0;
          for (size_t c : parts_of(seed, t, i, v.size())) {
            kdb::ByteArray kb = kdb::NewDeepCopyByteArray(k.data(), k.size());
            kdb::ByteArray vb = kdb::NewDeepCopyByteArray(v.data() + off, c);
            kdb::Status s = db.PutPart(wo, kb, vb, off, v.size());
            if (!s.IsOK()) {
              if (errors++ < 5) fprintf(stderr, "put %s: %s\n", k.c_str(), s.ToString().c_str());
              break;
            }
            off += c;
          }
        }
      });
    for (auto& x : th) x.join();
    db.Close();
  }
  uint64_t reads = 0;
  {
    kdb::Database db(options, argv[1]);
    if (!db.Open().IsOK()) return 1;
    kdb::ReadOptions ro;
    std::atomic<uint64_t> nread{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        kdb::ReadOptions r2;
        for (int i = 0; i < N; i++) {
          const std::string k = key_of(t, i), v = value_of(seed, t, i);
          if (v.size() <= 1024 * 1024) {
            std::string out;
            kdb::Status s = db.Get(r2, k, &out);
            if (!s.IsOK() || out != v) {
              if (errors++ < 5) {
                size_t at = 0;
                while (at < out.size() && at < v.size() && out[at] == v[at]) at++;
                size_t bad = 0;
                for (size_t j = 0; j < out.size() && j < v.size(); j++) bad += out[j] != v[j];
                fprintf(stderr, "get %s: %s size %zu got %zu, first diff at %zu (%zu bytes differ)\n", k.c_str(),
                        s.ToString().c_str(), v.size(), out.size(), at, bad);
              }
            }
          }
          kdb::MultipartReader mp = db.NewMultipartReader(r2, k);
          std::string out;
          for (mp.Begin(); mp.IsValid(); mp.Next()) {
            kdb::ByteArray part;
            mp.GetPart(&part);
            out += part.ToString();
          }
          if (!mp.GetStatus().IsOK() || out != v) {
            if (errors++ < 5) fprintf(stderr, "multipart %s: %s\n", k.c_str(), mp.GetStatus().ToString().c_str());
          }
          nread++;
        }
      });
    // one iteration over everything, beside the readers
    std::map<std::string, std::string> seen;
    {
      kdb::Iterator it = db.NewIterator(ro);
      for (it.Begin(); it.IsValid(); it.Next()) {
        kdb::ByteArray k = it.GetKey();
        kdb::ByteArray v = it.GetValue();
        if (it.GetStatus().IsMultipartRequired()) continue;
        seen[k.ToString()] = v.ToString();
      }
    }
    for (auto& x : th) x.join();
    for (auto& p : seen) {
      int t = 0, i = 0;
      if (sscanf(p.first.c_str(), "t%d-%d", &t, &i) != 2 || p.second != value_of(seed, t, i)) {
        if (errors++ < 5) fprintf(stderr, "iterator %s: wrong value\n", p.first.c_str());
      }
    }
    reads = nread.load();
    db.Close();
  }
  if (errors) {
    fprintf(stderr, "%d errors\n", errors.load());
    return 1;
  }
  printf("ok: %d threads x %d values written and read back (%llu reads)\n", T, N, (unsigned long long)reads);
  return 0;
}
