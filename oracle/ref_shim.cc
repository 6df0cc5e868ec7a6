// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY (compiled into oracle/_ref/).
//
// A C-ABI wrapper, written for this repo, around the REFERENCE's own codec
// objects (/root/reference/algorithm/{lz4,compressor,crc32c}.cc, compiled in
// place by oracle/Makefile; no reference source is copied here).  It lets
// tests/golden/make_golden.py drive the real reference through ctypes to emit
// golden fixtures and to cross-check oracle/lz4_oracle.c.
//
// Also restates the two std::mt19937 generators of unit-tests/test_db.cc
// (CompressibleDataGenerator 108-131 = G2, IncompressibleDataGenerator 87-105
// = G3).  They depend only on libstdc++'s mt19937/uniform_int_distribution,
// so running them here gives the same bytes the reference test harness sees.
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#include "algorithm/compressor.h"
#include "algorithm/crc32c.h"
#include "algorithm/lz4.h"

extern "C" {

int ref_compress_bound(int n) { return LZ4_compressBound(n); }

int ref_compress_limited(const char* src, char* dst, int n, int max_out) {
  return LZ4_compress_limitedOutput(src, dst, n, max_out);
}

// Decodes a block placed in a zero-padded scratch buffer, so the (at most one)
// byte the reference reads at iend is 0 -- the convention of the oracle and of
// the GPU kernel.  The destination is zero-initialised for the same reason.
int ref_decompress_partial(const char* src, int csize, char* dst, int target, int max_out) {
  size_t n = csize > 0 ? (size_t)csize : 0;
  std::vector<char> in(n + 64, 0);
  if (n) memcpy(in.data(), src, n);
  std::vector<char> out((size_t)(max_out > 0 ? max_out : 0) + 64, 0);
  int ret = LZ4_decompress_safe_partial(in.data(), out.data(), csize, target, max_out);
  if (ret > 0) memcpy(dst, out.data(), (size_t)ret);
  return ret;
}

// CompressorLZ4::Compress: returns the frame length, or -1 on IOError.
int64_t ref_frame_compress(const char* src, uint64_t n, char* frame_out) {
  kdb::CompressorLZ4 c;
  char* frame = nullptr;
  uint64_t fn = 0;
  kdb::Status s = c.Compress(const_cast<char*>(src), n, &frame, &fn);
  if (!s.IsOK()) return -1;
  memcpy(frame_out, frame, fn);
  delete[] frame;
  return (int64_t)fn;
}

// Streams CompressorLZ4::Uncompress over a concatenation of frames the way
// unit-tests/test_compression.cc:100-115 does; returns the number of frames
// decoded (or -1 on IOError) and writes the concatenated output.
int64_t ref_frames_uncompress(const char* frames, uint64_t total, char* out, uint64_t* out_total) {
  kdb::CompressorLZ4 c;
  c.ResetThreadLocalStorage();
  int64_t nframes = 0;
  uint64_t pos = 0;
  for (;;) {
    char* dst = nullptr;
    uint64_t dn = 0;
    char* fr = nullptr;
    uint64_t fn = 0;
    kdb::Status s = c.Uncompress(const_cast<char*>(frames), total, &dst, &dn, &fr, &fn);
    if (s.IsDone()) break;
    if (!s.IsOK()) { delete[] dst; return -1; }
    memcpy(out + pos, dst, dn);
    pos += dn;
    delete[] dst;
    nframes++;
  }
  *out_total = pos;
  return nframes;
}

uint32_t ref_crc32c_extend(uint32_t crc, const char* p, uint64_t n) {
  return kdb::crc32c::Extend(crc, p, n);
}

// Digest of a whole batch of CompressorLZ4::Compress frames (values
// src[off[i] .. +len[i]) in order): *total = sum of frame lengths, *crc =
// crc32c::Extend over the frames concatenated.  Pins byte identity at the
// BASELINE sizes (tests/golden/make_digests.py) without committing GBs.
// Returns -1 on the first IOError, else 0.
int ref_frames_digest(const char* src, const uint64_t* off, const uint32_t* len, uint64_t n, uint64_t* total,
                      uint32_t* crc) {
  kdb::CompressorLZ4 c;
  uint64_t t = 0;
  uint32_t x = 0;
  for (uint64_t i = 0; i < n; i++) {
    char* frame = nullptr;
    uint64_t fn = 0;
    kdb::Status s = c.Compress(const_cast<char*>(src) + off[i], len[i], &frame, &fn);
    if (!s.IsOK()) return -1;
    x = kdb::crc32c::Extend(x, frame, fn);
    t += fn;
    delete[] frame;
  }
  *total = t;
  *crc = x;
  return 0;
}

// G2: test_db.cc:108-131, one generator instance, `count` successive calls.
void ref_gen_g2(char* out, int size, int count) {
  std::seed_seq seq{1, 2, 3, 4, 5, 6, 7};
  std::mt19937 gen(seq);
  std::uniform_int_distribution<int> dist(0, 255);
  for (int v = 0; v < count; v++) {
    char* data = out + (size_t)v * size;
    int i = 0;
    while (i < size) {
      char ch = static_cast<char>(dist(gen));
      int rep = dist(gen) % 30 + 1;
      if (i + rep > size) rep = size - i;
      memset(data + i, ch, rep);
      i += rep;
    }
  }
}

// G3: test_db.cc:87-105.
void ref_gen_g3(char* out, int size, int count) {
  std::seed_seq seq{1, 2, 3, 4, 5, 6, 7};
  std::mt19937 gen(seq);
  std::uniform_int_distribution<int> dist(0, 255);
  for (int64_t i = 0; i < (int64_t)size * count; i++) out[i] = static_cast<char>(dist(gen));
}

}  // extern "C"

// ---- CPU baseline harness (bench.py cpu_baseline leg, kind "reference") ----
// Times the reference's own block codec -- LZ4_compress_limitedOutput with a
// bound-sized slot, then LZ4_decompress_safe_partial(target = max = size) --
// over n values of `size` bytes with `threads` std::threads, each owning a
// contiguous (blocked) range of values.  One untimed warm-up pass, then
// `passes` timed passes; compress and decompress phases are timed separately
// (steady_clock).  Returns 0, or -1 if any value fails to round-trip.
#include <chrono>
#include <thread>
extern "C" int ref_bench_roundtrip(const char* src, int n, int size, int threads, int passes,
                                   double* t_compress, double* t_decompress, uint64_t* comp_bytes) {
  const int bound = LZ4_compressBound(size);
  std::vector<char> blocks((size_t)n * bound);
  std::vector<int> blen(n);
  std::vector<char> out((size_t)n * size);
  int bad = 0;
  auto run = [&](bool comp) {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
      th.emplace_back([&, t]() {
        int lo = (int)((int64_t)n * t / threads), hi = (int)((int64_t)n * (t + 1) / threads);
        for (int i = lo; i < hi; i++) {
          if (comp) {
            blen[i] = LZ4_compress_limitedOutput(src + (size_t)i * size, &blocks[(size_t)i * bound], size, bound);
          } else {
            int r = LZ4_decompress_safe_partial(&blocks[(size_t)i * bound], &out[(size_t)i * size], blen[i], size, size);
            if (r != size) bad = 1;
          }
        }
      });
    }
    for (auto& x : th) x.join();
  };
  run(true);
  run(false);
  double tc = 0, td = 0;
  for (int p = 0; p < passes; p++) {
    auto a = std::chrono::steady_clock::now();
    run(true);
    auto b = std::chrono::steady_clock::now();
    run(false);
    auto c = std::chrono::steady_clock::now();
    tc += std::chrono::duration<double>(b - a).count();
    td += std::chrono::duration<double>(c - b).count();
  }
  uint64_t cb = 0;
  for (int i = 0; i < n; i++) cb += (uint64_t)blen[i];
  *t_compress = tc;
  *t_decompress = td;
  *comp_bytes = cb;
  if (memcmp(out.data(), src, (size_t)n * size) != 0) bad = 1;
  return bad ? -1 : 0;
}

// The same round trip over values of mixed sizes (bench.py --workload mixed):
// value i is src[off[i] .. off[i] + len[i]), every value one LZ4 block as
// CompressorLZ4::Compress makes it (a 64 KiB part is one block); the threads
// take contiguous byte-balanced ranges.
extern "C" int ref_bench_roundtrip_var(const char* src, const uint64_t* off, const uint32_t* len, int n,
                                       int threads, int passes, double* t_compress, double* t_decompress,
                                       uint64_t* comp_bytes) {
  std::vector<uint64_t> boff(n + 1, 0), ooff(n + 1, 0);
  for (int i = 0; i < n; i++) {
    boff[i + 1] = boff[i] + (uint64_t)LZ4_compressBound((int)len[i]);
    ooff[i + 1] = ooff[i] + len[i];
  }
  std::vector<char> blocks(boff[n]);
  std::vector<int> blen(n);
  std::vector<char> out(ooff[n]);
  std::vector<int> cut(threads + 1, n);
  cut[0] = 0;
  for (int t = 1, i = 0; t < threads; t++) {
    const uint64_t want = ooff[n] * (uint64_t)t / (uint64_t)threads;
    while (i < n && ooff[i] < want) i++;
    cut[t] = i;
  }
  int bad = 0;
  auto run = [&](bool comp) {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
      th.emplace_back([&, t]() {
        for (int i = cut[t]; i < cut[t + 1]; i++) {
          const int sz = (int)len[i], bound = (int)(boff[i + 1] - boff[i]);
          if (comp) {
            blen[i] = LZ4_compress_limitedOutput(src + off[i], &blocks[boff[i]], sz, bound);
          } else {
            int r = LZ4_decompress_safe_partial(&blocks[boff[i]], &out[ooff[i]], blen[i], sz, sz);
            if (r != sz) bad = 1;
          }
        }
      });
    }
    for (auto& x : th) x.join();
  };
  run(true);
  run(false);
  double tc = 0, td = 0;
  for (int p = 0; p < passes; p++) {
    auto a = std::chrono::steady_clock::now();
    run(true);
    auto b = std::chrono::steady_clock::now();
    run(false);
    auto c = std::chrono::steady_clock::now();
    tc += std::chrono::duration<double>(b - a).count();
    td += std::chrono::duration<double>(c - b).count();
  }
  uint64_t cb = 0;
  for (int i = 0; i < n; i++) cb += (uint64_t)blen[i];
  *t_compress = tc;
  *t_decompress = td;
  *comp_bytes = cb;
  for (int i = 0; i < n && !bad; i++)
    if (memcmp(&out[ooff[i]], src + off[i], len[i]) != 0) bad = 1;
  return bad ? -1 : 0;
}

// ByteArray's size/checksum setters are private to KingDB's own classes; the
// shim reaches them through one of the befriended names (NetworkTask lives in
// network/server.h, which is not part of this build), exactly as
// StorageEngine::GetEntry sets them (storage/storage_engine.h:497-508).
namespace kdb {
class NetworkTask {
 public:
  static void Set(ByteArray& v, uint64_t size, uint64_t svc, uint32_t checksum, uint32_t checksum_initial) {
    v.set_size(size);
    v.set_size_compressed(svc);
    v.set_checksum(checksum);
    v.set_checksum_initial(checksum_initial);
  }
};
}  // namespace kdb

// CompressorLZ4::UncompressByteArray (compressor.cc:140-249) on a stored value
// region, as Database::GetRaw calls it (database.cc:65-68).  Returns 0 OK,
// 1 IOError "Invalid checksum.", 2 any other IOError; *out_n = value size.
extern "C" int ref_uncompress_value(const char* stored, uint64_t stored_len, uint64_t svc, uint64_t size,
                                    uint32_t checksum, uint32_t checksum_initial, int verify, char* out,
                                    uint64_t* out_n) {
  std::vector<char> buf(stored_len + 64, 0);
  if (stored_len) memcpy(buf.data(), stored, stored_len);
  kdb::ByteArray v = kdb::NewDeepCopyByteArray(buf.data(), stored_len + 64);
  kdb::NetworkTask::Set(v, size, svc, checksum, checksum_initial);
  kdb::CompressorLZ4 c;
  kdb::ByteArray o;
  kdb::Status s = c.UncompressByteArray(v, verify != 0, &o);
  *out_n = o.size();
  if (o.size()) memcpy(out, o.data(), o.size());
  if (s.IsOK()) return 0;
  return s.ToString().find("Invalid checksum") != std::string::npos ? 1 : 2;
}

// ---- CPU baseline for the read path (bench.py --workload get, kind "reference") ----
// Database::GetRaw's decode step over n stored values: CompressorLZ4::
// UncompressByteArray (verify off, ReadOptions' default) with `threads`
// std::threads on blocked ranges, each with its own CompressorLZ4.  The
// ByteArrays are built before the clock starts; one warm-up pass, then
// `passes` timed passes.  Returns 0, or -1 if any value fails or differs in
// size from `size`.
extern "C" int ref_bench_get(const char* stored, const uint64_t* off, const uint64_t* len, int n, uint64_t size,
                             int threads, int passes, double* seconds) {
  std::vector<kdb::ByteArray> vals(n);
  for (int i = 0; i < n; i++) {
    std::vector<char> buf(len[i] + 64, 0);
    memcpy(buf.data(), stored + off[i], len[i]);
    vals[i] = kdb::NewDeepCopyByteArray(buf.data(), len[i] + 64);
    kdb::NetworkTask::Set(vals[i], size, len[i], 0, 0);
  }
  int bad = 0;
  auto run = [&]() {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
      th.emplace_back([&, t]() {
        kdb::CompressorLZ4 c;
        const int lo = (int)((int64_t)n * t / threads), hi = (int)((int64_t)n * (t + 1) / threads);
        for (int i = lo; i < hi; i++) {
          kdb::ByteArray o;
          kdb::Status s = c.UncompressByteArray(vals[i], false, &o);
          if (!s.IsOK() || o.size() != size) bad = 1;
        }
      });
    }
    for (auto& x : th) x.join();
  };
  run();
  auto a = std::chrono::steady_clock::now();
  for (int p = 0; p < passes; p++) run();
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
  return bad ? -1 : 0;
}
