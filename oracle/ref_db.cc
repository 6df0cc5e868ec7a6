// oracle/ref_db.cc -- TEST INFRASTRUCTURE ONLY (compiled into oracle/_ref/ by
// `make -C oracle ref`, linked against the REFERENCE's own objects compiled in
// place from /root/reference; no reference source is copied here).
//
// Drives the real KingDB write path (Database::PutPart -> WriteBuffer ->
// HSTableManager, interface/database.cc:87-276, storage/hstable_manager.h:628-847)
// over a put stream read from a file, then closes the database so every
// HSTable is flushed with its offset array.  tests/golden/make_golden.py runs
// it to pin the write-path restatement (oracle/lz4_oracle.c orc_put_*) and the
// GPU put kernels against the bytes the reference itself writes.
//
//   ref_db <dbdir> <stream.bin> [maximum_part_size [hstable_size [hash [none]]]]   (hash: 0 murmur3, 1 xxhash;
//   none: compression off -- a diagnostic of what the write path costs without the codec)
//
// stream.bin: records of
//   u32 key_len, key bytes, u64 size_value, u32 nchunks,
//   nchunks x (u32 chunk_len, chunk bytes)
// and each chunk is handed to Database::PutPart(key, chunk, offset, size_value)
// in order (offset = bytes of the value already sent), like a client
// streaming a value in parts (network/server.cc:258).  A record whose nchunks
// has bit 31 set gives each chunk an explicit offset instead:
//   nchunks x (u32 chunk_len, u64 offset, chunk bytes)
// (a client that sends parts out of order, with gaps or overlaps, or
// interleaves the parts of two values -- the puts PutPartValidSize may refuse,
// database.cc:261-266).
//
// KDB_DB_KEEP_GOING=1: a refused PutPart is reported ("put <record> chunk
// <c>: <status>" on stderr) and the stream goes on; the database is closed as
// usual and the exit status is 3 if any put was refused.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <thread>
#include <string>
#include <vector>

#include "interface/database.h"
#include "util/byte_array.h"
#include "util/status.h"

static bool rd(FILE* f, void* p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

// ref_db --verify <dbdir> <stream.bin> [options as above]: opens the database and reads every
// key of the stream back three ways -- Database::Get (verify_checksums off: the
// reference's double CRC stream fails it for compressed values, SURVEY.md
// §0-7), the iterator's GetValue, and a MultipartReader per key -- and returns
// 1 if any value read back differs from the last one put for its key.  (The fault-injection test of the
// flush hook: no entry reaches an HSTable without its frame and checksum.)
static int verify(int argc, char** argv) {
  const char *dir = argv[2], *stream = argv[3];
  kdb::Logger::set_current_level("emerg");
  kdb::DatabaseOptions options;
  if (argc > 4) options.storage__maximum_part_size = strtoull(argv[4], nullptr, 0);
  if (argc > 5) options.storage__hstable_size = strtoull(argv[5], nullptr, 0);
  if (argc > 6) options.hash = strtoul(argv[6], nullptr, 0) ? kdb::kxxHash_64 : kdb::kMurmurHash3_64;
  kdb::Database db(options, dir);
  kdb::Status s = db.Open();
  if (!s.IsOK()) {
    fprintf(stderr, "open: %s\n", s.ToString().c_str());
    return 1;
  }
  FILE* f = fopen(stream, "rb");
  if (!f) return 1;
  std::vector<std::pair<std::string, std::string>> kv;
  for (;;) {
    uint32_t klen;
    if (fread(&klen, 4, 1, f) != 1) break;
    std::string key(klen, '\0');
    uint64_t vsize;
    uint32_t nchunks;
    if (!rd(f, &key[0], klen) || !rd(f, &vsize, 8) || !rd(f, &nchunks, 4)) return 1;
    const bool explicit_offsets = (nchunks & 0x80000000u) != 0;
    nchunks &= 0x7FFFFFFFu;
    std::string value;
    uint64_t off = 0;
    for (uint32_t c = 0; c < nchunks; c++) {
      uint32_t clen;
      if (!rd(f, &clen, 4)) return 1;
      if (explicit_offsets && !rd(f, &off, 8)) return 1;
      std::string buf(clen, '\0');
      if (!rd(f, &buf[0], clen)) return 1;
      if (value.size() < off + clen) value.resize(off + clen, '\0');   // (the bytes as the parts lay them)
      value.replace(off, clen, buf);
      off += clen;
    }
    kv.emplace_back(key, value);
  }
  fclose(f);
  std::map<std::string, std::string> last;
  for (auto& p : kv) last[p.first] = p.second;
  uint64_t found = 0, missing = 0, bad = 0;
  kdb::ReadOptions ro;
  for (auto& p : last) {
    std::string out;
    kdb::Status g = db.Get(ro, p.first, &out);
    if (g.IsNotFound()) {
      missing++;
    } else if (!g.IsOK() || out != p.second) {
      bad++;
      if (bad <= 5) fprintf(stderr, "key %s: %s\n", p.first.c_str(), g.ToString().c_str());
    } else {
      found++;
    }
  }
  // the same values through the iterator (GetValue) and MultipartReader
  uint64_t it_items = 0, it_bad = 0, mp_bad = 0;
  {
    kdb::Iterator it = db.NewIterator(ro);
    for (it.Begin(); it.IsValid(); it.Next()) {
      kdb::ByteArray k = it.GetKey(), v = it.GetValue();
      it_items++;
      auto f = last.find(k.ToString());
      if (f == last.end() || !it.GetStatus().IsOK() || v.ToString() != f->second) {
        if (it_bad++ < 5) fprintf(stderr, "iterator key %s: %s\n", k.ToString().c_str(), it.GetStatus().ToString().c_str());
      }
    }
  }
  for (auto& p : last) {
    std::string probe;
    if (!db.Get(ro, p.first, &probe).IsOK()) continue;   // (missing: counted above)
    kdb::MultipartReader mp = db.NewMultipartReader(ro, p.first);
    std::string out;
    for (mp.Begin(); mp.IsValid(); mp.Next()) {   // (a part's status is the stream's: "unfinished" mid-way)
      kdb::ByteArray part;
      mp.GetPart(&part);
      out += part.ToString();
    }
    if (!mp.GetStatus().IsOK() || out != p.second) {
      if (mp_bad++ < 5) fprintf(stderr, "multipart key %s: %s\n", p.first.c_str(), mp.GetStatus().ToString().c_str());
    }
  }
  db.Close();
  printf("verify %llu found %llu missing %llu bad %llu iterated %llu iterator_bad %llu multipart_bad\n",
         (unsigned long long)found, (unsigned long long)missing, (unsigned long long)bad,
         (unsigned long long)it_items, (unsigned long long)it_bad, (unsigned long long)mp_bad);
  return bad || it_bad || mp_bad ? 1 : 0;
}

// ref_db --readrandom <dbdir> <keys> <reads> <threads> [maximum_part_size [hstable_size [hash]]]:
// db_bench's ReadRandom (/root/reference/doc/bench/db_bench_kingdb.cc:505-518)
// on a database already written (keys "%016d" of 0 .. keys-1): <threads>
// client threads share <reads> Database::Get calls of uniformly random keys
// (std::mt19937 per thread: the reference's leveldb Random is not vendored),
// ReadOptions defaults.  Prints reads/s, the values found and their bytes.
static int readrandom(int argc, char** argv) {
  const char* dir = argv[2];
  const long keys = atol(argv[3]), reads = atol(argv[4]);
  const int threads = atoi(argv[5]);
  kdb::Logger::set_current_level("emerg");
  kdb::DatabaseOptions options;
  if (argc > 6) options.storage__maximum_part_size = strtoull(argv[6], nullptr, 0);
  if (argc > 7) options.storage__hstable_size = strtoull(argv[7], nullptr, 0);
  if (argc > 8) options.hash = strtoul(argv[8], nullptr, 0) ? kdb::kxxHash_64 : kdb::kMurmurHash3_64;
  kdb::Database db(options, dir);
  kdb::Status s = db.Open();
  if (!s.IsOK()) {
    fprintf(stderr, "open: %s\n", s.ToString().c_str());
    return 1;
  }
  std::vector<uint64_t> found(threads, 0), bytes(threads, 0);
  std::vector<std::thread> th;
  const auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      std::mt19937_64 rng(301 + t);
      kdb::ReadOptions ro;
      const long n = reads / threads + (t < reads % threads ? 1 : 0);
      for (long i = 0; i < n; i++) {
        char key[100];
        snprintf(key, sizeof(key), "%016d", (int)(rng() % (uint64_t)keys));
        std::string value;
        if (db.Get(ro, key, &value).IsOK()) {
          found[t]++;
          bytes[t] += value.size();
        }
      }
    });
  for (auto& x : th) x.join();
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t f = 0, b = 0;
  for (int t = 0; t < threads; t++) {
    f += found[t];
    b += bytes[t];
  }
  db.Close();
  printf("readrandom %ld reads %d threads %.6f s %.1f reads_per_s found %llu bytes %llu\n", reads, threads, sec,
         reads / sec, (unsigned long long)f, (unsigned long long)b);
  return f == (uint64_t)reads ? 0 : 1;
}

// ref_db --two <dirA> <dirB> <streamA.bin> <streamB.bin> [maximum_part_size [hstable_size [hash]]]:
// ONE client thread writes two databases at once, part by part in turn (the
// next part of stream A's current record, then the next of B's): each
// database must end up with the files a run of its stream alone writes.  (The
// reference keeps PutPartValidSize's state per Database and per thread,
// database.cc:143-266, so interleaving the parts of values in two databases
// is legal; the flush hook's per-thread lane and value tracking must be kept
// per database too.)  Regular streams only (no explicit offsets).
struct PartCursor {
  FILE* f = nullptr;
  std::string key;
  uint64_t vsize = 0, off = 0;
  uint32_t left = 0;
  bool next(std::string* k, std::vector<char>* part, uint64_t* off_out, uint64_t* vs) {
    while (left == 0) {
      uint32_t klen;
      if (fread(&klen, 4, 1, f) != 1) return false;
      key.assign(klen, '\0');
      if (!rd(f, &key[0], klen) || !rd(f, &vsize, 8) || !rd(f, &left, 4)) return false;
      left &= 0x7FFFFFFFu;
      off = 0;
    }
    uint32_t clen;
    if (!rd(f, &clen, 4)) return false;
    part->resize(clen);
    if (!rd(f, part->data(), clen)) return false;
    *k = key;
    *off_out = off;
    *vs = vsize;
    off += clen;
    left--;
    return true;
  }
};

static int two(int argc, char** argv) {
  kdb::Logger::set_current_level("emerg");
  kdb::DatabaseOptions options;
  options.compression = kdb::kLZ4Compression;
  if (argc > 6) options.storage__maximum_part_size = strtoull(argv[6], nullptr, 0);
  if (argc > 7) options.storage__hstable_size = strtoull(argv[7], nullptr, 0);
  if (argc > 8) options.hash = strtoul(argv[8], nullptr, 0) ? kdb::kxxHash_64 : kdb::kMurmurHash3_64;
  kdb::Database da(options, argv[2]), dbb(options, argv[3]);
  kdb::Database* db[2] = {&da, &dbb};
  PartCursor cur[2];
  for (int i = 0; i < 2; i++) {
    kdb::Status s = db[i]->Open();
    if (!s.IsOK()) {
      fprintf(stderr, "open %d: %s\n", i, s.ToString().c_str());
      return 1;
    }
    cur[i].f = fopen(argv[4 + i], "rb");
    if (!cur[i].f) return 1;
  }
  kdb::WriteOptions wo;
  bool more[2] = {true, true};
  uint64_t parts = 0;
  while (more[0] || more[1]) {
    for (int i = 0; i < 2; i++) {
      if (!more[i]) continue;
      std::string key;
      std::vector<char> part;
      uint64_t off, vs;
      if (!cur[i].next(&key, &part, &off, &vs)) {
        more[i] = false;
        continue;
      }
      kdb::ByteArray k = kdb::NewDeepCopyByteArray(key.data(), key.size());
      kdb::ByteArray v = kdb::NewDeepCopyByteArray(part.data(), part.size());
      kdb::Status s = db[i]->PutPart(wo, k, v, off, vs);
      if (!s.IsOK()) {
        fprintf(stderr, "db %d part %llu: %s\n", i, (unsigned long long)parts, s.ToString().c_str());
        return 1;
      }
      parts++;
    }
  }
  for (int i = 0; i < 2; i++) {
    fclose(cur[i].f);
    db[i]->Close();
  }
  printf("%llu parts into two databases\n", (unsigned long long)parts);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 4 && !strcmp(argv[1], "--verify")) return verify(argc, argv);
  if (argc >= 6 && !strcmp(argv[1], "--two")) return two(argc, argv);
  if (argc >= 6 && !strcmp(argv[1], "--readrandom")) return readrandom(argc, argv);
  if (argc < 3) {
    fprintf(stderr, "usage: ref_db <dbdir> <stream.bin> [maximum_part_size [hstable_size [hash [none]]]]\n");
    return 2;
  }
  kdb::Logger::set_current_level("emerg");
  kdb::DatabaseOptions options;
  options.compression = kdb::kLZ4Compression;
  if (argc > 3) options.storage__maximum_part_size = strtoull(argv[3], nullptr, 0);
  if (argc > 4) options.storage__hstable_size = strtoull(argv[4], nullptr, 0);
  if (argc > 5) options.hash = strtoul(argv[5], nullptr, 0) ? kdb::kxxHash_64 : kdb::kMurmurHash3_64;
  if (argc > 6 && !strcmp(argv[6], "none")) options.compression = kdb::kNoCompression;   // (diagnostics)
  kdb::Database db(options, argv[1]);
  kdb::Status s = db.Open();
  if (!s.IsOK()) {
    fprintf(stderr, "open: %s\n", s.ToString().c_str());
    return 1;
  }
  // the whole stream is read into memory first, so the timed region is the
  // write path alone: Database::PutPart per chunk, then Close (flush + offset arrays)
  FILE* f = fopen(argv[2], "rb");
  if (!f) return 1;
  std::vector<char> all;
  {
    char buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof(buf), f)) > 0) all.insert(all.end(), buf, buf + r);
    fclose(f);
  }
  f = fmemopen(all.data(), all.size(), "rb");
  if (!f) return 1;
  const char* kg = getenv("KDB_DB_KEEP_GOING");
  const bool keep_going = kg && *kg && *kg != '0';
  uint64_t refused = 0;
  const auto t0 = std::chrono::steady_clock::now();
  kdb::WriteOptions wo;
  uint64_t puts = 0;
  for (;;) {
    uint32_t klen;
    if (fread(&klen, 4, 1, f) != 1) break;
    std::string key(klen, '\0');
    uint64_t vsize;
    uint32_t nchunks;
    if (!rd(f, &key[0], klen) || !rd(f, &vsize, 8) || !rd(f, &nchunks, 4)) return 1;
    const bool explicit_offsets = (nchunks & 0x80000000u) != 0;
    nchunks &= 0x7FFFFFFFu;
    uint64_t off = 0;
    for (uint32_t c = 0; c < nchunks; c++) {
      uint32_t clen;
      if (!rd(f, &clen, 4)) return 1;
      if (explicit_offsets && !rd(f, &off, 8)) return 1;
      std::vector<char> buf(clen);
      if (!rd(f, buf.data(), clen)) return 1;
      kdb::ByteArray k = kdb::NewDeepCopyByteArray(key.data(), key.size());
      kdb::ByteArray v = kdb::NewDeepCopyByteArray(buf.data(), clen);
      s = db.PutPart(wo, k, v, off, vsize);
      if (!s.IsOK()) {
        fprintf(stderr, "put %llu chunk %u: %s\n", (unsigned long long)puts, c, s.ToString().c_str());
        if (!keep_going) return 1;
        refused++;
      }
      off += clen;
    }
    puts++;
  }
  fclose(f);
  const double t_put = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  db.Close();
  const double t_all = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  // puts: until the last PutPart returned (db_bench's view: writes are buffered);
  // with close: until every HSTable is on disk with its offset array
  printf("%llu puts %.6f s put %.6f s with close\n", (unsigned long long)puts, t_put, t_all);
  return refused ? 3 : 0;
}
