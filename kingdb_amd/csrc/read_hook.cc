// kingdb_amd/csrc/read_hook.cc -- the read-side hooks
// (kingdb_include/interface/lz4_read.h): batched GPU decode of stored values
// for the iterators' GetValue and for MultipartReader.  Compiled by the KingDB
// build that applies the hooks (oracle/kingdb_hook.py, INTEGRATION.md level 5).
//
// Semantics are MultipartReader's (/root/reference/interface/multipart.h:65-154),
// which the iterators' GetValue runs per value (iterator.h:221-243, 446-468):
// frames decoded one after the other, the all-zero header that starts a raw
// tail, the raw tail in 1 MiB steps, and -- with verify_checksums -- a CRC32C
// over every stored byte seeded with crc32c(key), compared only when the value
// ends in frames.  kdb_get_values_batch's verify mode 2 is exactly that check.
#include "interface/lz4_read.h"

#include <cstring>
#include <mutex>

#include "../../include/kdb_lz4.h"
#include "../../include/kdb_put.h"
#include "algorithm/compressor.h"

namespace kdb {

namespace {

inline uint64_t a64(uint64_t x) { return (x + 63) & ~uint64_t(63); }

// Per-thread pinned host + device staging and a stream (the iterators and
// MultipartReaders of one thread share it).
struct ReadStaging {
  void* host = nullptr;
  void* dev = nullptr;
  void* stream = nullptr;
  uint64_t hcap = 0, dcap = 0;
  int device = -1;
  ~ReadStaging() { release(); }
  void release() {
    if (host) kdb_lz4_host_free(host);
    if (dev) kdb_lz4_free(dev);
    if (stream) kdb_lz4_stream_destroy(stream);
    host = dev = stream = nullptr;
    hcap = dcap = 0;
  }
  void drop() {   // after a failure: nothing queued may still write the buffers we reuse
    if (stream && kdb_lz4_stream_sync(stream) == KDB_LZ4_OK) {
      release();
      return;
    }
    host = dev = stream = nullptr;
    hcap = dcap = 0;
  }
  static uint64_t grow(uint64_t cap, uint64_t want) {
    uint64_t c = cap ? cap : (4ull << 20);
    while (c < want) c *= 2;
    return c;
  }
  bool reserve(uint64_t hbytes, uint64_t dbytes) {
    int d = 0;
    if (kdb_lz4_get_device(&d) != KDB_LZ4_OK) return false;
    if (d != device) {
      release();
      device = d;
    }
    if (!stream && kdb_lz4_stream_create(&stream) != KDB_LZ4_OK) return false;
    if (hbytes > hcap) {
      if (host) kdb_lz4_host_free(host);
      host = nullptr;
      const uint64_t c = grow(hcap, hbytes);
      hcap = 0;
      if (kdb_lz4_host_alloc(&host, c) != KDB_LZ4_OK) return false;
      hcap = c;
    }
    if (dbytes > dcap) {
      if (dev) kdb_lz4_free(dev);
      dev = nullptr;
      const uint64_t c = grow(dcap, dbytes);
      dcap = 0;
      if (kdb_lz4_malloc(&dev, c) != KDB_LZ4_OK) return false;
      dcap = c;
    }
    return true;
  }
};

Status decode_failed() { return Status::IOError("LZ4_decompress_safe_partial() failed"); }

// One batch through kdb_get_values_batch; status codes (get.hip): 0, -1 a frame
// failed, -2 checksum, KDB_LZ4_VALUE_UNSUPPORTED.  out_len = bytes defined.
int gpu_decode(std::vector<ByteArray>& values, bool verify, ByteArray* arena, std::vector<uint64_t>* out_at,
               std::vector<uint64_t>* out_len, std::vector<int32_t>* status) {
  const uint32_t n = (uint32_t)values.size();
  uint64_t sbytes = 0, obytes = 0, frame_cap = 0, max_in = 0, max_out = 0;
  for (ByteArray& v : values) {
    const CompressorLZ4::StoredView w = CompressorLZ4::View(v);
    const uint64_t svc = w.size_compressed, sz = w.size;
    if (svc > 0xFFFFFFFFull || sz > 0xFFFFFFFFull) return KDB_LZ4_EUNSUPPORTED;
    sbytes += a64(svc);
    obytes += a64(sz);
    frame_cap += svc / 8 + 1;
    if (svc > max_in) max_in = svc;
    if (sz > max_out) max_out = sz;
  }
  // layout (host and device alike): [meta][stored]; device adds [out][scratch]
  const uint64_t o_soff = 0, o_avail = 8ull * n, o_svc = 16ull * n, o_size = 24ull * n, o_ooff = 32ull * n,
                 o_ck = 40ull * n, o_ci = 44ull * n, o_olen = 48ull * n, o_st = 56ull * n,
                 meta = a64(60ull * n), o_stored = meta, in_bytes = o_stored + sbytes + 64;
  const uint64_t o_out = a64(in_bytes), scratch = kdb_get_scratch_bytes(n, frame_cap),
                 o_scr = a64(o_out + obytes + 64), dev_bytes = o_scr + scratch;
  const uint64_t h_out = a64(in_bytes), host_bytes = h_out + obytes + 64;
  thread_local ReadStaging stg;
  if (!stg.reserve(host_bytes, dev_bytes)) return KDB_LZ4_EHIP;
  char* hb = static_cast<char*>(stg.host);
  char* db = static_cast<char*>(stg.dev);
  auto H64 = [&](uint64_t o) { return reinterpret_cast<uint64_t*>(hb + o); };
  auto H32 = [&](uint64_t o) { return reinterpret_cast<uint32_t*>(hb + o); };
  uint64_t so = 0, oo = 0;
  for (uint32_t i = 0; i < n; i++) {
    ByteArray& v = values[i];
    const CompressorLZ4::StoredView w = CompressorLZ4::View(v);
    const uint64_t svc = w.size_compressed;
    H64(o_soff)[i] = so;
    H64(o_avail)[i] = svc;
    H64(o_svc)[i] = svc;
    H64(o_size)[i] = w.size;
    H64(o_ooff)[i] = oo;
    H32(o_ck)[i] = w.checksum;
    H32(o_ci)[i] = w.checksum_initial;
    memcpy(hb + o_stored + so, v.data(), svc);
    so += a64(svc);
    oo += a64(w.size);
  }
  void* st = stg.stream;
  auto D8 = [&](uint64_t o) { return reinterpret_cast<uint8_t*>(db + o); };
  auto D32 = [&](uint64_t o) { return reinterpret_cast<uint32_t*>(db + o); };
  auto D64 = [&](uint64_t o) { return reinterpret_cast<uint64_t*>(db + o); };
  int rc = kdb_lz4_memcpy_h2d(db, hb, in_bytes, st);
  if (!rc)
    rc = kdb_get_values_batch(st, D8(o_stored), D64(o_soff), D64(o_avail), D64(o_svc), D64(o_size), n, D8(o_out),
                              D64(o_ooff), verify ? 2 : 0, D32(o_ck), D32(o_ci), frame_cap, (uint32_t)max_in,
                              (uint32_t)max_out, D8(o_scr), scratch, D64(o_olen),
                              reinterpret_cast<int32_t*>(db + o_st));
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb + o_olen, db + o_olen, 12ull * n, st);
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb + h_out, db + o_out, obytes, st);
  if (!rc) rc = kdb_lz4_stream_sync(st);
  if (rc) {
    stg.drop();
    return rc;
  }
  char* a = new char[obytes + 1];
  memcpy(a, hb + h_out, obytes);
  *arena = NewShallowCopyByteArray(a, obytes + 1);
  out_at->resize(n);
  out_len->resize(n);
  status->resize(n);
  for (uint32_t i = 0; i < n; i++) {
    (*out_at)[i] = H64(o_ooff)[i];
    (*out_len)[i] = H64(o_olen)[i];
    (*status)[i] = reinterpret_cast<const int32_t*>(hb + o_st)[i];
  }
  return KDB_LZ4_OK;
}

}  // namespace

bool LZ4DecodeValues(std::vector<ByteArray>& values, bool verify, std::vector<ByteArray>* out,
                     std::vector<Status>* st) {
  out->assign(values.size(), ByteArray());
  st->assign(values.size(), Status::OK());
  ByteArray arena;
  std::vector<uint64_t> at, len;
  std::vector<int32_t> status;
  if (gpu_decode(values, verify, &arena, &at, &len, &status) != KDB_LZ4_OK) {
    for (Status& s : *st) s = Status::IOError("GPU decode batch failed");
    return false;
  }
  for (size_t i = 0; i < values.size(); i++) {
    (*out)[i] = CompressorLZ4::Slice(arena, at[i], values[i].size());
    if (status[i] == -2) (*st)[i] = Status::IOError("Invalid checksum.");
    else if (status[i] != 0) (*st)[i] = decode_failed();
  }
  return true;
}

// ------------------------------------------------------------- LZ4ReadAhead
ByteArray LZ4ReadAhead::Get(const ReadOptions& read_options, ByteArray& value, uint64_t max_size, Status* status,
                            const Peek& peek) {
  // the iterator asks in order: the expected value, or one a little further
  // on (entries Next() skipped); anything else starts a new batch
  const char* key = value.data();
  size_t i = cursor_;
  while (i < batch_.size() && i < cursor_ + 64 && batch_[i].stored != key) i++;
  if (i >= batch_.size() || batch_[i].stored != key || batch_[i].out.size() != value.size()) {
    std::vector<ByteArray> batch;
    batch.push_back(value);
    std::vector<ByteArray> ahead;
    peek(&ahead);
    uint64_t bytes = CompressorLZ4::View(value).size_compressed;
    for (ByteArray& v : ahead) {
      if (batch.size() >= kMaxValues || bytes >= kMaxBytes) break;
      const uint64_t svc = CompressorLZ4::View(v).size_compressed;
      if (svc == 0 || v.size() > max_size) continue;
      batch.push_back(v);
      bytes += svc;
    }
    std::vector<ByteArray> out;
    std::vector<Status> st;
    LZ4DecodeValues(batch, read_options.verify_checksums, &out, &st);
    batch_.clear();
    batch_.reserve(batch.size());
    for (size_t j = 0; j < batch.size(); j++) batch_.push_back(Decoded{batch[j].data(), out[j], st[j]});
    i = 0;
  }
  cursor_ = i + 1;
  *status = batch_[i].st;
  ByteArray r = batch_[i].out;
  batch_[i].out = ByteArray();
  return r;
}

// ------------------------------------------------------- LZ4MultipartDecode
void LZ4MultipartDecode::Prepare(const ReadOptions& read_options, ByteArray& value) {
  active_ = false;
  parts_.clear();
  next_ = 0;
  out_ = ByteArray();
  value_ = value;
  const uint64_t svc = CompressorLZ4::View(value).size_compressed;
  if (svc == 0) return;   // not compressed: the reference's raw path, no codec
  // the frame walk MultipartReader::Next does (multipart.h:65-115): frames
  // until the end or an all-zero header, which starts the raw tail
  const char* d = value.data();
  std::vector<uint64_t> frame_raw;
  uint64_t off = 0, tail_at = 0;
  bool tail = false;
  while (off < svc) {
    if (svc - off < 8) return;          // malformed: the reference's own path decides
    bool zero = true;
    for (int b = 0; b < 8; b++) zero = zero && d[off + b] == 0;
    if (zero) {
      tail = true;
      tail_at = off + 8;
      break;
    }
    uint32_t c, sz;
    memcpy(&c, d + off, 4);
    memcpy(&sz, d + off + 4, 4);
    if (c > 0 && c < 8) return;
    frame_raw.push_back(sz);
    off += c > 0 ? (uint64_t)c : 8ull + sz;
  }
  if (!tail && off != svc) return;
  std::vector<ByteArray> one{value};
  ByteArray arena;
  std::vector<uint64_t> at, len;
  std::vector<int32_t> status;
  if (gpu_decode(one, read_options.verify_checksums, &arena, &at, &len, &status) != KDB_LZ4_OK) return;
  out_ = CompressorLZ4::Slice(arena, at[0], value.size());
  active_ = true;
  fail_at_end_ = status[0] == -1 || status[0] == KDB_LZ4_VALUE_UNSUPPORTED;
  // every frame that decoded before a failing one is a part (out_len = the bytes defined)
  uint64_t o = 0;
  for (uint64_t r : frame_raw) {
    if (fail_at_end_ && o + r > len[0]) break;
    parts_.push_back(Part{o, r, 0});
    o += r;
  }
  if (fail_at_end_) {
    final_ = decode_failed();
    return;
  }
  if (tail) {   // the raw tail in 1 MiB steps, views of the stored bytes (multipart.h:118-146)
    for (uint64_t in = tail_at; in < svc;) {
      const uint64_t step = svc - in < (1ull << 20) ? svc - in : (1ull << 20);
      parts_.push_back(Part{in, step, 1});
      in += step;
    }
    final_ = Status::OK();   // no CRC comparison after a raw tail
  } else {
    final_ = status[0] == -2 ? Status::IOError("Invalid checksum.") : Status::OK();
  }
}

void LZ4MultipartDecode::Next(ByteArray* chunk, Status* status, bool* is_valid_stream) {
  if (next_ < parts_.size()) {
    const Part& p = parts_[next_++];
    *chunk = CompressorLZ4::Slice(p.kind == 0 ? out_ : value_, p.at, p.size);
    // a decoded frame leaves the stream's status as it was ("Stream is
    // unfinished" after Begin, multipart.h:46); a raw step sets OK (:146)
    if (p.kind == 1) *status = Status::OK();
    return;
  }
  *is_valid_stream = false;
  *status = final_;
  if (fail_at_end_) *chunk = ByteArray();
}

}  // namespace kdb
