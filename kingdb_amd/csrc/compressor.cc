// kingdb_amd/csrc/compressor.cc -- CompressorLZ4 drop-in over the gfx950 codec.
//
// Control flow and Status behaviour follow /root/reference/algorithm/compressor.cc
// line by line (cited per method); every LZ4 block is produced / decoded by the
// HIP kernels behind include/kdb_lz4.h.
//
// Built two ways: standalone (against kdb_types.h's mirrors, e.g. tests/cpp),
// or inside KingDB with -DKDB_LZ4_IN_KINGDB and the shadow include directory
// kingdb_amd/kingdb_include ahead of KingDB's root (oracle/Makefile `kingdb`,
// INTEGRATION.md level 2).
#include "compressor.h"

#include <cstring>
#include <mutex>
#include <string>

#include "kdb_lz4.h"

KDB_LZ4_NS_OPEN

namespace {
inline void put_u32le(char* p, uint32_t v) {
  for (int i = 0; i < 4; i++) p[i] = (char)(v >> (8 * i));
}
inline uint32_t get_u32le(const char* p) {
  uint32_t v = 0;
  for (int i = 0; i < 4; i++) v |= (uint32_t)(uint8_t)p[i] << (8 * i);
  return v;
}

// CRC32C (Castagnoli, reflected), slice-by-8.  Same value as the reference's
// crc32c::Extend (algorithm/crc32c.cc:296-340).
struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
      for (int s = 1; s < 8; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTables& crc_tables() {
  static const Crc32cTables tables;
  return tables;
}
}  // namespace

#if defined(__x86_64__)
// The same CRC with SSE4.2's crc32 instruction (the Castagnoli polynomial):
// every Uncompress streams its frame through the CRC (compressor.cc:126), so a
// 4 KiB Get pays ~2.4 KB of it on the host.
static __attribute__((target("sse4.2"))) uint32_t crc32c_extend_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t l = crc ^ 0xffffffffu;
  for (; n >= 8; n -= 8, p += 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    l = __builtin_ia32_crc32di(l, w);
  }
  uint32_t c = (uint32_t)l;
  for (; n; n--) c = __builtin_ia32_crc32qi(c, *p++);
  return c ^ 0xffffffffu;
}
static const bool kHwCrc32c = __builtin_cpu_supports("sse4.2");
#endif

uint32_t Crc32cExtend(uint32_t crc, const char* data, size_t n) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
#if defined(__x86_64__)
  if (kHwCrc32c) return crc32c_extend_hw(crc, p, n);
#endif
  const Crc32cTables& T = crc_tables();
  uint32_t l = crc ^ 0xffffffffu;
  while (n >= 8) {
    uint32_t lo = l ^ ((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
    uint32_t hi = (uint32_t)p[4] | (uint32_t)p[5] << 8 | (uint32_t)p[6] << 16 | (uint32_t)p[7] << 24;
    l = T.t[7][lo & 0xff] ^ T.t[6][(lo >> 8) & 0xff] ^ T.t[5][(lo >> 16) & 0xff] ^ T.t[4][lo >> 24] ^
        T.t[3][hi & 0xff] ^ T.t[2][(hi >> 8) & 0xff] ^ T.t[1][(hi >> 16) & 0xff] ^ T.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) l = T.t[0][(l ^ *p++) & 0xff] ^ (l >> 8);
  return l ^ 0xffffffffu;
}

void CRC32LZ4::stream(const char* data, size_t n) {  // crc32c.h:87-92
  ts_.put(Crc32cExtend((uint32_t)ts_.get(), data, n));
}

// compressor.cc:9-12
// Per device: kdb_lz4_warmup readies the calling thread's current device once
// (cached per device inside the library, retried after a failure), so a
// database opened on another device does not pay its first launches and
// self-test inside its first puts.  No device: the calls report it later.
void CompressorLZ4::WarmUp() { (void)kdb_lz4_warmup(); }

void CompressorLZ4::ResetThreadLocalStorage() {
  ts_compress_.reset();
  ts_uncompress_.reset();
}

// compressor.cc:15-65
Status CompressorLZ4::Compress(char* source, uint64_t size_source, char** dest, uint64_t* size_dest) {
  uint32_t bound = (uint32_t)kdb_lz4_compressBound((int)size_source);
  *size_dest = 0;
  *dest = new char[8 + bound];
  int ret = kdb_lz4_compress_limitedOutput(source, (*dest) + 8, (int)size_source, (int)bound);
  if (ret <= 0) {
    delete[] * dest;
    *dest = nullptr;
    return Status::IOError("LZ4_compress_limitedOutput() failed");
  }
  uint32_t size_compressed = (uint32_t)ret + 8;
  uint32_t size_compressed_stored = size_compressed;
  if ((uint64_t)ret > size_source) {  // raw fallback, compressor.cc:40-48
    if (size_source > 8 + (uint64_t)bound) {
      delete[] * dest;
      *dest = new char[8 + size_source];
    }
    memcpy((*dest) + 8, source, size_source);
    size_compressed = (uint32_t)size_source + 8;
    size_compressed_stored = 0;
  }
  put_u32le(*dest, size_compressed_stored);
  put_u32le((*dest) + 4, (uint32_t)size_source);
  ts_compress_.put(ts_compress_.get() + size_compressed);
  *size_dest = size_compressed;
  return Status::OK();
}

// compressor.cc:68-72
bool CompressorLZ4::IsUncompressionDone(uint64_t size_source_total) {
  return ts_uncompress_.get() == size_source_total;
}

// compressor.cc:75-137
Status CompressorLZ4::Uncompress(char* source, uint64_t size_source_total, char** dest, uint64_t* size_dest,
                                 char** frame_out, uint64_t* size_frame_out, bool do_memory_allocation) {
  uint64_t offset_uncompress = ts_uncompress_.get();
  if (do_memory_allocation) *dest = nullptr;
  if (offset_uncompress == size_source_total) return Status::Done();

  uint32_t size_compressed = get_u32le(source + offset_uncompress);
  uint32_t size_source = get_u32le(source + offset_uncompress + 4);

  if (size_compressed > 0) {
    size_compressed -= 8;
    *size_dest = 0;
    if (do_memory_allocation) *dest = new char[size_source];
    int size = (int)size_compressed;
    int ret = kdb_lz4_decompress_safe_partial(source + offset_uncompress + 8, *dest, size, (int)size_source,
                                              (int)size_source);
    if (ret <= 0) {
      if (do_memory_allocation) {
        delete[] * dest;
        *dest = nullptr;
      }
      return Status::IOError("LZ4_decompress_safe_partial() failed");
    }
    *size_dest = (uint64_t)ret;
  } else {
    size_compressed = size_source;
    *size_dest = size_source;
    if (do_memory_allocation) *dest = new char[size_source];
    memcpy(*dest, source + offset_uncompress + 8, size_source);
  }

  crc32_.stream(source + offset_uncompress, (size_t)size_compressed + 8);  // compressor.cc:126
  *frame_out = source + offset_uncompress;
  *size_frame_out = (uint64_t)size_compressed + 8;
  offset_uncompress += (uint64_t)size_compressed + 8;
  ts_uncompress_.put(offset_uncompress);
  return Status::OK();
}

// compressor.cc:140-249
Status CompressorLZ4::UncompressByteArray(ByteArray& value, bool do_checksum_verification,
                                          ByteArray* value_uncompressed) {
  if (do_checksum_verification) {
    crc32_.ResetThreadLocalStorage();
    crc32_.put(value.checksum_initial());
  }
  bool is_compressed = value.is_compressed();
  bool is_compression_disabled = false;
  uint64_t offset_in = 0;
  uint64_t offset_out = 0;
  ResetThreadLocalStorage();

  *value_uncompressed = ByteArray::NewAllocatedMemoryByteArray(value.size());
  value_uncompressed->set_size(value.size());
  value_uncompressed->set_size_compressed(0);

  while (true) {
    if (is_compressed && !is_compression_disabled) {
      if (IsUncompressionDone(value.size_compressed())) {
        if (!do_checksum_verification || crc32_.get() == value.checksum()) return Status::OK();
        return Status::IOError("Invalid checksum.");
      }
      if (HasFrameHeaderDisabledCompression(value.data() + offset_in)) {
        is_compression_disabled = true;
        if (do_checksum_verification) crc32_.stream(value.data() + offset_in, size_frame_header());
        offset_in += size_frame_header();
      }
      if (!is_compression_disabled) {
        char* frame;
        uint64_t size_frame;
        uint64_t size_out;
        char* buffer_out = value_uncompressed->data() + offset_out;
        const uint32_t crc_before = crc32_.get();
        Status s = Uncompress(value.data(), value.size_compressed(), &buffer_out, &size_out, &frame, &size_frame,
                              false);
        if (s.IsDone()) return Status::OK();
        if (!s.IsOK()) return s;
        if (do_checksum_verification) {
          if (crc_double_stream_) {
            crc32_.stream(frame, size_frame);  // compressor.cc:202 (second pass: reference quirk)
          } else {
            (void)crc_before;  // Uncompress already streamed this frame exactly once
          }
        }
        offset_in += size_frame;
        offset_out += size_out;
      }
    }
    if (!is_compressed || is_compression_disabled) {
      uint64_t size_left = (is_compressed && is_compression_disabled) ? value.size_compressed() : value.size();
      if (offset_in == size_left) return Status::OK();
      char* data_left = value.data() + offset_in;
      const uint64_t step = 1024 * 1024;
      uint64_t size_current = offset_in + step < size_left ? step : size_left - offset_in;
      if (do_checksum_verification) crc32_.stream(data_left, size_current);
      memcpy(value_uncompressed->data() + offset_out, data_left, size_current);
      offset_in += size_current;
      offset_out += size_current;
      return Status::OK();
    }
  }
}

// ---------------------------------------------------------------- batches
namespace {
// Per-thread staging of the batch methods: pinned host and device buffers
// that grow on demand and are kept across calls (an allocation per call cost
// milliseconds: hipHostMalloc/hipMalloc of the whole batch), plus a stream.
struct BatchStaging {
  void* host = nullptr;
  void* dev = nullptr;
  void* stream = nullptr;
  uint64_t cap = 0;
  int device = -1;
  ~BatchStaging() { release(); }
  void release() {
    if (host) kdb_lz4_host_free(host);
    if (dev) kdb_lz4_free(dev);
    if (stream) kdb_lz4_stream_destroy(stream);
    host = dev = stream = nullptr;
    cap = 0;
  }
  // After a failed call: wait for whatever the stream still has queued; if
  // even that fails, forget the buffers (leaked, not freed: a kernel may still
  // write them) so the next call allocates fresh ones.
  void drain_or_drop() {
    if (stream && kdb_lz4_stream_sync(stream) == KDB_LZ4_OK) return;
    host = dev = stream = nullptr;
    cap = 0;
  }
  bool reserve(uint64_t bytes) {
    int d = 0;
    if (kdb_lz4_get_device(&d) != KDB_LZ4_OK) return false;
    if (d != device) {           // buffers and stream belong to one device
      release();
      device = d;
    }
    if (!stream && kdb_lz4_stream_create(&stream) != KDB_LZ4_OK) return false;
    if (bytes <= cap) return true;
    uint64_t want = cap ? cap : (1ull << 20);
    while (want < bytes) want *= 2;
    if (host) kdb_lz4_host_free(host);
    if (dev) kdb_lz4_free(dev);
    host = dev = nullptr;
    cap = 0;
    if (kdb_lz4_host_alloc(&host, want) != KDB_LZ4_OK || kdb_lz4_malloc(&dev, want) != KDB_LZ4_OK) return false;
    cap = want;
    return true;
  }
};
BatchStaging& batch_staging() {
  thread_local BatchStaging s;
  return s;
}
inline uint64_t a16(uint64_t x) { return (x + 15) & ~uint64_t(15); }
}  // namespace

Status CompressorLZ4::CompressFrames(uint32_t n, char* const* raw_in, const uint64_t* size_raw_in, char** frames,
                                     uint64_t* frame_sizes) {
  if (n == 0) return Status::OK();
  // layout: [src_off n][src_len n][dst_off n][frame_len n][status n] | src | dst
  uint64_t meta = a16(n * (8 + 4 + 8 + 4 + 4));
  uint64_t src_bytes = 0, dst_bytes = 0;
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (size_raw_in[i] > 0xFFFFFFFFull) return Status::InvalidArgument("value too large");
    src_bytes += a16(size_raw_in[i]);
    dst_bytes += a16(kdb_lz4_frame_bound((uint32_t)size_raw_in[i]));
    if (size_raw_in[i] > max_len) max_len = (uint32_t)size_raw_in[i];
  }
  BatchStaging& b = batch_staging();
  if (!b.reserve(meta + src_bytes + dst_bytes)) return Status::IOError("GPU allocation failed");
  char* hb = static_cast<char*>(b.host);
  uint64_t* src_off = reinterpret_cast<uint64_t*>(hb);
  uint32_t* src_len = reinterpret_cast<uint32_t*>(hb + 8ull * n);
  uint64_t* dst_off = reinterpret_cast<uint64_t*>(hb + 12ull * n);
  uint32_t* frame_len = reinterpret_cast<uint32_t*>(hb + 20ull * n);
  int32_t* status = reinterpret_cast<int32_t*>(hb + 24ull * n);
  uint64_t so = meta, dof = meta + src_bytes;
  for (uint32_t i = 0; i < n; i++) {
    src_off[i] = so;
    src_len[i] = (uint32_t)size_raw_in[i];
    memcpy(hb + so, raw_in[i], size_raw_in[i]);
    so += a16(size_raw_in[i]);
    dst_off[i] = dof;
    dof += a16(kdb_lz4_frame_bound((uint32_t)size_raw_in[i]));
  }
  char* db = static_cast<char*>(b.dev);
  void* st = b.stream;
  int rc = kdb_lz4_memcpy_h2d(db, hb, meta + src_bytes, st);
  if (!rc)
    rc = kdb_lz4_compress_frames_batch(st, reinterpret_cast<uint8_t*>(db), reinterpret_cast<uint64_t*>(db),
                                       reinterpret_cast<uint32_t*>(db + 8ull * n), n, max_len,
                                       reinterpret_cast<uint8_t*>(db), reinterpret_cast<uint64_t*>(db + 12ull * n),
                                       reinterpret_cast<uint32_t*>(db + 20ull * n),
                                       reinterpret_cast<int32_t*>(db + 24ull * n));
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb, db, meta, st);
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb + meta + src_bytes, db + meta + src_bytes, dst_bytes, st);
  if (!rc) rc = kdb_lz4_stream_sync(st);
  if (rc) {
    b.drain_or_drop();   // nothing queued may still write the staging the next call reuses
    return Status::IOError("GPU compress batch failed");
  }
  for (uint32_t i = 0; i < n; i++) {
    if (status[i] != 0) {
      for (uint32_t j = 0; j < i; j++) {
        delete[] frames[j];
        frames[j] = nullptr;
      }
      return Status::IOError("LZ4_compress_limitedOutput() failed", std::to_string(i));
    }
    frames[i] = new char[frame_len[i]];
    memcpy(frames[i], hb + dst_off[i], frame_len[i]);
    frame_sizes[i] = frame_len[i];
  }
  return Status::OK();
}

Status CompressorLZ4::UncompressFrames(uint32_t n, char* const* frames, const uint64_t* frame_avail,
                                       char* const* out, const uint64_t* out_cap, uint64_t* size_out) {
  if (n == 0) return Status::OK();
  // layout: [src_off][avail][dst_off][dst_cap][out_len][status] | src | dst
  uint64_t meta = a16(n * (8 + 4 + 8 + 4 + 4 + 4));
  uint64_t src_bytes = 0, dst_bytes = 0;
  uint32_t max_in = 0, max_out = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (frame_avail[i] < 8 || frame_avail[i] > 0xFFFFFFFFull || out_cap[i] > 0xFFFFFFFFull)
      return Status::InvalidArgument("frame size");
    src_bytes += a16(frame_avail[i]);
    dst_bytes += a16(out_cap[i]);
    if (frame_avail[i] > max_in) max_in = (uint32_t)frame_avail[i];
    if (out_cap[i] > max_out) max_out = (uint32_t)out_cap[i];
  }
  BatchStaging& b = batch_staging();
  if (!b.reserve(meta + src_bytes + dst_bytes)) return Status::IOError("GPU allocation failed");
  char* hb = static_cast<char*>(b.host);
  uint64_t* src_off = reinterpret_cast<uint64_t*>(hb);
  uint32_t* avail = reinterpret_cast<uint32_t*>(hb + 8ull * n);
  uint64_t* dst_off = reinterpret_cast<uint64_t*>(hb + 12ull * n);
  uint32_t* dst_cap = reinterpret_cast<uint32_t*>(hb + 20ull * n);
  uint32_t* out_len = reinterpret_cast<uint32_t*>(hb + 24ull * n);
  int32_t* status = reinterpret_cast<int32_t*>(hb + 28ull * n);
  uint64_t so = meta, dof = meta + src_bytes;
  for (uint32_t i = 0; i < n; i++) {
    src_off[i] = so;
    avail[i] = (uint32_t)frame_avail[i];
    memcpy(hb + so, frames[i], frame_avail[i]);
    so += a16(frame_avail[i]);
    dst_off[i] = dof;
    dst_cap[i] = (uint32_t)out_cap[i];
    dof += a16(out_cap[i]);
  }
  char* db = static_cast<char*>(b.dev);
  void* st = b.stream;
  int rc = kdb_lz4_memcpy_h2d(db, hb, meta + src_bytes, st);
  if (!rc)
    rc = kdb_lz4_decompress_frames_batch(
        st, reinterpret_cast<uint8_t*>(db), reinterpret_cast<uint64_t*>(db), reinterpret_cast<uint32_t*>(db + 8ull * n),
        n, max_in, max_out, reinterpret_cast<uint8_t*>(db), reinterpret_cast<uint64_t*>(db + 12ull * n),
        reinterpret_cast<uint32_t*>(db + 20ull * n), reinterpret_cast<uint32_t*>(db + 24ull * n),
        reinterpret_cast<int32_t*>(db + 28ull * n));
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb, db, meta, st);
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb + meta + src_bytes, db + meta + src_bytes, dst_bytes, st);
  if (!rc) rc = kdb_lz4_stream_sync(st);
  if (rc) {
    b.drain_or_drop();
    return Status::IOError("GPU decompress batch failed");
  }
  for (uint32_t i = 0; i < n; i++) {
    if (status[i] != 0) return Status::IOError("LZ4_decompress_safe_partial() failed", std::to_string(i));
    memcpy(out[i], hb + dst_off[i], out_len[i]);
    size_out[i] = out_len[i];
  }
  return Status::OK();
}

KDB_LZ4_NS_CLOSE  // namespace kdb
