// kingdb_amd/csrc/compressor.h -- drop-in replacement for KingDB's CompressorLZ4
// (/root/reference/algorithm/compressor.h:102-176).
//
// Same class name, namespace, public methods, frame format, Status codes and
// buffer-ownership rules as the reference; the LZ4 work runs in the gfx950
// kernels through include/kdb_lz4.h.  Per-thread stream state (the reference's
// ThreadStorage, thread/threadstorage.h:23-46) is kept per (instance, thread).
//
// Added (not replacing): CompressFrames / UncompressFrames, which move a whole
// batch of values through one H2D copy, one kernel launch and one D2H copy.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "kdb_types.h"

// Outside KingDB the class sits in the inline namespace kdb::standalone with
// the type mirrors (kdb_types.h); inside (KDB_LZ4_IN_KINGDB, set by
// kingdb_amd/kingdb_include/algorithm/compressor.h and by the build of this
// file for KingDB) it is kdb::CompressorLZ4 itself, the friend that
// util/byte_array.h names.
#ifdef KDB_LZ4_IN_KINGDB
#define KDB_LZ4_NS_OPEN namespace kdb {
#define KDB_LZ4_NS_CLOSE }
#else
#define KDB_LZ4_NS_OPEN namespace kdb { inline namespace standalone {
#define KDB_LZ4_NS_CLOSE } }
#endif

KDB_LZ4_NS_OPEN

// thread/threadstorage.h:23-46: one uint64_t per calling thread, default 0.
class ThreadStorageLZ4 {
 public:
  uint64_t get() {
    std::lock_guard<std::mutex> l(mu_);
    return v_[std::this_thread::get_id()];
  }
  void put(uint64_t x) {
    std::lock_guard<std::mutex> l(mu_);
    v_[std::this_thread::get_id()] = x;
  }
  void reset() { put(0); }

 private:
  std::mutex mu_;
  std::map<std::thread::id, uint64_t> v_;
};

// algorithm/crc32c.h:74-103: CRC32C stream state per thread.
class CRC32LZ4 {
 public:
  void stream(const char* data, size_t n);
  uint32_t get() { return (uint32_t)ts_.get(); }
  void put(uint32_t c) { ts_.put(c); }
  void ResetThreadLocalStorage() { ts_.reset(); }

 private:
  ThreadStorageLZ4 ts_;
};

uint32_t Crc32cExtend(uint32_t crc, const char* data, size_t n);

class CompressorLZ4 {
 public:
  // An instance readies its thread's current device (kdb_lz4_warmup, once per
  // device: the lane-order self-test, the code object, the runtime's
  // first-launch costs), so a Database pays them when it is built, not in its
  // first puts.
  CompressorLZ4() { WarmUp(); }
  // compressor.h:110-113: assignment does not copy state.
  CompressorLZ4& operator=(const CompressorLZ4&) { return *this; }
  virtual ~CompressorLZ4() {}

  void ResetThreadLocalStorage();

  Status Compress(char* raw_in, uint64_t size_raw_in, char** compressed_out, uint64_t* size_compressed_out);

  bool IsUncompressionDone(uint64_t size_source);
  Status Uncompress(char* source, uint64_t size_source, char** dest, uint64_t* size_dest, char** frame_out,
                    uint64_t* size_frame_out, bool do_memory_allocation = true);

  Status UncompressByteArray(ByteArray& value, bool do_checksum_verification, ByteArray* value_uncompressed);

  void DisableCompressionInFrameHeader(char* frame) {
    for (uint64_t i = 0; i < size_frame_header(); i++) frame[i] = 0;
  }
  bool HasFrameHeaderDisabledCompression(char* frame) {
    for (uint64_t i = 0; i < size_frame_header(); i++)
      if (frame[i] != 0) return false;
    return true;
  }
  uint64_t size_compressed() { return ts_compress_.get(); }
  uint64_t MaxInputSize() { return 0x7E000000; }  // LZ4_MAX_INPUT_SIZE, lz4.h:102
  uint64_t size_frame_header() { return 8; }
  uint64_t size_uncompressed_frame(uint64_t size_data) { return size_data + 8; }
  void AdjustCompressedSize(int64_t inc) {
    int64_t size = ts_compress_.get() + inc;
    ts_compress_.put(size);
  }

  // ---- batch additions -------------------------------------------------
  // Compresses n independent values (one frame each) in one GPU launch.
  // frames[i] receives a new[] buffer (caller delete[]s), like Compress().
  // Does not touch the per-thread stream offsets.
  Status CompressFrames(uint32_t n, char* const* raw_in, const uint64_t* size_raw_in, char** frames,
                        uint64_t* frame_sizes);
  // Decodes n single frames in one launch into caller buffers out[i] of
  // out_cap[i] bytes; size_out[i] = *size_dest.  Per-frame failures are
  // reported in the returned Status (first failing index in message).
  Status UncompressFrames(uint32_t n, char* const* frames, const uint64_t* frame_avail, char* const* out,
                          const uint64_t* out_cap, uint64_t* size_out);

  // Bytes [offset, offset + size) of `whole`'s view, sharing its storage.  ByteArray's offset/size setters are private to its
  // friends, this class among them (util/byte_array.h:184-192, 269-276): the
  // flush hook hands each order a slice of one arena per GPU batch instead of
  // a new[] buffer per order.
  static ByteArray Slice(const ByteArray& whole, uint64_t offset, uint64_t size) {
    ByteArray b = whole;
    b.increment_offset(offset);   // relative to whole's own view
    b.set_size(size);
    b.set_size_compressed(0);
    return b;
  }

  // A stored value's fields the read hooks need (private to ByteArray's
  // friends, like Slice): size, size_compressed, checksum, checksum_initial.
  struct StoredView {
    uint64_t size, size_compressed;
    uint32_t checksum, checksum_initial;
  };
  static StoredView View(const ByteArray& v) {
    ByteArray& w = const_cast<ByteArray&>(v);
    return StoredView{w.size(), w.size_compressed(), w.checksum(), w.checksum_initial()};
  }

  // Reference quirk: Uncompress() always streams each frame
  // into crc32_ and UncompressByteArray() streams it again when verifying, so
  // verification of a compressed value fails.  true (default) = bug-for-bug.
  void set_crc_double_stream(bool on) { crc_double_stream_ = on; }

 private:
  ThreadStorageLZ4 ts_compress_;
  ThreadStorageLZ4 ts_uncompress_;
  CRC32LZ4 crc32_;
  bool crc_double_stream_ = true;
  static void WarmUp();
};

KDB_LZ4_NS_CLOSE  // namespace kdb
