// kingdb_amd/csrc/kdb_types.h -- the parts of KingDB's util/ types that the
// CompressorLZ4 drop-in's signatures name, for builds OUTSIDE a KingDB tree.
//
// Inside KingDB (define KDB_LZ4_IN_KINGDB) the real headers are used instead:
// util/status.h (Status, status.h:20-85) and util/byte_array.h (ByteArray,
// byte_array.h:182-298).  These mirrors keep the same names, codes and the
// members CompressorLZ4 touches, so the drop-in compiles identically in both.
//
// The mirrors live in the inline namespace kdb::standalone (and so does the
// standalone CompressorLZ4, compressor.h): source still says kdb::Status,
// but the mangled names differ from KingDB's, so an object built against the
// mirrors can never be linked into a KingDB build by mistake -- the link
// fails instead of two ByteArray layouts meeting at run time.
#pragma once

#ifdef KDB_LZ4_IN_KINGDB
#include "util/byte_array.h"
#include "util/status.h"
#else

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>

namespace kdb {
inline namespace standalone {

// util/status.h:20-85 (codes status.h:72-79).
class Status {
 public:
  Status() : code_(kOK) {}
  explicit Status(int code) : code_(code) {}
  Status(int code, std::string m1, std::string m2) : code_(code), message1_(std::move(m1)), message2_(std::move(m2)) {}
  static Status OK() { return Status(); }
  static Status Done() { return Status(kDone); }
  static Status MultipartRequired() { return Status(kMultipartRequired); }
  static Status NotFound(const std::string& a, const std::string& b = "") { return Status(kNotFound, a, b); }
  static Status InvalidArgument(const std::string& a, const std::string& b = "") {
    return Status(kInvalidArgument, a, b);
  }
  static Status IOError(const std::string& a, const std::string& b = "") { return Status(kIOError, a, b); }
  bool IsOK() const { return code_ == kOK; }
  bool IsNotFound() const { return code_ == kNotFound; }
  bool IsInvalidArgument() const { return code_ == kInvalidArgument; }
  bool IsIOError() const { return code_ == kIOError; }
  bool IsDone() const { return code_ == kDone; }
  bool IsMultipartRequired() const { return code_ == kMultipartRequired; }
  int code() const { return code_; }
  std::string ToString() const {
    static const char* names[] = {"OK", "Not found: ", "Delete order", "Invalid argument: ", "IO error: ",
                                  "Done", "Multipart required"};
    std::string r = (code_ >= 0 && code_ <= 6) ? names[code_] : "Unknown code";
    if (code_ == kNotFound || code_ == kInvalidArgument || code_ == kIOError) {
      r += message1_;
      if (!message2_.empty()) r += ": " + message2_;
    }
    return r;
  }
  enum Code { kOK = 0, kNotFound = 1, kDeleteOrder = 2, kInvalidArgument = 3, kIOError = 4, kDone = 5,
              kMultipartRequired = 6 };

 private:
  int code_;
  std::string message1_, message2_;
};

// util/byte_array.h:182-298: a view (data, size, offset) over a shared
// resource, plus the compressed size and the two checksums the read path sets
// (storage_engine.h:497-508).  Only the allocation kinds the codec path
// creates are mirrored: allocated (owned new[]), shallow copy (takes a new[]
// buffer), deep copy and pointer (borrowed).
class ByteArray {
 public:
  ByteArray() = default;
  char* data() { return buf_ ? buf_.get() + offset_ : const_cast<char*>(borrowed_) + offset_; }
  const char* data_const() const { return buf_ ? buf_.get() + offset_ : borrowed_ + offset_; }
  uint64_t size() const { return size_; }
  uint64_t size_compressed() const { return size_compressed_; }
  void set_size(uint64_t s) { size_ = s; }
  void set_size_compressed(uint64_t s) { size_compressed_ = s; }
  uint64_t is_compressed() const { return size_compressed_ != 0; }
  void set_offset(uint64_t o) { offset_ = o; }
  void increment_offset(uint64_t i) { offset_ += i; }
  uint32_t checksum() const { return checksum_; }
  uint32_t checksum_initial() const { return checksum_initial_; }
  void set_checksum(uint32_t c) { checksum_ = c; }
  void set_checksum_initial(uint32_t c) { checksum_initial_ = c; }
  std::string ToString() const { return std::string(data_const(), size_); }

  static ByteArray NewAllocatedMemoryByteArray(uint64_t size) {
    ByteArray b;
    b.buf_ = std::shared_ptr<char>(new char[size ? size : 1], std::default_delete<char[]>());
    b.size_ = size;
    return b;
  }
  static ByteArray NewShallowCopyByteArray(char* data, uint64_t size) {  // takes ownership of new[]
    ByteArray b;
    b.buf_ = std::shared_ptr<char>(data, std::default_delete<char[]>());
    b.size_ = size;
    return b;
  }
  static ByteArray NewDeepCopyByteArray(const char* data, uint64_t size) {
    ByteArray b = NewAllocatedMemoryByteArray(size);
    if (size) memcpy(b.buf_.get(), data, size);
    return b;
  }
  static ByteArray NewPointerByteArray(const char* data, uint64_t size) {
    ByteArray b;
    b.borrowed_ = data;
    b.size_ = size;
    return b;
  }

 private:
  std::shared_ptr<char> buf_;
  const char* borrowed_ = nullptr;
  uint64_t size_ = 0, size_compressed_ = 0, offset_ = 0;
  uint32_t checksum_ = 0, checksum_initial_ = 0;
};

inline ByteArray NewShallowCopyByteArray(char* data, uint64_t size) {
  return ByteArray::NewShallowCopyByteArray(data, size);
}

}  // namespace standalone
}  // namespace kdb
#endif  // KDB_LZ4_IN_KINGDB
