// kingdb_amd/csrc/hstable.cc -- host side of the GPU write path: cuts the
// dense entry stream that put.hip produces into HSTable files, byte for byte
// what KingDB's HSTableManager writes for the same put stream.
//
//   OpenNewFile              storage/hstable_manager.h:260-290 (file ids and
//                            timestamps count from 1; 8 KiB header block:
//                            HSTableHeader + DatabaseOptionEncoder, format.h:324-425)
//   WriteOrdersAndFlushFile  hstable_manager.h:714-847 (a file is closed before
//                            an order once offset_end_ > size_block_, after a
//                            multipart first part / at the end of a batch once
//                            offset_end_ >= size_block_ -- FlushCurrentFile 312-359)
//   WriteOffsetArray         hstable_manager.h:380-420 (varint64 hash, varint32
//                            offset per entry; HSTableFooter format.h:480-493;
//                            CRC32C of rows + footer)
// A file holding a multipart entry whose last part never registered
// (put.hip kind 2) keeps no offset array, as in the reference
// (FlushOffsetArray, hstable_manager.h:361-378: writes in progress).
//
// The entry bytes themselves are GPU output; this file only does the
// per-file framing (tens of bytes per file plus ~12 bytes per entry).
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <memory>
#include <thread>
#include <string>
#include <vector>

#include "../../include/kdb_put.h"

namespace {

constexpr uint64_t kHeaderSize = 8192;        // internal__hstable_header_size (util/options.h:43)
constexpr uint64_t kMagic = 0x4D454F57;       // hstable_manager.h:1215

// crc32c::Value (crc32c.cc:296-340) over the file header and the offset
// array: slice-by-8 tables (the offset array is ~12 bytes per entry).
struct CrcTab {
  uint32_t t[8][256];
  CrcTab() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
      for (int k = 1; k < 8; k++) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xffu];
  }
};
const CrcTab kTab;
#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n) {   // same polynomial
  uint64_t l = 0xFFFFFFFFu;
  for (; n >= 8; n -= 8, p += 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    l = __builtin_ia32_crc32di(l, w);
  }
  uint32_t c = (uint32_t)l;
  for (; n; n--) c = __builtin_ia32_crc32qi(c, *p++);
  return c ^ 0xFFFFFFFFu;
}
const bool kHwCrc = __builtin_cpu_supports("sse4.2");
#endif
uint32_t crc32c(const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (kHwCrc) return crc32c_hw(p, n);
#endif
  uint32_t l = 0xFFFFFFFFu;
  for (; n >= 8; n -= 8, p += 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    w ^= l;
    l = kTab.t[7][w & 0xff] ^ kTab.t[6][(w >> 8) & 0xff] ^ kTab.t[5][(w >> 16) & 0xff] ^ kTab.t[4][(w >> 24) & 0xff] ^
        kTab.t[3][(w >> 32) & 0xff] ^ kTab.t[2][(w >> 40) & 0xff] ^ kTab.t[1][(w >> 48) & 0xff] ^ kTab.t[0][w >> 56];
  }
  for (; n; n--) l = kTab.t[0][(l ^ *p++) & 0xffu] ^ (l >> 8);
  return l ^ 0xFFFFFFFFu;
}

void put32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i)); }
void put64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }
size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 128) { v >>= 7; n++; }
  return n;
}
uint8_t* varint(uint8_t* p, uint64_t v) {
  while (v >= 128) { *p++ = (uint8_t)(v | 128); v >>= 7; }
  *p++ = (uint8_t)v;
  return p;
}

// DatabaseOptionEncoder::EncodeTo (format.h:324-340): version 0.9.0.0, data
// format 1.0, hstable size, hash, compression LZ4 (1), checksum CRC32C (1).
void db_options(uint64_t hstable_size, uint32_t hash_type, uint8_t* b) {
  const uint32_t w[6] = {0, 9, 0, 0, 1, 0};
  for (int i = 0; i < 6; i++) put32(b + 4 + 4 * i, w[i]);
  put64(b + 28, hstable_size);
  put32(b + 36, hash_type);
  put32(b + 40, 1);
  put32(b + 44, 1);
  put32(b, crc32c(b + 4, 44));
}

// A growable byte buffer that does not zero what it is about to overwrite
// (std::vector::resize would: a second pass over every entry byte).
struct Buf {
  std::unique_ptr<uint8_t[]> p;
  size_t cap = 0, n = 0;
  void reserve(size_t c) {
    if (c <= cap) return;
    std::unique_ptr<uint8_t[]> q(new uint8_t[c]);
    if (n) memcpy(q.get(), p.get(), n);
    p = std::move(q);
    cap = c;
  }
  void append(const void* src, size_t len) {
    if (n + len > cap) reserve(std::max(n + len, cap * 2));
    uint8_t* d = p.get() + n;
    const uint8_t* s = static_cast<const uint8_t*>(src);
    // large runs (a chunk's worth of entries) are copied by a few threads:
    // one core's memcpy is the host side's bottleneck otherwise
    constexpr size_t kPiece = 2u << 20;
    const size_t pieces = std::min<size_t>(len / kPiece, 8);
    if (pieces >= 2) {
      const size_t step = (len / pieces + 63) & ~(size_t)63;
      std::vector<std::thread> th;
      for (size_t k = 1; k < pieces; k++) {
        const size_t a = k * step, b = std::min(len, a + step);
        if (a < b) th.emplace_back([=] { memcpy(d + a, s + a, b - a); });
      }
      memcpy(d, s, std::min(len, step));
      for (auto& t : th) t.join();
    } else {
      memcpy(d, s, len);
    }
    n += len;
  }
  size_t size() const { return n; }
  uint8_t* data() { return p.get(); }
  const uint8_t* data() const { return p.get(); }
};

}  // namespace

struct kdb_hstable_writer {
  uint64_t size_block;
  uint32_t hash_type;
  uint32_t fileid = 0;
  uint64_t timestamp = 0;
  bool open = false;
  Buf cur;                                  // the open file's bytes (== offset_end_)
  std::vector<std::pair<uint64_t, uint32_t>> offarray;
  bool padding_flag = false, incomplete = false;
  std::vector<std::pair<uint32_t, Buf>> files;   // closed files
  std::vector<Buf> spare;                   // buffers of files dropped by reset(), reused

  void open_file() {                        // OpenNewFile
    fileid++;
    timestamp++;
    if (!spare.empty()) {
      cur = std::move(spare.back());
      spare.pop_back();
    }
    cur.reserve(size_block + size_block / 8 * 5 + (1u << 20));   // + offset array (<= 15 B per >= 26 B entry)
    cur.n = 0;
    uint8_t hb[kHeaderSize] = {0};
    cur.append(hb, kHeaderSize);
    uint8_t* b = cur.data();
    put32(b + 4, 1);                        // data format 1.0 (format.h:28-29)
    put32(b + 8, 0);
    put32(b + 12, 1);                       // kUncompactedRegularType
    put64(b + 16, timestamp);
    put32(b, crc32c(b + 4, 20));
    db_options(size_block, hash_type, b + 24);
    offarray.clear();
    offarray.reserve(size_block / 64);
    padding_flag = incomplete = false;
    open = true;
  }
  void close_file() {                       // CloseCurrentFile -> FlushOffsetArray
    if (!open) return;
    if (!incomplete) {
      // OffsetArrayRow::EncodeTo per entry (varint64 hash, varint32 offset), then the footer
      const size_t start = cur.size();
      cur.reserve(start + offarray.size() * 15 + 36);
      uint8_t* q = cur.data() + start;
      const size_t rows = offarray.size();
      const size_t T = std::min<size_t>(8, rows / 16384 + 1);
      if (T == 1) {
        for (auto& r : offarray) {
          q = varint(q, r.first);
          q = varint(q, r.second);
        }
      } else {                              // rows encoded by T threads into their byte ranges
        std::vector<size_t> lo(T + 1), bytes(T + 1, 0);
        for (size_t k = 0; k <= T; k++) lo[k] = rows * k / T;
        auto each = [&](auto&& fn) {
          std::vector<std::thread> th;
          for (size_t k = 1; k < T; k++) th.emplace_back(fn, k);
          fn(0);
          for (auto& t : th) t.join();
        };
        each([&](size_t k) {
          size_t b = 0;
          for (size_t i = lo[k]; i < lo[k + 1]; i++) b += varint_len(offarray[i].first) + varint_len(offarray[i].second);
          bytes[k + 1] = b;
        });
        for (size_t k = 1; k <= T; k++) bytes[k] += bytes[k - 1];
        each([&](size_t k) {
          uint8_t* o = q + bytes[k];
          for (size_t i = lo[k]; i < lo[k + 1]; i++) {
            o = varint(o, offarray[i].first);
            o = varint(o, offarray[i].second);
          }
        });
        q += bytes[T];
      }
      put32(q, 1);
      put32(q + 4, padding_flag ? 1u : 0u);
      put64(q + 8, start);
      put64(q + 16, offarray.size());
      put64(q + 24, kMagic);
      q += 32;
      put32(q, crc32c(cur.data() + start, (size_t)(q - (cur.data() + start))));
      cur.n = (size_t)(q + 4 - cur.data());
    }
    files.emplace_back(fileid, std::move(cur));
    cur = Buf();
    open = false;
  }
};

extern "C" {

int kdb_hstable_db_options(uint64_t hstable_size, uint32_t hash_type, uint8_t* out48) {
  if (!out48 || hash_type > 1) return KDB_PUT_EINVAL;
  db_options(hstable_size, hash_type, out48);
  return KDB_PUT_OK;
}

int kdb_hstable_writer_create(uint64_t hstable_size, uint32_t hash_type, kdb_hstable_writer** w) {
  if (!w || hash_type > 1 || hstable_size <= kHeaderSize) return KDB_PUT_EINVAL;
  *w = new kdb_hstable_writer{hstable_size, hash_type};
  return KDB_PUT_OK;
}

int kdb_hstable_writer_append(kdb_hstable_writer* w, const uint8_t* entries, const uint64_t* entry_off,
                              const uint32_t* entry_len, const uint64_t* hashed, const uint32_t* kind,
                              const int32_t* status, uint32_t n) {
  if (!w || (n && (!entries || !entry_off || !entry_len || !hashed || !kind || !status))) return KDB_PUT_EINVAL;
  // Entries are appended in runs: consecutive entries of one file are one
  // memcpy (the dense stream holds them back to back).
  uint64_t fsize = w->cur.size();           // offset_end_ of the open file, run included
  const uint8_t* run = nullptr;
  uint64_t run_len = 0;
  auto flush_run = [&]() {
    if (run_len) w->cur.append(run, run_len);
    run = nullptr;
    run_len = 0;
  };
  auto close = [&]() {
    flush_run();
    w->close_file();
    fsize = 0;
  };
  for (uint32_t i = 0; i < n; i++) {
    if (status[i] != 0) continue;           // the reference returned IOError: no order
    if (w->open && fsize > w->size_block) close();                    // FlushCurrentFile(true, 0)
    if (!w->open) {
      w->open_file();
      fsize = w->cur.size();
    }
    if (fsize > 0xFFFFFFFFull) return KDB_PUT_EINVAL;
    w->offarray.emplace_back(hashed[i], (uint32_t)fsize);
    const uint8_t* e = entries + entry_off[i];
    if (run_len && run + run_len != e) flush_run();
    if (!run_len) run = e;
    run_len += entry_len[i];
    fsize += entry_len[i];
    if (kind[i] != 0) {                     // multipart first part: FlushCurrentFile(0, padding)
      w->padding_flag = true;
      if (kind[i] == 2) w->incomplete = true;
      if (fsize >= w->size_block) close();
    }
  }
  flush_run();
  if (w->open && w->cur.size() >= w->size_block) w->close_file();    // end of batch: FlushCurrentFile(0, 0)
  return KDB_PUT_OK;
}

int kdb_hstable_writer_close(kdb_hstable_writer* w) {
  if (!w) return KDB_PUT_EINVAL;
  w->close_file();
  return KDB_PUT_OK;
}

int kdb_hstable_writer_file_count(const kdb_hstable_writer* w, uint32_t* count) {
  if (!w || !count) return KDB_PUT_EINVAL;
  *count = (uint32_t)w->files.size();
  return KDB_PUT_OK;
}

int kdb_hstable_writer_file(const kdb_hstable_writer* w, uint32_t i, uint32_t* fileid, const uint8_t** data,
                            uint64_t* size) {
  if (!w || i >= w->files.size() || !fileid || !data || !size) return KDB_PUT_EINVAL;
  *fileid = w->files[i].first;
  *data = w->files[i].second.data();
  *size = w->files[i].second.size();
  return KDB_PUT_OK;
}

int kdb_hstable_writer_save(const kdb_hstable_writer* w, const char* dir) {
  if (!w || !dir) return KDB_PUT_EINVAL;
  for (auto& f : w->files) {
    char name[64];
    snprintf(name, sizeof(name), "/%08x", f.first);      // HSTableManager::GetFilepath
    FILE* fp = fopen((std::string(dir) + name).c_str(), "wb");
    if (!fp) return KDB_PUT_EIO;
    const bool ok = fwrite(f.second.data(), 1, f.second.size(), fp) == f.second.size();
    if (fclose(fp) != 0 || !ok) return KDB_PUT_EIO;
  }
  return KDB_PUT_OK;
}

int kdb_hstable_writer_reset(kdb_hstable_writer* w) {
  if (!w) return KDB_PUT_EINVAL;
  for (auto& f : w->files) w->spare.push_back(std::move(f.second));
  w->files.clear();
  if (w->open) w->spare.push_back(std::move(w->cur));
  w->cur = Buf();
  w->offarray.clear();
  w->open = w->padding_flag = w->incomplete = false;
  w->fileid = 0;
  w->timestamp = 0;
  return KDB_PUT_OK;
}

int kdb_hstable_writer_destroy(kdb_hstable_writer* w) {
  delete w;
  return KDB_PUT_OK;
}

}  // extern "C"
