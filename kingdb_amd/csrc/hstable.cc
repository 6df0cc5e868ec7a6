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
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kdb_put.h"

namespace {

constexpr uint64_t kHeaderSize = 8192;        // internal__hstable_header_size (util/options.h:43)
constexpr uint64_t kMagic = 0x4D454F57;       // hstable_manager.h:1215

uint32_t crc_table[256];
bool crc_ready = false;
uint32_t crc32c(const uint8_t* p, size_t n) {   // crc32c::Value (crc32c.cc:296-340)
  if (!crc_ready) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      crc_table[i] = c;
    }
    crc_ready = true;
  }
  uint32_t l = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) l = crc_table[(l ^ p[i]) & 0xffu] ^ (l >> 8);
  return l ^ 0xFFFFFFFFu;
}

void put32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i)); }
void put64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }
void put_varint(std::vector<uint8_t>& o, uint64_t v) {
  while (v >= 128) { o.push_back((uint8_t)(v | 128)); v >>= 7; }
  o.push_back((uint8_t)v);
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

}  // namespace

struct kdb_hstable_writer {
  uint64_t size_block;
  uint32_t hash_type;
  uint32_t fileid = 0;
  uint64_t timestamp = 0;
  bool open = false;
  std::vector<uint8_t> cur;                 // the open file's bytes (== offset_end_)
  std::vector<std::pair<uint64_t, uint32_t>> offarray;
  bool padding_flag = false, incomplete = false;
  std::vector<std::pair<uint32_t, std::vector<uint8_t>>> files;   // closed files

  void open_file() {                        // OpenNewFile
    fileid++;
    timestamp++;
    cur.assign(kHeaderSize, 0);
    uint8_t* b = cur.data();
    put32(b + 4, 1);                        // data format 1.0 (format.h:28-29)
    put32(b + 8, 0);
    put32(b + 12, 1);                       // kUncompactedRegularType
    put64(b + 16, timestamp);
    put32(b, crc32c(b + 4, 20));
    db_options(size_block, hash_type, b + 24);
    offarray.clear();
    padding_flag = incomplete = false;
    open = true;
  }
  void close_file() {                       // CloseCurrentFile -> FlushOffsetArray
    if (!open) return;
    if (!incomplete) {
      std::vector<uint8_t> tail;
      tail.reserve(offarray.size() * 14 + 36);
      for (auto& r : offarray) {
        put_varint(tail, r.first);
        put_varint(tail, r.second);
      }
      uint8_t f[36];
      put32(f, 1);
      put32(f + 4, padding_flag ? 1u : 0u);
      put64(f + 8, cur.size());
      put64(f + 16, offarray.size());
      put64(f + 24, kMagic);
      tail.insert(tail.end(), f, f + 32);
      uint8_t c[4];
      put32(c, crc32c(tail.data(), tail.size()));
      tail.insert(tail.end(), c, c + 4);
      cur.insert(cur.end(), tail.begin(), tail.end());
    }
    files.emplace_back(fileid, std::move(cur));
    cur.clear();
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
  for (uint32_t i = 0; i < n; i++) {
    if (status[i] != 0) continue;           // the reference returned IOError: no order
    if (w->open && w->cur.size() > w->size_block) w->close_file();    // FlushCurrentFile(true, 0)
    if (!w->open) w->open_file();
    const uint64_t off = w->cur.size();
    if (off > 0xFFFFFFFFull) return KDB_PUT_EINVAL;
    w->offarray.emplace_back(hashed[i], (uint32_t)off);
    w->cur.insert(w->cur.end(), entries + entry_off[i], entries + entry_off[i] + entry_len[i]);
    if (kind[i] != 0) {                     // multipart first part: FlushCurrentFile(0, padding)
      w->padding_flag = true;
      if (kind[i] == 2) w->incomplete = true;
      if (w->cur.size() >= w->size_block) w->close_file();
    }
  }
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

int kdb_hstable_writer_destroy(kdb_hstable_writer* w) {
  delete w;
  return KDB_PUT_OK;
}

}  // extern "C"
