// kingdb_amd/csrc/put.hip -- the write path around the codec, on the GPU
// (SURVEY.md §8f rows f1, f2, f4): for a batch of puts, KingDB's per-part
// frame policy, the value CRC32C, the key hash and the HSTable entry encoding,
// so that one launch sequence turns a write-buffer's worth of (key, value)
// pairs into the exact entry bytes HSTableManager appends to its files.
//
// Reference semantics (one client thread, parts of a value sent in order):
//   * Database::PutPartValidSize (interface/database.cc:128-276): per chunk a
//     CompressorLZ4 frame, the disable rule (:196-209: all-zero 8-byte header +
//     raw bytes, raw for every later chunk), offset_chunk_compressed,
//     size_value_compressed (:237-248) and crc32 = CRC32C(key || every
//     chunk_final) (:251-257);
//   * HSTableManager (storage/hstable_manager.h): WriteFirstPartOrSmallOrder
//     (628-712) appends header + key + first chunk and reserves size_value +
//     padding for a multipart value; WriteMiddleOrLastPart (514-626) pwrites
//     each later chunk at its compressed offset and rewrites the header when
//     Order::IsLastPart (util/order.h:52-55) holds -- including the reference's
//     corner cases (a first chunk that already looks "last" makes the entry
//     self-contained and drops later chunks; a last chunk that does not look
//     last leaves the first-part header and no offset array);
//   * EntryHeader::EncodeTo (storage/format.h:224-255), crc32c::crc8
//     (algorithm/crc32c.cc:439-475), XXH64 / MurmurHash3_x64_128 of the key
//     (algorithm/hash.cc:9-23).
//
// Pipeline (stream-ordered; every kernel reads only what earlier ones wrote):
//   put_prep_kernel     thread per value: each part's raw offset and frame slot size
//   scan                frame slot offsets (launch_exclusive_scan, pack.hip)
//   frame compress      the LZ4 kernels over every part (launch_compress)
//   put_policy_kernel   thread per value: the frame policy and the entry layout
//   scan                dense entry offsets
//   put_entry_small_kernel  thread per value, for single-part entries of at most
//                       512 bytes of key + chunk_final: copy, CRC32C, key hash,
//                       EntryHeader bytes
//   put_entry_kernel    wave per value, the rest: key + stored chunks copied into
//                       place, CRC32C (64-lane chunked, GF(2) tree combine), key
//                       hash, EntryHeader bytes
// The host (hstable.cc) then cuts the dense entry stream into HSTable files
// and writes their headers and offset arrays.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/kdb_lz4.h"
#include "crc_device.h"
#include "lz4_device.h"

namespace kdb_lz4 {

hipError_t launch_compress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                           const uint32_t* src_len, uint32_t n, uint32_t min_len, uint32_t max_len, uint8_t* dst,
                           const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                           int32_t* ret);
hipError_t launch_exclusive_scan(hipStream_t st, const uint32_t* len, uint32_t n, uint64_t* off, uint64_t* total);

namespace {

constexpr uint32_t kEntryFull = 0x8, kUncompacted = 0x2, kHasPadding = 0x4;   // format.h:34-42

// ----------------------------------------------------------------- hashes
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// XXH64(p, len, 0) (algorithm/xxhash.cc:427).
constexpr uint64_t XP1 = 11400714785074694791ULL, XP2 = 14029467366897019727ULL, XP3 = 1609587929392839161ULL,
                   XP4 = 9650029242287828579ULL, XP5 = 2870177450012600261ULL;
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * XP2;
  acc = rotl64(acc, 31);
  return acc * XP1;
}
__device__ uint64_t xxh64(const uint8_t* p, uint32_t len) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = XP1 + XP2, v2 = XP2, v3 = 0, v4 = 0 - XP1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xround(v1, ld64(p));
      v2 = xround(v2, ld64(p + 8));
      v3 = xround(v3, ld64(p + 16));
      v4 = xround(v4, ld64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = (h ^ xround(0, v1)) * XP1 + XP4;
    h = (h ^ xround(0, v2)) * XP1 + XP4;
    h = (h ^ xround(0, v3)) * XP1 + XP4;
    h = (h ^ xround(0, v4)) * XP1 + XP4;
  } else {
    h = XP5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xround(0, ld64(p));
    h = rotl64(h, 27) * XP1 + XP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)ld32(p) * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * XP5;
    h = rotl64(h, 11) * XP1;
    p++;
  }
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}

// MurmurHash3_x64_128(p, len, 0), first 8 bytes (murmurhash3.cc:255-330).
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
__device__ uint64_t murmur3_64(const uint8_t* d, uint32_t len) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0, h2 = 0;
  const uint32_t nb = len / 16u;
  for (uint32_t i = 0; i < nb; i++) {
    uint64_t k1 = ld64(d + 16u * i), k2 = ld64(d + 16u * i + 8u);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* t = d + 16u * nb;
  const uint32_t r = len & 15u;
  uint64_t k1 = 0, k2 = 0;
  for (uint32_t i = r; i > 8u; i--) k2 ^= (uint64_t)t[i - 1u] << (8u * (i - 9u));
  if (r > 8u) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
  for (uint32_t i = r < 8u ? r : 8u; i > 0u; i--) k1 ^= (uint64_t)t[i - 1u] << (8u * (i - 1u));
  if (r > 0u) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= (uint64_t)len;
  h2 ^= (uint64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  return h1 + h2;
}

// ----------------------------------------------------------------- CRC-8 of the header
// crc32c::crc8 (crc32c.cc:439-475): reflected, polynomial 0xB2, pre/post xor 0xff.
struct Crc8Table {
  uint8_t t[256];
};
constexpr Crc8Table make_crc8() {
  Crc8Table c{};
  for (unsigned i = 0; i < 256; i++) {
    unsigned v = i;
    for (int k = 0; k < 8; k++) v = (v & 1u) ? (v >> 1) ^ 0xB2u : v >> 1;
    c.t[i] = (uint8_t)v;
  }
  return c;
}
__constant__ Crc8Table kCrc8 = make_crc8();

__host__ __device__ __forceinline__ uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 128) { v >>= 7; n++; }
  return n;
}
__device__ __forceinline__ uint8_t* put_varint(uint8_t* p, uint64_t v) {
  while (v >= 128) { *p++ = (uint8_t)(v | 128); v >>= 7; }
  *p++ = (uint8_t)v;
  return p;
}

__host__ __device__ __forceinline__ uint64_t padding_size(uint64_t size_value) {   // format.h:63-71
  return (size_value / 65536u + 1u) * 8u;
}
// EntryHeader::EncodeTo's size (compression on: fixed64 size_value_compressed).
__host__ __device__ __forceinline__ uint32_t header_len(uint32_t flags, uint64_t klen, uint64_t size_value,
                                                        uint64_t pad) {
  return 1u + 4u + varint_len(flags) + varint_len(klen) + varint_len(size_value) + 8u + varint_len(pad) + 8u;
}

// Part modes (how chunk_final is made from the chunk), plus a flag for chunks
// the HSTable never receives (still part of the value's CRC, database.cc:256)
constexpr uint32_t kModeFrame = 0, kModeDisabled = 1, kModeRaw = 2, kModeMask = 3, kDropped = 4;

// Per-value layout written by the policy kernel, read by the entry kernel.
struct ValueLayout {
  uint64_t svc;           // size_value_compressed (database.cc:237-248)
  uint64_t svc_hdr;       // size_value_compressed in the header as written last
  uint64_t stored;        // bytes of chunk_final written into the entry (contiguous from 0)
  uint64_t crc_bytes;     // bytes of every chunk_final (the CRC's span after the key)
  uint32_t flags;         // header flags as written last
  uint32_t hdr_crc_final; // 1: the header carries the value CRC, 0: it carries 0
  uint64_t pad_hdr;       // size_padding in the header
  uint32_t kind;          // 0 self-contained, 1 multipart finished, 2 multipart never finished
  int32_t status;         // 0, or -1 (IOError)
};

// Entries small enough for one thread: a single part (or none) and at most
// kSmallEntry bytes of key + chunk_final -- db_bench's 16 B keys / 100 B values.
// A wave spends on the 64-lane CRC tree and the lane-0 header what a thread
// spends on the whole entry, so these run thread per value; the rest wave per
// value
// (the policy kernel lists the latter in `big`: count, then value indices).
constexpr uint32_t kSmallEntry = 512;
__device__ __forceinline__ bool small_entry(const ValueLayout& L, uint32_t np, uint32_t klen) {
  return L.status == 0 && np <= 1u && (uint64_t)klen + L.crc_bytes <= kSmallEntry;
}

// Thread per value: raw offset of each part and its frame slot size.
__global__ void put_prep_kernel(const uint64_t* __restrict__ value_off, const uint32_t* __restrict__ part_first,
                                const uint32_t* __restrict__ chunk_len, uint32_t n, uint64_t* __restrict__ part_src,
                                uint32_t* __restrict__ part_slot) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    uint64_t o = value_off[v];
    for (uint32_t p = part_first[v]; p < part_first[v + 1]; p++) {
      part_src[p] = o;
      const uint32_t c = chunk_len[p];
      part_slot[p] = (8u + compress_bound(c) + 15u) & ~15u;
      o += c;
    }
  }
}

// Thread per value: Database::PutPartValidSize over the value's chunks, then
// the HSTableManager view of the resulting orders.
__global__ void put_policy_kernel(const uint32_t* __restrict__ key_len, const uint64_t* __restrict__ value_len,
                                  const uint32_t* __restrict__ part_first, const uint32_t* __restrict__ chunk_len,
                                  const uint32_t* __restrict__ frame_len, const int32_t* __restrict__ fstatus,
                                  uint32_t n, uint64_t* __restrict__ occ, uint32_t* __restrict__ plen,
                                  uint32_t* __restrict__ mode, ValueLayout* __restrict__ lay,
                                  uint32_t* __restrict__ entry_len, uint32_t* __restrict__ big) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const uint64_t V = value_len[v];
    const uint64_t pad = padding_size(V);
    const uint32_t p0 = part_first[v], p1 = part_first[v + 1];
    bool enabled = true;
    uint64_t ts_offset = 0, comp_total = 0, off = 0, svc = 0, crc_bytes = 0;
    int32_t status = 0;
    for (uint32_t p = p0; p < p1; p++) {
      const uint64_t csz = chunk_len[p];
      const bool first = off == 0, last = csz + off == V;
      const bool do_comp = csz != 0;                                        // database.cc:155-158
      uint64_t o = off;
      if (first) { enabled = true; ts_offset = 0; }                         // :160-163
      if (!enabled) { o = ts_offset; ts_offset = o + csz; }                 // :165-172
      uint32_t m = kModeRaw;
      uint64_t fsz = csz;
      if (do_comp && enabled) {
        if (first) comp_total = 0;                                          // :178-180
        o = comp_total;                                                     // :183
        if (fstatus[p] != 0) { status = -1; break; }                        // :190
        const uint64_t F = frame_len[p];
        comp_total += F;
        const uint64_t size_remaining = V - off;                            // :197-199
        const uint64_t space_left = V + pad - o;
        if (size_remaining - csz + 8u > space_left - F) {                   // :200-209
          comp_total -= F;
          fsz = csz + 8u;
          enabled = false;
          ts_offset = comp_total + fsz;
          m = kModeDisabled;
        } else {
          m = kModeFrame;
          fsz = F;
        }
      }
      if (do_comp && last) svc = enabled ? comp_total : (first ? ts_offset : o + csz);   // :237-248
      if (o + fsz > V + (do_comp ? pad : 0)) { status = -1; break; }        // :261-267
      occ[p] = o;
      plen[p] = (uint32_t)fsz;
      mode[p] = m;
      crc_bytes += fsz;
      off += csz;
    }
    ValueLayout L{};
    L.status = status;
    L.svc = svc;
    L.crc_bytes = crc_bytes;
    const uint32_t klen = key_len[v];
    if (status != 0) {
      L.kind = 0;
      lay[v] = L;
      entry_len[v] = 0;
      big[1u + atomicAdd(big, 1u)] = v;          // its status is the wave kernel's to write
      continue;
    }
    // HSTableManager over the orders: order i carries size_value_compressed and
    // crc only if it is the last call (database.cc:237, 256).
    const uint32_t np = p1 - p0;
    auto is_last = [&](uint32_t i) {                                        // util/order.h:52-55
      const uint64_t so = (i == np - 1) ? svc : 0u;
      const uint64_t end = occ[p0 + i] + plen[p0 + i];
      return (so == 0 && end == V) || (so != 0 && end == so);
    };
    if (np == 0 || is_last(0)) {   // self-contained (WriteFirstPartOrSmallOrder)
      L.kind = 0;
      L.flags = kEntryFull;
      L.pad_hdr = 0;
      L.svc_hdr = np == 1 ? svc : 0u;
      L.hdr_crc_final = np == 1 ? 1u : 0u;
      L.stored = np ? plen[p0] : 0u;
      for (uint32_t i = 1; i < np; i++) mode[p0 + i] |= kDropped;
      entry_len[v] = header_len(L.flags, klen, V, 0) + klen + (uint32_t)L.stored;
    } else {
      uint32_t t = np;   // first later order that looks like a last part
      for (uint32_t i = 1; i < np; i++)
        if (is_last(i)) { t = i; break; }
      for (uint32_t i = (t < np ? t + 1 : np); i < np; i++) mode[p0 + i] |= kDropped;
      const uint32_t wl = t < np ? t : np - 1;
      L.stored = occ[p0 + wl] + plen[p0 + wl];
      L.pad_hdr = pad;
      if (t < np) {                                                          // hstable_manager.h:548-568
        L.kind = 1;
        L.svc_hdr = t == np - 1 ? svc : 0u;
        L.hdr_crc_final = t == np - 1 ? 1u : 0u;
        L.flags = kEntryFull | (L.svc_hdr > 0 ? (kUncompacted | kHasPadding) : 0u);
      } else {                                                               // first-part header stays
        L.kind = 2;
        L.svc_hdr = 0;
        L.hdr_crc_final = 0;
        L.flags = kEntryFull | kUncompacted | kHasPadding;
      }
      // header size is the same for both headers (hstable_manager.h:575-578 checks it)
      entry_len[v] = header_len(L.flags, klen, V, pad) + klen + (uint32_t)(V + pad);
    }
    lay[v] = L;
    if (!small_entry(L, np, klen)) big[1u + atomicAdd(big, 1u)] = v;
  }
}

// Byte j of chunk_final of part p.
struct PartSrc {
  const uint8_t* values;
  const uint8_t* frames;
  const uint64_t* part_src;
  const uint64_t* frame_off;
  const uint32_t* mode;
  __device__ __forceinline__ uint8_t byte(uint32_t p, uint64_t j) const {
    const uint32_t m = mode[p] & kModeMask;
    if (m == kModeFrame) return frames[frame_off[p] + j];
    if (m == kModeDisabled) return j < 8u ? (uint8_t)0 : values[part_src[p] + j - 8u];
    return values[part_src[p] + j];
  }
};

// The CRC's message: the key, then every chunk_final back to back.
struct PutMsg {
  const uint8_t* key;
  uint32_t klen;
  PartSrc src;
  const uint32_t* plen;
  uint32_t p0, p1;
  __device__ uint32_t feed(uint64_t a, uint64_t b, uint32_t c, const uint32_t* s_t) const {
    uint64_t m = a;
    for (; m < b && m < klen; m++) c = crc::step(c, key[m], s_t);
    if (m >= b) return c;
    uint64_t j = m - klen, base = 0;
    uint32_t p = p0;
    while (p < p1 && j >= base + plen[p]) { base += plen[p]; p++; }
    for (; m < b; m++, j++) {
      while (p < p1 && j >= base + plen[p]) { base += plen[p]; p++; }
      c = crc::step(c, src.byte(p, j - base), s_t);
    }
    return c;
  }
};

constexpr int kEntryBlock = 256;

// The CRC32C register c over n bytes copied from src to dst (any alignment
// each): unaligned dword loads, 16 in flight at a time (indices clamped into
// the n bytes, so every load is unconditional and none reads past them), the
// slice-by-4 step per dword, unaligned dword stores; the last n % 4 bytes one
// by one.  Round 6: the byte loop before it loaded, stepped and stored one
// byte per iteration, and as the stores may alias the sources every load
// waited for the one before it (put_entry_small_kernel 185 us per 128 Ki puts).
typedef uint32_t __attribute__((aligned(1))) u32u;
__device__ __forceinline__ uint32_t crc_copy(const uint8_t* src, uint8_t* dst, uint32_t n, uint32_t c,
                                             const uint32_t* s4, const uint32_t* s_t) {
  const uint32_t nd = n >> 2;
#pragma unroll 1
  for (uint32_t d0 = 0; d0 < nd; d0 += 16u) {
    const uint32_t left = nd - d0;
    uint32_t w[16];
#pragma unroll
    for (uint32_t k = 0; k < 16u; ++k) w[k] = *reinterpret_cast<const u32u*>(src + 4u * (d0 + min(k, left - 1u)));
#pragma unroll
    for (uint32_t k = 0; k < 16u; ++k) {
      if (k < left) {
        c = crc::step4(c, w[k], s4);
        *reinterpret_cast<u32u*>(dst + 4u * (d0 + k)) = w[k];
      }
    }
  }
#pragma unroll 1
  for (uint32_t j = nd << 2; j < n; j++) {
    const uint8_t b = src[j];
    dst[j] = b;
    c = crc::step(c, b, s_t);
  }
  return c;
}


// Thread per value (small_entry values only): key and chunk_final copied into
// place with CRC32C(key || chunk_final) (database.cc:251-257) folded into the
// copy, the key hash, and the EntryHeader bytes with their CRC-8 emitted in
// order (format.h:224-255, crc32c.cc:439-475).
__global__ __launch_bounds__(256) void put_entry_small_kernel(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, const uint32_t* __restrict__ key_len,
    const uint64_t* __restrict__ value_len, const uint32_t* __restrict__ part_first, PartSrc src,
    const uint64_t* __restrict__ occ, const uint32_t* __restrict__ plen, const ValueLayout* __restrict__ lay,
    uint32_t n, uint32_t hash_type, uint8_t* __restrict__ entries, const uint64_t* __restrict__ entry_off,
    uint64_t* __restrict__ hashed, uint32_t* __restrict__ crc_out, uint32_t* __restrict__ kind_out,
    int32_t* __restrict__ status_out) {
  __shared__ uint32_t s_t[256];
  __shared__ uint32_t s4[1024];
  __shared__ uint8_t s_c8[256];
  crc::stage_table(s_t);
  crc::stage_table4(s4);
  for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) s_c8[i] = kCrc8.t[i];
  __syncthreads();
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const ValueLayout L = lay[v];
    const uint32_t p0 = part_first[v], np = part_first[v + 1] - p0;
    const uint32_t klen = key_len[v];
    if (!small_entry(L, np, klen)) continue;
    status_out[v] = 0;
    kind_out[v] = L.kind;
    const uint64_t V = value_len[v];
    const uint8_t* key = keys + key_off[v];
    const uint32_t hl = header_len(L.flags, klen, V, L.pad_hdr);
    uint8_t* dst = entries + entry_off[v];
    // (sources resolved once: stores through dst may alias anything, so the
    // compiler would reload the part's mode and offsets per store)
    uint32_t c = crc_copy(key, dst + hl, klen, 0xFFFFFFFFu, s4, s_t);
    if (np == 1u) {
      const uint32_t m = src.mode[p0] & kModeMask;
      const uint32_t len = plen[p0];
      uint8_t* vd = dst + hl + klen + occ[p0];
      // chunk_final byte j = cb[j - skip] for j >= skip, 0 below (the disable header)
      const uint32_t skip = m == kModeDisabled ? 8u : 0u;
      const uint8_t* cb = m == kModeFrame ? src.frames + src.frame_off[p0] : src.values + src.part_src[p0];
      const uint32_t z = skip < len ? skip : len;
      for (uint32_t j = 0; j < z; j++) {
        vd[j] = 0;
        c = crc::step(c, 0u, s_t);
      }
      if (len > skip) c = crc_copy(cb, vd + skip, len - skip, c, s4, s_t);
    }
    const uint32_t crc = c ^ 0xFFFFFFFFu;
    const uint64_t h = hash_type == 1 ? xxh64(key, klen) : murmur3_64(key, klen);
    hashed[v] = h;
    crc_out[v] = crc;
    // header bytes 1 .. hl-1 in order, each into the CRC-8, then byte 0
    uint32_t pos = 1, c8 = 0xffu;
    auto emit = [&](uint32_t b) {
      dst[pos++] = (uint8_t)b;
      c8 = s_c8[(c8 ^ b) & 0xffu];
    };
    auto emit_varint = [&](uint64_t x) {
      while (x >= 128u) { emit((uint32_t)(x & 127u) | 128u); x >>= 7; }
      emit((uint32_t)x);
    };
    const uint32_t cc = L.hdr_crc_final ? crc : 0u;
    for (int i = 0; i < 4; i++) emit((cc >> (8 * i)) & 0xffu);
    emit_varint(L.flags);
    emit_varint(klen);
    emit_varint(V);
    for (int i = 0; i < 8; i++) emit((uint32_t)(L.svc_hdr >> (8 * i)) & 0xffu);
    emit_varint(L.pad_hdr);
    for (int i = 0; i < 8; i++) emit((uint32_t)(h >> (8 * i)) & 0xffu);
    dst[0] = (uint8_t)(c8 ^ 0xffu);
  }
}

// Wave per value: entry bytes at entries + entry_off[v].
__global__ __launch_bounds__(kEntryBlock) void put_entry_kernel(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, const uint32_t* __restrict__ key_len,
    const uint64_t* __restrict__ value_len, const uint32_t* __restrict__ part_first, PartSrc src,
    const uint64_t* __restrict__ occ, const uint32_t* __restrict__ plen, const ValueLayout* __restrict__ lay,
    uint32_t n, uint32_t hash_type, uint8_t* __restrict__ entries, const uint64_t* __restrict__ entry_off,
    const uint32_t* __restrict__ entry_len, uint64_t* __restrict__ hashed, uint32_t* __restrict__ crc_out,
    uint32_t* __restrict__ kind_out, int32_t* __restrict__ status_out, const uint32_t* __restrict__ big) {
  const uint32_t nbig = big[0];
  if (blockIdx.x * (kEntryBlock / 64) >= nbig) return;
  __shared__ uint32_t s_t[256];
  __shared__ uint8_t s_c8[256];
  __shared__ uint8_t s_hdr[kEntryBlock / 64][64];
  crc::stage_table(s_t);
  for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) s_c8[i] = kCrc8.t[i];
  __syncthreads();
  const uint32_t lane = lane_id();
  const uint32_t wib = threadIdx.x / 64u;
  uint8_t* hdr = s_hdr[wib];
  const uint32_t nw = gridDim.x * (kEntryBlock / 64);
  for (uint32_t i = blockIdx.x * (kEntryBlock / 64) + wib; i < nbig; i += nw) {
    const uint32_t v = uni(big[1u + i]);
    const ValueLayout L = lay[v];
    const uint32_t klen = uni(key_len[v]);
    if (lane == 0) { status_out[v] = L.status; kind_out[v] = L.kind; }
    if (L.status != 0) continue;
    const uint64_t V = value_len[v];
    const uint8_t* key = keys + key_off[v];
    const uint32_t hl = header_len(L.flags, klen, V, L.pad_hdr);
    uint8_t* dst = entries + entry_off[v];
    const uint32_t p0 = uni(part_first[v]), p1 = uni(part_first[v + 1]);

    // key, then each written chunk_final at its compressed offset
    for (uint32_t i = lane; i < klen; i += 64u) dst[hl + i] = key[i];
    uint8_t* vdst = dst + hl + klen;
    for (uint32_t p = p0; p < p1; p++) {
      if (src.mode[p] & kDropped) continue;
      const uint64_t o = occ[p], len = plen[p];
      for (uint64_t j = lane; j < len; j += 64u) vdst[o + j] = src.byte(p, j);
    }
    // never-written bytes of a multipart value's reserved region are zero
    // (the reference extends the file with ftruncate, hstable_manager.h:325-333)
    const uint64_t region = (uint64_t)entry_len[v] - hl - klen;
    for (uint64_t j = L.stored + lane; j < region; j += 64u) vdst[j] = 0;

    // CRC32C(key || every chunk_final) (database.cc:251-257), on the wave
    const PutMsg msg{key, klen, src, plen, p0, p1};
    const uint32_t crc = crc::extend_wave(0u, (uint64_t)klen + L.crc_bytes, msg, s_t);

    if (lane == 0) {
      const uint64_t h = hash_type == 1 ? xxh64(key, klen) : murmur3_64(key, klen);
      hashed[v] = h;
      crc_out[v] = crc;
      uint8_t* q = hdr + 1;
      const uint32_t cc = L.hdr_crc_final ? crc : 0u;
      for (int i = 0; i < 4; i++) *q++ = (uint8_t)(cc >> (8 * i));
      q = put_varint(q, L.flags);
      q = put_varint(q, klen);
      q = put_varint(q, V);
      for (int i = 0; i < 8; i++) *q++ = (uint8_t)(L.svc_hdr >> (8 * i));
      q = put_varint(q, L.pad_hdr);
      for (int i = 0; i < 8; i++) *q++ = (uint8_t)(h >> (8 * i));
      uint32_t c8 = 0xffu;                        // crc8(0, header + 1, hl - 1)
      for (uint32_t i = 1; i < hl; i++) c8 = s_c8[(c8 ^ hdr[i]) & 0xffu];
      hdr[0] = (uint8_t)(c8 ^ 0xffu);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane < hl) dst[lane] = hdr[lane];
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void zero_u64_kernel(uint64_t* p) { *p = 0; }

}  // namespace

// Device scratch the batch needs (see kdb_put_entries_batch).
uint64_t put_scratch_bytes(uint32_t n, uint32_t nparts, uint64_t raw_bytes) {
  const uint64_t frames = raw_bytes + raw_bytes / 255u + (uint64_t)nparts * 40u + 64u;
  const uint64_t parts = (uint64_t)nparts * (8 + 4 + 8 + 4 + 4 + 8 + 4 + 4);
  const uint64_t vals = (uint64_t)n * (sizeof(ValueLayout) + 8 + 4) + 64u;
  // every array of launch_put_entries starts on a 256-byte boundary: 13 arrays
  return frames + parts + vals + 13u * 256u;
}

hipError_t launch_put_entries(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len,
                              const uint8_t* values, const uint64_t* value_off, const uint64_t* value_len,
                              const uint32_t* part_first, const uint32_t* chunk_len, uint32_t nparts,
                              uint32_t max_chunk, uint32_t n, uint32_t hash_type, uint8_t* scratch,
                              uint64_t scratch_bytes, uint64_t raw_bytes, uint8_t* entries, uint64_t* entry_off,
                              uint32_t* entry_len, uint64_t* total, uint64_t* hashed, uint32_t* crc,
                              uint32_t* kind, int32_t* status) {
  if (scratch_bytes < put_scratch_bytes(n, nparts, raw_bytes)) return hipErrorInvalidValue;
  uint8_t* s = scratch;
  auto take = [&](uint64_t bytes) {
    uint8_t* r = s;
    s += (bytes + 255u) & ~255ull;
    return r;
  };
  uint8_t* frames = take(raw_bytes + raw_bytes / 255u + (uint64_t)nparts * 40u + 64u);
  uint64_t* part_src = reinterpret_cast<uint64_t*>(take((uint64_t)nparts * 8u));
  uint32_t* part_slot = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  uint64_t* frame_off = reinterpret_cast<uint64_t*>(take((uint64_t)nparts * 8u));
  uint32_t* frame_len = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  int32_t* fstatus = reinterpret_cast<int32_t*>(take((uint64_t)nparts * 4u));
  uint64_t* occ = reinterpret_cast<uint64_t*>(take((uint64_t)nparts * 8u));
  uint32_t* plen = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  uint32_t* mode = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  ValueLayout* lay = reinterpret_cast<ValueLayout*>(take((uint64_t)n * sizeof(ValueLayout)));
  uint64_t* ftotal = reinterpret_cast<uint64_t*>(take(8));
  uint32_t* big = reinterpret_cast<uint32_t*>(take(4u + (uint64_t)n * 4u));   // count, then value indices
  (void)part_slot;
  if (n == 0) {
    hipLaunchKernelGGL(zero_u64_kernel, dim3(1), dim3(1), 0, st, total);
    return hipGetLastError();
  }
  const uint32_t tb = 256, tg = (n + tb - 1) / tb < 4096u ? (n + tb - 1) / tb : 4096u;
  hipLaunchKernelGGL(put_prep_kernel, dim3(tg), dim3(tb), 0, st, value_off, part_first, chunk_len, n, part_src,
                     part_slot);
  if (nparts) {
    hipError_t e = launch_exclusive_scan(st, part_slot, nparts, frame_off, ftotal);
    if (e != hipSuccess) return e;
    e = launch_compress(true, st, values, part_src, chunk_len, nparts, 0u, max_chunk, frames, frame_off,
                                   nullptr, frame_len, fstatus);
    if (e != hipSuccess) return e;
  }
  {
    const hipError_t e = hipMemsetAsync(big, 0, 4, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(put_policy_kernel, dim3(tg), dim3(tb), 0, st, key_len, value_len, part_first, chunk_len,
                     frame_len, fstatus, n, occ, plen, mode, lay, entry_len, big);
  {
    const hipError_t e = launch_exclusive_scan(st, entry_len, n, entry_off, total);
    if (e != hipSuccess) return e;
  }
  const uint32_t eg = (n + 3) / 4 < 16384u ? (n + 3) / 4 : 16384u;
  PartSrc ps{values, frames, part_src, frame_off, mode};
  const uint32_t sg = (n + 255) / 256 < 4096u ? (n + 255) / 256 : 4096u;
  hipLaunchKernelGGL(put_entry_small_kernel, dim3(sg), dim3(256), 0, st, keys, key_off, key_len, value_len,
                     part_first, ps, occ, plen, lay, n, hash_type, entries, entry_off, hashed, crc, kind, status);
  hipLaunchKernelGGL(put_entry_kernel, dim3(eg), dim3(kEntryBlock), 0, st, keys, key_off, key_len, value_len,
                     part_first, ps, occ, plen, lay, n, hash_type, entries, entry_off, entry_len, hashed, crc, kind,
                     status, big);
  return hipGetLastError();
}

}  // namespace kdb_lz4

// ------------------------------------------------------------------ C ABI
using namespace kdb_lz4;

extern "C" uint64_t kdb_put_scratch_bytes(uint32_t n, uint32_t nparts, uint64_t raw_bytes) {
  return put_scratch_bytes(n, nparts, raw_bytes);
}

extern "C" int kdb_put_entries_batch(void* stream, const uint8_t* keys, const uint64_t* key_off,
                                     const uint32_t* key_len, const uint8_t* values, const uint64_t* value_off,
                                     const uint64_t* value_len, const uint32_t* part_first,
                                     const uint32_t* chunk_len, uint32_t nparts, uint32_t max_chunk, uint32_t n,
                                     uint32_t hash_type, uint8_t* scratch, uint64_t scratch_bytes,
                                     uint64_t raw_bytes, uint8_t* entries, uint64_t* entry_off,
                                     uint32_t* entry_len, uint64_t* total, uint64_t* hashed, uint32_t* crc,
                                     uint32_t* kind, int32_t* status) {
  if (!total || (n && (!keys || !key_off || !key_len || !value_off || !value_len || !part_first || !entries ||
                       !entry_off || !entry_len || !hashed || !crc || !kind || !status || !scratch)) ||
      (nparts && (!values || !chunk_len)) || hash_type > 1 || max_chunk > kMaxInput)
    return KDB_LZ4_EINVAL;
  if (scratch_bytes < put_scratch_bytes(n, nparts, raw_bytes)) return KDB_LZ4_EINVAL;
  const hipError_t e = launch_put_entries((hipStream_t)stream, keys, key_off, key_len, values, value_off, value_len,
                                          part_first, chunk_len, nparts, max_chunk, n, hash_type, scratch,
                                          scratch_bytes, raw_bytes, entries, entry_off, entry_len, total, hashed, crc,
                                          kind, status);
  if (e == hipSuccess) return KDB_LZ4_OK;
  return (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? KDB_LZ4_ENODEV : KDB_LZ4_EHIP;
}
