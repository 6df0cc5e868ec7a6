/*
 * oracle/lz4_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the LZ4 r1.3.0 block codec vendored by KingDB
 * (/root/reference/algorithm/lz4.{h,cc}) and of KingDB's CompressorLZ4 frame
 * wrapper (/root/reference/algorithm/compressor.cc), plus CRC32C and the
 * synthetic data generators the benchmark configs name.
 *
 * It exists only as the CHECKER: tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product (kingdb_amd/) never
 * links, loads or calls anything in this directory; the product path runs the
 * HIP kernels in kingdb_amd/csrc and fails loudly if they are unavailable.
 *
 * Parity of this restatement is PINNED against the reference itself: the
 * recipe in oracle/Makefile compiles the reference's own lz4.cc/compressor.cc
 * from /root/reference into oracle/_ref/ (never copied into the repo), and
 * tests/golden/make_golden.py uses that build to emit the committed golden
 * fixtures and to cross-check this file on randomized inputs.
 *
 * Style note: this is written index-based (positions, not pointers) so that it
 * reads like the GPU kernels' specification; every rule cites the reference
 * line it restates.  All arithmetic is integer/byte.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

/* ---- constants: lz4.cc:222-246, lz4.h:60,102-103 ---------------------- */
#define ORC_MINMATCH      4            /* lz4.cc:226 */
#define ORC_LASTLITERALS  5            /* lz4.cc:229 */
#define ORC_MFLIMIT       12           /* lz4.cc:230  (COPYLENGTH+MINMATCH) */
#define ORC_MINLENGTH     13           /* lz4.cc:231  (MFLIMIT+1) */
#define ORC_64KLIMIT      (65536 + 11) /* lz4.cc:237 */
#define ORC_SKIPSTRENGTH  6            /* lz4.cc:238 */
#define ORC_MAX_DISTANCE  65535        /* lz4.cc:241 */
#define ORC_ML_MASK       15u          /* lz4.cc:244 */
#define ORC_RUN_MASK      15u          /* lz4.cc:246 */
#define ORC_MAX_INPUT     0x7E000000u  /* lz4.h:102 */
#define ORC_HASHLOG       12           /* LZ4_MEMORY_USAGE(14) - 2, lz4.cc:222 */

static inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* lz4.h:103 / lz4.cc:371 */
int orc_compress_bound(int isize) {
  if ((unsigned)isize > ORC_MAX_INPUT) return 0;
  return isize + isize / 255 + 16;
}

/* lz4.cc:373-379: byU16 uses a 13-bit hash (>>19), byU32 a 12-bit one (>>20). */
static inline uint32_t hash_at(const uint8_t* src, uint32_t pos, int wide) {
  uint32_t v = rd32(src + pos) * 2654435761u;
  return wide ? (v >> (32 - ORC_HASHLOG)) : (v >> (32 - ORC_HASHLOG - 1));
}

/* lz4.cc:412-428: common prefix length of [a..) and [b..), never reaching
 * `limit` (an absolute position).  The 8/4/2/1-byte stepping of the reference
 * is equivalent to min(LCP, limit - a). */
static uint32_t common_len(const uint8_t* src, uint32_t a, uint32_t b, uint32_t limit) {
  uint32_t n = 0;
  while (a + n < limit && src[a + n] == src[b + n]) n++;
  return n;
}

/*
 * LZ4_compress_limitedOutput (lz4.cc:664-682) instantiating
 * LZ4_compress_generic(limitedOutput, byU16|byU32, noDict, noDictIssue)
 * (lz4.cc:431-641).  Returns bytes written, or 0 when the output does not fit
 * in max_out (checked exactly where the reference checks).
 *
 * NOTE: like the reference, a run of zero-literal sequences is not checked
 * against max_out (lz4.cc:626-628 re-enters _next_match with no test), so with
 * a max_out below the bound the encoder may write past max_out before a later
 * check returns 0.  Callers give `dst` room for orc_compress_bound(isize) + 8
 * bytes; the return value (0 or the size) is what is specified.
 *
 * The table holds positions; it is zero-initialised (lz4.cc:669), so an empty
 * slot reads back as position 0.
 */
int orc_compress_limited(const uint8_t* src, uint8_t* dst, int isize, int max_out) {
  uint32_t table[8192];
  memset(table, 0, sizeof(table));                              /* lz4.cc:669 */
  if ((uint32_t)isize > ORC_MAX_INPUT) return 0;                /* lz4.cc:465 */
  const int wide = isize >= ORC_64KLIMIT;                       /* lz4.cc:673-676 */
  const uint32_t n = (uint32_t)isize;
  const int64_t olimit = max_out;
  int64_t op = 0;                       /* next output byte */
  uint32_t anchor = 0;                  /* first pending literal */
  uint32_t ip = 0;

  if (n >= ORC_MINLENGTH) {                                     /* lz4.cc:483 */
    const uint32_t mflimit = n - ORC_MFLIMIT;
    const uint32_t matchlimit = n - ORC_LASTLITERALS;
    uint32_t fwd_h;
    table[hash_at(src, 0, wide)] = 0;                           /* lz4.cc:486 */
    ip = 1;
    fwd_h = hash_at(src, ip, wide);                             /* lz4.cc:487 */

    for (;;) {
      uint32_t ref;
      int64_t token;
      /* ---- search loop, lz4.cc:494-527 ---- */
      {
        uint32_t fwd_ip = ip;
        uint32_t step = 1;
        uint32_t nb = 1u << ORC_SKIPSTRENGTH;
        for (;;) {
          uint32_t h = fwd_h;
          ip = fwd_ip;
          fwd_ip += step;
          step = (nb++) >> ORC_SKIPSTRENGTH;
          if (fwd_ip > mflimit) goto last_literals;            /* lz4.cc:510 */
          ref = table[h];                                       /* lz4.cc:512 */
          fwd_h = hash_at(src, fwd_ip, wide);                   /* lz4.cc:525 */
          table[h] = ip;                                        /* lz4.cc:526 */
          if (wide && ref + ORC_MAX_DISTANCE < ip) continue;    /* lz4.cc:530 (byU32 only) */
          if (rd32(src + ref) == rd32(src + ip)) break;         /* lz4.cc:531 */
        }
      }
      /* ---- catch up, lz4.cc:535 ---- */
      while (ip > anchor && ref > 0 && src[ip - 1] == src[ref - 1]) { ip--; ref--; }

      /* ---- literal length + literals, lz4.cc:537-554 ---- */
      {
        uint32_t lit = ip - anchor;
        token = op++;
        if (op + lit + (2 + 1 + ORC_LASTLITERALS) + lit / 255 > olimit) return 0;
        if (lit >= ORC_RUN_MASK) {
          int64_t len = (int64_t)lit - ORC_RUN_MASK;
          dst[token] = (uint8_t)(ORC_RUN_MASK << 4);
          for (; len >= 255; len -= 255) dst[op++] = 255;
          dst[op++] = (uint8_t)len;
        } else {
          dst[token] = (uint8_t)(lit << 4);
        }
        memcpy(dst + op, src + anchor, lit);
        op += lit;
      }

    next_match:
      /* ---- offset, lz4.cc:558 ---- */
      {
        uint32_t off = ip - ref;
        dst[op++] = (uint8_t)off;
        dst[op++] = (uint8_t)(off >> 8);
      }
      /* ---- match length, lz4.cc:562-596 ---- */
      {
        uint32_t ml = common_len(src, ip + ORC_MINMATCH, ref + ORC_MINMATCH, matchlimit);
        ip += ORC_MINMATCH + ml;
        if (ml >= ORC_ML_MASK) {
          if (op + (1 + ORC_LASTLITERALS) + (ml >> 8) > olimit) return 0;
          dst[token] += ORC_ML_MASK;
          ml -= ORC_ML_MASK;
          for (; ml >= 510; ml -= 510) { dst[op++] = 255; dst[op++] = 255; }
          if (ml >= 255) { ml -= 255; dst[op++] = 255; }
          dst[op++] = (uint8_t)ml;
        } else {
          dst[token] += (uint8_t)ml;
        }
      }
      anchor = ip;
      if (ip > mflimit) break;                                  /* lz4.cc:601 */

      /* ---- fill table + test next position, lz4.cc:604-628 ---- */
      table[hash_at(src, ip - 2, wide)] = ip - 2;
      {
        uint32_t h = hash_at(src, ip, wide);
        ref = table[h];
        table[h] = ip;
        if (ref + ORC_MAX_DISTANCE >= ip && rd32(src + ref) == rd32(src + ip)) {
          token = op++;
          dst[token] = 0;
          goto next_match;
        }
      }
      fwd_h = hash_at(src, ++ip, wide);                         /* lz4.cc:631 */
    }
  }

last_literals:
  /* ---- last literals, lz4.cc:634-645 ---- */
  {
    int64_t run = (int64_t)n - anchor;
    if (op + run + 1 + (run + 255 - ORC_RUN_MASK) / 255 > (int64_t)(uint32_t)max_out) return 0;
    if (run >= (int64_t)ORC_RUN_MASK) {
      int64_t r = run - ORC_RUN_MASK;
      dst[op++] = (uint8_t)(ORC_RUN_MASK << 4);
      for (; r >= 255; r -= 255) dst[op++] = 255;
      dst[op++] = (uint8_t)r;
    } else {
      dst[op++] = (uint8_t)(run << 4);
    }
    memcpy(dst + op, src + anchor, (size_t)run);
    op += run;
  }
  return (int)op;
}

/*
 * LZ4_decompress_safe_partial (lz4.cc:1050-1053) =
 * LZ4_decompress_generic(endOnInputSize, partial, target, noDict) (lz4.cc:876-1042).
 *
 * Returns bytes decoded, or -(consumed)-1 on malformed input, with `consumed`
 * the input cursor at the point the reference detects the error.
 *
 * Out-of-range input bytes: the reference reads the token and the first
 * literal-length byte without checking ip < iend (lz4.cc:917, 924).  Those are
 * the only reads that can leave [src, src+csize); this restatement (and the
 * GPU kernel) define such a byte as 0, and the golden fixtures are generated
 * with zero padding after every block so the reference sees the same value.
 */
int orc_decompress_safe_partial(const uint8_t* src, uint8_t* dst, int csize,
                                int target, int max_out) {
  const int64_t iend = csize;
  const int64_t oend = max_out;
  int64_t ip = 0, op = 0;
  int64_t oexit = target;
  if (oexit > oend - ORC_MFLIMIT) oexit = oend - ORC_MFLIMIT;          /* lz4.cc:910 */
  if (max_out == 0) return (csize == 1 && src[0] == 0) ? 0 : -1;      /* lz4.cc:911 */
#define IN(i) ((i) >= 0 && (i) < iend ? src[(i)] : 0)

  for (;;) {
    uint32_t token = IN(ip); ip++;
    int64_t length = token >> 4;
    if (length == ORC_RUN_MASK) {                                      /* lz4.cc:920-927 */
      uint32_t s;
      do { s = IN(ip); ip++; length += s; } while (ip < iend - ORC_RUN_MASK && s == 255);
    }
    /* literals, lz4.cc:932-956 */
    {
      int64_t cpy = op + length;
      if (cpy > oexit || ip + length > iend - (2 + 1 + ORC_LASTLITERALS)) {
        if (cpy > oend) goto fail;
        if (ip + length > iend) goto fail;
        memcpy(dst + op, src + ip, (size_t)length);
        ip += length;
        op += length;
        break;
      }
      memcpy(dst + op, src + ip, (size_t)length);
      ip += length;
      op = cpy;
    }
    /* offset, lz4.cc:959-960 (checkOffset: dictSize 0 < 64K) */
    int64_t ref = op - (int64_t)(IN(ip) | (IN(ip + 1) << 8));
    ip += 2;
    if (ref < 0) goto fail;
    /* match length, lz4.cc:963-973 */
    length = token & ORC_ML_MASK;
    if (length == ORC_ML_MASK) {
      uint32_t s;
      do {
        if (ip > iend - ORC_LASTLITERALS) goto fail;
        s = IN(ip); ip++;
        length += s;
      } while (s == 255);
    }
    /* copy, lz4.cc:1005-1030: the end-of-block rule is "match end must stay
     * <= oend-5"; the dec32/dec64 overlap trick equals a forward byte copy. */
    {
      int64_t mend = op + length + ORC_MINMATCH;
      if (mend > oend - 12 && mend > oend - ORC_LASTLITERALS) goto fail;
      /* The reference also writes op..op+7 before that test (lz4.cc:1008-1018);
       * those bytes lie inside [0, oend) and are rewritten later, so the
       * observable result on success is the forward byte copy below. */
      for (int64_t i = 0; i < length + ORC_MINMATCH; i++) dst[op + i] = dst[ref + i];
      op = mend;
    }
  }
  return (int)op;
fail:
  return (int)(-ip - 1);
#undef IN
}

/* ---- CRC32C (Castagnoli, reflected 0x82F63B78): crc32c.cc:296-340 ------- */
static uint32_t crc_table[256];
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    crc_table[i] = c;
  }
}
/* filled before main (callers may be concurrent threads) */
__attribute__((constructor)) static void crc_init_ctor(void) { crc_init(); }
uint32_t orc_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint32_t l = crc ^ 0xffffffffu;
  for (size_t i = 0; i < n; i++) l = crc_table[(l ^ p[i]) & 0xff] ^ (l >> 8);
  return l ^ 0xffffffffu;
}

/*
 * CompressorLZ4::Compress frame bytes (compressor.cc:15-65).
 * frame = u32le(size_compressed_stored) u32le(size_source) payload.
 * Writes the frame into `frame` (capacity >= 8 + max(bound, n)) and returns its
 * length, or -1 where the reference returns IOError (ret <= 0).
 */
int64_t orc_frame_compress(const uint8_t* src, uint64_t n, uint8_t* frame) {
  uint32_t bound = (uint32_t)orc_compress_bound((int)n);
  int ret = orc_compress_limited(src, frame + 8, (int)n, (int)bound);
  if (ret <= 0) return -1;                                      /* compressor.cc:31-34 */
  uint32_t stored = (uint32_t)ret + 8;
  uint64_t flen = (uint64_t)ret + 8;
  if ((uint64_t)ret > n) {                                      /* compressor.cc:40-48 */
    memcpy(frame + 8, src, n);
    flen = n + 8;
    stored = 0;
  }
  uint32_t n32 = (uint32_t)n;
  for (int i = 0; i < 4; i++) { frame[i] = (uint8_t)(stored >> (8 * i)); frame[4 + i] = (uint8_t)(n32 >> (8 * i)); }
  return (int64_t)flen;
}

/*
 * Digest of a batch of frames (values src[off[i] .. +len[i]) in order):
 * *total = sum of frame lengths, *crc = CRC32C of the frames concatenated.
 * The same digest oracle/ref_shim.cc's ref_frames_digest takes of the
 * reference's frames (tests/golden/digests.json).  -1 on IOError.
 */
int orc_frames_digest(const uint8_t* src, const uint64_t* off, const uint32_t* len, uint64_t n,
                      uint64_t* total, uint32_t* crc) {
  uint64_t t = 0, cap = 0;
  uint32_t x = 0;
  uint8_t* fr = NULL;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t need = 8 + (uint64_t)orc_compress_bound((int)len[i]) + len[i] + 64;
    if (need > cap) {
      free(fr);
      cap = need;
      fr = (uint8_t*)malloc(cap);
      if (!fr) return -1;
    }
    int64_t f = orc_frame_compress(src + off[i], len[i], fr);
    if (f < 0) { free(fr); return -1; }
    x = orc_crc32c_extend(x, fr, (size_t)f);
    t += (uint64_t)f;
  }
  free(fr);
  *total = t;
  *crc = x;
  return 0;
}

/*
 * CompressorLZ4::Uncompress of ONE frame at `frame` (compressor.cc:75-137),
 * do_memory_allocation=false flavour.  Returns 0 (OK) and sets *out_n and
 * *frame_n, or -1 (IOError) when the block decoder returns <= 0.
 */
int orc_frame_uncompress(const uint8_t* frame, uint8_t* out, uint64_t* out_n, uint64_t* frame_n) {
  uint32_t stored = rd32(frame), raw = rd32(frame + 4);
  if (stored > 0) {
    uint32_t csz = stored - 8;
    int ret = orc_decompress_safe_partial(frame + 8, out, (int)csz, (int)raw, (int)raw);
    if (ret <= 0) return -1;
    *out_n = (uint64_t)ret;
    *frame_n = (uint64_t)csz + 8;
  } else {
    memcpy(out, frame + 8, raw);
    *out_n = raw;
    *frame_n = (uint64_t)raw + 8;
  }
  return 0;
}

/* ---- Write path: CRC-8, varints, key hashes, EntryHeader,
 *      Database::PutPartValidSize's frame policy ---------------------------- */

/* crc32c::crc8 (crc32c.cc:439-475): reflected CRC-8, table for polynomial 0xB2
 * (reflected), pre/post xor 0xff; crc8(c, p, 0) returns c unchanged. */
static uint8_t crc8_table[256];
__attribute__((constructor)) static void crc8_init(void) {   /* before main: callers may be concurrent */
  for (unsigned i = 0; i < 256; i++) {
    unsigned c = i;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xB2u : c >> 1;
    crc8_table[i] = (uint8_t)c;
  }
}
uint8_t orc_crc8(unsigned crc, const uint8_t* p, size_t n) {
  if (n == 0) return (uint8_t)crc;
  crc ^= 0xffu;
  for (size_t i = 0; i < n; i++) crc = crc8_table[(crc ^ p[i]) & 0xffu];
  return (uint8_t)(crc ^ 0xffu);
}

/* EncodeVarint32/64 (algorithm/coding.cc, LevelDB format): 7 bits per byte, LE. */
static uint8_t* put_varint64(uint8_t* p, uint64_t v) {
  while (v >= 128) { *p++ = (uint8_t)(v | 128); v >>= 7; }
  *p++ = (uint8_t)v;
  return p;
}
static uint8_t* put_fixed32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i)); return p + 4; }
static uint8_t* put_fixed64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); return p + 8; }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

/* XXH64(data, len, 0) (algorithm/xxhash.cc:427, hash.cc:20-23). */
#define XP1 11400714785074694791ULL
#define XP2 14029467366897019727ULL
#define XP3 1609587929392839161ULL
#define XP4 9650029242287828579ULL
#define XP5 2870177450012600261ULL
static inline uint64_t xround(uint64_t acc, uint64_t in) { acc += in * XP2; acc = rotl64(acc, 31); return acc * XP1; }
static inline uint64_t xmerge(uint64_t acc, uint64_t v) { acc ^= xround(0, v); return acc * XP1 + XP4; }
uint64_t orc_xxh64(const uint8_t* p, size_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + XP5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rotl64(h, 27) * XP1 + XP4; p += 8; }
  if (p + 4 <= end) { h ^= (uint64_t)rd32(p) * XP1; h = rotl64(h, 23) * XP2 + XP3; p += 4; }
  while (p < end) { h ^= (uint64_t)(*p) * XP5; h = rotl64(h, 11) * XP1; p++; }
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
  return h;
}

/* MurmurHash3_x64_128(data, len, 0) first 8 bytes (murmurhash3.cc:255-330, hash.cc:9-17). */
static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
  return k;
}
uint64_t orc_murmur3_64(const uint8_t* data, size_t len) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0, h2 = 0;
  const size_t nb = len / 16;
  for (size_t i = 0; i < nb; i++) {
    uint64_t k1 = rd64(data + 16 * i), k2 = rd64(data + 16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* t = data + nb * 16;
  uint64_t k1 = 0, k2 = 0;
  size_t r = len & 15;
  for (size_t i = r; i > 8; i--) k2 ^= (uint64_t)t[i - 1] << (8 * (i - 9));
  if (r > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
  for (size_t i = (r < 8 ? r : 8); i > 0; i--) k1 ^= (uint64_t)t[i - 1] << (8 * (i - 1));
  if (r > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

/* EntryHeader::EncodeTo with compression on (storage/format.h:224-255): crc8
 * byte, fixed32 checksum_content, varint flags / size_key / size_value, fixed64
 * size_value_compressed, varint size_padding, fixed64 hash.  Returns its size. */
int orc_entry_header(uint32_t checksum, uint32_t flags, uint64_t size_key, uint64_t size_value,
                     uint64_t size_value_compressed, uint64_t size_padding, uint64_t hash, uint8_t* out) {
  uint8_t* p = put_fixed32(out + 1, checksum);
  p = put_varint64(p, flags);
  p = put_varint64(p, size_key);
  p = put_varint64(p, size_value);
  p = put_fixed64(p, size_value_compressed);
  p = put_varint64(p, size_padding);
  p = put_fixed64(p, hash);
  out[0] = orc_crc8(0, out + 1, (size_t)(p - out) - 1);
  return (int)(p - out);
}

/* EntryHeader::CalculatePaddingSize (format.h:63-71). */
uint64_t orc_padding(uint64_t size_value) { return (size_value / 65536u + 1u) * 8u; }

/*
 * Database::PutPartValidSize (interface/database.cc:128-276) for every chunk of
 * one value, sent in order by one thread (offset = bytes already sent), with
 * LZ4 compression on.  Per chunk i: part_off[i] = offset_chunk_compressed,
 * part_len[i] = bytes of chunk_final, written to stored + part_off[i] (stored
 * holds size_value + padding bytes).  Also *svc = size_value_compressed (set on
 * the last chunk, 0 when the value is empty) and *crc = CRC32C(key || every
 * chunk_final), as handed to WriteBuffer::PutPart.  Returns 0, or -1 where the
 * reference returns an IOError (compressor failure, or the write-outside-the-
 * allocated-memory check at database.cc:263-267).
 */
int orc_put_value(const uint8_t* key, uint32_t klen, const uint8_t* value, uint64_t size_value,
                  const uint32_t* chunk_len, uint32_t nchunks, uint8_t* stored, uint64_t* part_off,
                  uint32_t* part_len, uint64_t* svc, uint32_t* crc) {
  int enabled = 1;
  uint64_t ts_offset = 0, comp_total = 0, off = 0;
  const uint64_t pad = orc_padding(size_value);
  uint32_t c32 = 0;
  *svc = 0;
  uint8_t* fr = (uint8_t*)malloc(8 + 2 * (size_t)size_value + 64);
  for (uint32_t i = 0; i < nchunks; i++) {
    const uint64_t csz = chunk_len[i];
    const uint8_t* chunk = value + off;
    const int first = off == 0, last = csz + off == size_value;
    const int do_comp = csz != 0;                                     /* :155-158 */
    uint64_t occ = off;
    if (first) { enabled = 1; ts_offset = 0; }                        /* :160-163 */
    if (!enabled) { occ = ts_offset; ts_offset = occ + csz; }         /* :165-172 */
    const uint8_t* fin = chunk;
    uint64_t fsz = csz;
    int hdr_zero = 0;
    if (do_comp && enabled) {
      if (first) comp_total = 0;                                      /* :178-180 */
      occ = comp_total;                                               /* :183 */
      int64_t F = orc_frame_compress(chunk, csz, fr);                 /* :186-189 */
      if (F < 0) { free(fr); return -1; }
      comp_total += (uint64_t)F;
      const uint64_t size_remaining = size_value - off;               /* :197-199 */
      const uint64_t space_left = size_value + pad - occ;
      if (size_remaining - csz + 8u > space_left - (uint64_t)F) {     /* :200-209 */
        comp_total -= (uint64_t)F;
        fsz = csz + 8u;
        enabled = 0;
        ts_offset = comp_total + fsz;
        hdr_zero = 1;
      } else {
        fin = fr;
        fsz = (uint64_t)F;
      }
    }
    if (do_comp && last) {                                            /* :237-248 */
      if (enabled) *svc = comp_total;
      else if (first) *svc = ts_offset;
      else *svc = occ + csz;
    }
    if (occ + fsz > size_value + (do_comp ? pad : 0)) { free(fr); return -1; }   /* :261-267 */
    if (first) c32 = orc_crc32c_extend(0, key, klen);                 /* :251-256 */
    if (hdr_zero) {
      memset(stored + occ, 0, 8);
      memcpy(stored + occ + 8, chunk, csz);
    } else if (fsz) {
      memcpy(stored + occ, fin, fsz);
    }
    c32 = orc_crc32c_extend(c32, stored + occ, fsz);
    part_off[i] = occ;
    part_len[i] = (uint32_t)fsz;
    off += csz;
  }
  free(fr);
  *crc = c32;
  return 0;
}

/*
 * One Database::PutPartValidSize call (interface/database.cc:128-276) over a
 * client thread's state -- the four ThreadStorage slots it reads and writes
 * (ts_compression_enabled_, ts_offset_, the compressor's ts_compress_ and
 * crc32_'s value; thread/threadstorage.h:23-46, all 0 for a thread that never
 * called).  Unlike orc_put_value (one well-formed value) this takes parts in
 * any order a client may send them, which is what the flush hook's batch
 * (include/kdb_flush.h) must match call for call.  LZ4 on.
 * Outputs: chunk_final into `fin` (capacity 8 + bound(csz)), *mode (0 frame,
 * 1 all-zero header + raw, 2 raw, 3 Compress failed), *occ, *fsz, *svc, *crc
 * (the crc32 argument: the running CRC at a last part, else 0).  Returns 0, or
 * -1 where the call returns IOError (mode 3: at :189, before the CRC; else at
 * :261-267, after it).
 */
typedef struct orc_put_state { uint64_t ts_offset, comp_total; uint32_t enabled, crc; } orc_put_state;
int orc_put_part(orc_put_state* st, const uint8_t* key, uint32_t klen, const uint8_t* chunk, uint64_t csz,
                 uint64_t offset_chunk, uint64_t size_value, uint8_t* fin, uint32_t* mode, uint64_t* occ_out,
                 uint64_t* fsz_out, uint64_t* svc_out, uint32_t* crc_out) {
  const uint64_t pad = orc_padding(size_value);
  const int first = offset_chunk == 0, last = csz + offset_chunk == size_value;
  const int do_comp = csz != 0;                                       /* :154-157 */
  uint64_t occ = offset_chunk, fsz = csz, svc = 0;
  *mode = 2;
  if (first) { st->enabled = 1; st->ts_offset = 0; }                  /* :159-162 */
  if (!st->enabled) { occ = st->ts_offset; st->ts_offset = occ + csz; }   /* :164-171 */
  if (do_comp && st->enabled) {
    if (first) st->comp_total = 0;                                    /* :177-179 */
    occ = st->comp_total;                                             /* :182 */
    const int64_t F = orc_frame_compress(chunk, csz, fin);            /* :185-189 */
    if (F < 0) { *mode = 3; *occ_out = occ; *fsz_out = 0; *svc_out = 0; *crc_out = 0; return -1; }
    st->comp_total += (uint64_t)F;
    const uint64_t size_remaining = size_value - offset_chunk;        /* :197-199 */
    const uint64_t space_left = size_value + pad - occ;
    if (size_remaining - csz + 8u > space_left - (uint64_t)F) {       /* :199-209 */
      st->comp_total -= (uint64_t)F;
      fsz = csz + 8u;
      st->enabled = 0;
      st->ts_offset = st->comp_total + fsz;
      memset(fin, 0, 8);
      memcpy(fin + 8, chunk, csz);
      *mode = 1;
    } else {
      fsz = (uint64_t)F;
      *mode = 0;
    }
  }
  if (*mode == 2 && csz) memcpy(fin, chunk, csz);
  if (do_comp && last) svc = st->enabled ? st->comp_total : (first ? st->ts_offset : occ + csz);   /* :237-248 */
  if (first) st->crc = orc_crc32c_extend(0, key, klen);               /* :251-255 */
  st->crc = orc_crc32c_extend(st->crc, fin, fsz);                     /* :256 */
  *crc_out = last ? st->crc : 0u;                                     /* :257 */
  *occ_out = occ;
  *fsz_out = fsz;
  *svc_out = svc;
  return occ + fsz > size_value + (do_comp ? pad : 0) ? -1 : 0;       /* :261-267 */
}

/*
 * CompressorLZ4::UncompressByteArray (algorithm/compressor.cc:140-249) over
 * CompressorLZ4::Uncompress (compressor.cc:75-137): the read of one stored
 * value (Database::GetRaw, interface/database.cc:65-68).  `stored` holds
 * `avail` readable bytes (the entry's value region); svc = size_value_compressed
 * (0: the value is not compressed), size = size_value.  verify: 0 none,
 * 1 the reference's checksum check -- each frame streamed into the CRC twice,
 * Uncompress (:126) and UncompressByteArray (:202) -- 2 the same with each frame
 * streamed once (the corrected check).  Returns 0 OK, -1 IOError from the
 * block decoder, -2 IOError "Invalid checksum.", -3 where the reference would
 * read or write outside the value (malformed sizes; undefined there).
 * *out_n = bytes of `out` the reference defines.
 */
int orc_get_value(const uint8_t* stored, uint64_t avail, uint64_t svc, uint64_t size, uint32_t checksum,
                  uint32_t checksum_initial, int verify, uint8_t* out, uint64_t* out_n) {
  uint32_t crc = verify ? checksum_initial : 0;                  /* :144-147 */
  const int compressed = svc != 0;
  int disabled = 0;
  uint64_t in = 0, o = 0;
  *out_n = 0;
  for (;;) {
    if (compressed && !disabled) {
      if (in == svc) {                                           /* :159-169 */
        if (!verify || crc == checksum) return 0;
        return -2;
      }
      if (in > svc || in + 8 > avail) return -3;
      int zero = 1;                                              /* HasFrameHeaderDisabledCompression */
      for (int i = 0; i < 8; i++) zero &= stored[in + i] == 0;
      if (zero) {                                                /* :171-178 */
        disabled = 1;
        if (verify) crc = orc_crc32c_extend(crc, stored + in, 8);
        in += 8;
      } else {
        uint32_t st = rd32(stored + in), raw = rd32(stored + in + 4);
        uint64_t fsz;
        if (o + raw > size) return -3;
        if (st > 0) {                                            /* :92-113 */
          uint32_t csz = st - 8;                                 /* u32 wrap below 8 */
          if ((int)csz < 0) return -1;  /* negative block size: the r1.3.0 decoder fails at its first check */
          if ((uint64_t)csz + 8 > avail - in) return -3;
          int ret = orc_decompress_safe_partial(stored + in + 8, out + o, (int)csz, (int)raw, (int)raw);
          if (ret <= 0) return -1;
          fsz = (uint64_t)csz + 8;
          o += (uint64_t)ret;
        } else {                                                 /* :114-121 */
          if ((uint64_t)raw + 8 > avail - in) return -3;
          memcpy(out + o, stored + in + 8, raw);
          fsz = (uint64_t)raw + 8;
          o += raw;
        }
        if (verify) {                                            /* :126 (+ :202) */
          crc = orc_crc32c_extend(crc, stored + in, fsz);
          if (verify == 1) crc = orc_crc32c_extend(crc, stored + in, fsz);
        }
        in += fsz;
        *out_n = o;
      }
    }
    if (!compressed || disabled) {                               /* :224-247 */
      const uint64_t left = compressed ? svc : size;
      if (in == left) return 0;
      if (in > left) return -3;
      uint64_t cur = left - in < 1048576u ? left - in : 1048576u;
      if (in + cur > avail || o + cur > size) return -3;
      memcpy(out + o, stored + in, cur);
      o += cur;
      *out_n = o;
      return 0;
    }
  }
}

/* ---- Generators ----------------------------------------------------------
 * G1: db_bench's RandomGenerator (doc/bench/db_bench_kingdb.cc:113-142) over
 * LevelDB's Random(301) (Park-Miller, A=16807, M=2^31-1) and
 * test::CompressibleString(ratio 0.5, len 100) = 50 chars ' '+Uniform(95)
 * repeated to 100.  LevelDB util/random.h + util/testutil.cc are not vendored in
 * the reference; this restates their published algorithm (LevelDB 1.x).
 */
static inline uint32_t pm_next(uint32_t s) {
  uint64_t product = (uint64_t)s * 16807u;
  uint32_t r = (uint32_t)((product >> 31) + (product & 2147483647u));
  if (r > 2147483647u) r -= 2147483647u;
  return r;
}
/* Fills `out` with `npieces` 100-byte pieces starting from Random(seed). */
void orc_g1_pieces(uint32_t seed, uint64_t npieces, uint8_t* out) {
  uint32_t s = seed & 0x7fffffffu;
  if (s == 0 || s == 2147483647u) s = 1;
  for (uint64_t p = 0; p < npieces; p++) {
    uint8_t raw[50];
    for (int i = 0; i < 50; i++) { s = pm_next(s); raw[i] = (uint8_t)(' ' + s % 95); }
    memcpy(out + p * 100, raw, 50);
    memcpy(out + p * 100 + 50, raw, 50);
  }
}

/* ---- CPU baseline harness (bench.py cpu_baseline leg, kind "port") -------
 * Same protocol as oracle/ref_shim.cc:ref_bench_roundtrip, over this
 * restatement: blocked partition over pthreads, one warm-up pass, `passes`
 * timed passes, compress and decompress phases timed separately. */
#include <pthread.h>
#include <stdlib.h>
#include <time.h>

typedef struct {
  const uint8_t* src; uint8_t* blocks; int* blen; uint8_t* out;
  int lo, hi, size, bound, comp, bad;
} orc_job;

static void* orc_bench_worker(void* p) {
  orc_job* j = (orc_job*)p;
  for (int i = j->lo; i < j->hi; i++) {
    if (j->comp) {
      j->blen[i] = orc_compress_limited(j->src + (size_t)i * j->size, j->blocks + (size_t)i * j->bound,
                                        j->size, j->bound);
    } else {
      int r = orc_decompress_safe_partial(j->blocks + (size_t)i * j->bound, j->out + (size_t)i * j->size,
                                          j->blen[i], j->size, j->size);
      if (r != j->size) j->bad = 1;
    }
  }
  return NULL;
}

static double orc_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int orc_bench_phase(orc_job* jobs, int threads, int comp) {
  pthread_t th[256];
  int bad = 0;
  for (int t = 0; t < threads; t++) { jobs[t].comp = comp; pthread_create(&th[t], NULL, orc_bench_worker, &jobs[t]); }
  for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); bad |= jobs[t].bad; }
  return bad;
}

int orc_bench_roundtrip(const uint8_t* src, int n, int size, int threads, int passes,
                        double* t_compress, double* t_decompress, uint64_t* comp_bytes) {
  if (threads > 256) threads = 256;
  const int bound = orc_compress_bound(size) + 8;
  uint8_t* blocks = (uint8_t*)malloc((size_t)n * bound);
  int* blen = (int*)malloc(sizeof(int) * (size_t)n);
  uint8_t* out = (uint8_t*)malloc((size_t)n * size + 64);
  orc_job jobs[256];
  for (int t = 0; t < threads; t++) {
    orc_job j = {src, blocks, blen, out, (int)((int64_t)n * t / threads), (int)((int64_t)n * (t + 1) / threads),
                 size, bound - 8, 0, 0};
    jobs[t] = j;
  }
  int bad = orc_bench_phase(jobs, threads, 1) | orc_bench_phase(jobs, threads, 0);
  double tc = 0, td = 0;
  for (int p = 0; p < passes; p++) {
    double a = orc_now();
    bad |= orc_bench_phase(jobs, threads, 1);
    double b = orc_now();
    bad |= orc_bench_phase(jobs, threads, 0);
    double c = orc_now();
    tc += b - a;
    td += c - b;
  }
  uint64_t cb = 0;
  for (int i = 0; i < n; i++) cb += (uint64_t)blen[i];
  *t_compress = tc; *t_decompress = td; *comp_bytes = cb;
  if (memcmp(out, src, (size_t)n * size) != 0) bad = 1;
  free(blocks); free(blen); free(out);
  return bad ? -1 : 0;
}
