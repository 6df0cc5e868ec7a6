// kingdb_amd/csrc/lz4_compress.hip -- gfx950 LZ4 r1.3.0 block compressor.
//
// Replaces LZ4_compress_limitedOutput (/root/reference/algorithm/lz4.cc:664-682)
// = LZ4_compress_generic(limitedOutput, byU16, noDict, noDictIssue)
// (lz4.cc:431-641), fused with CompressorLZ4::Compress's frame epilogue
// (algorithm/compressor.cc:26-59).  Output is byte-identical to the reference.
//
// Persistent launch: one wavefront (workgroup of 64) per resident slot takes
// values from device-scope work counters, one value ahead.  Size classes
// (launch_compress): values <= 4 KiB are staged in LDS next to a two-plane
// 12-bit table (16 KiB per value; ten such waves per 160 KiB workgroup, so 10
// values per CU -- one-wave workgroups of 16 KiB held 9) and the next value is
// prefetched into registers while the current one is parsed; 4-8 KiB values
// are staged next to a u16 table; larger values are read in place from
// HBM/L2 with only the table (u16 for byU16, u32 for byU32) in LDS.  The
// table is zeroed per value (lz4.cc:669: an empty slot reads as position 0).
// Every LDS read is clamped into its region.  Each sequence's bytes (token,
// length runs, literals, offset) are written straight to HBM by one
// wave-wide byte store per 64 bytes.
//
// The greedy parse is sequential by definition; what is parallel is:
//  * the search loop (lz4.cc:494-527): the positions it visits from a start
//    `s` are a closed-form function of the iteration index (step =
//    nb++ >> SKIPSTRENGTH), so 64 iterations are evaluated at once, one per
//    lane.  Iteration k's table get must see every earlier iteration's put:
//    one lane-ordered LDS exchange (ds_mskor_rtn_b32) per table plane does
//    the get+put of all 64 iterations, each lane reading its slot as the
//    lanes before it left it (see "hash tables" below).  The first matching
//    lane ends the chunk; the puts of the lanes after it are undone, leaving
//    exactly the table state of the sequential loop;
//  * the catch-up loop (lz4.cc:531) and LZ4_count (lz4.cc:562-578), issued
//    together: the match length after catching up c bytes is c + the length
//    measured from the original position, so neither waits for the other;
//  * the byte emission of a sequence.
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>

#include "lz4_device.h"
#include "service.h"

namespace kdb_lz4 {

// Position visited at iteration k of a search run started at s (lz4.cc:497-507):
// p(0)=s, p(k+1)=p(k)+step(k), step(0)=1, step(k)=(63+k)>>6 for k>=1, i.e.
// p(k) = s + 1 + sum_{t=64}^{62+k} floor(t/64) for k >= 1.
// (kWide: 64-bit intermediates -- a search can run ~500K iterations on 2 GB.)
template <bool kWide>
__device__ __forceinline__ uint32_t search_pos(uint32_t s, uint32_t k) {
  if (k == 0) return s;
  const uint32_t nn = 62u + k, q = nn >> 6, r = nn & 63u;
  if (kWide) return (uint32_t)min((uint64_t)s + 1u + 32ull * q * (q - 1u) + (uint64_t)q * (r + 1u), 0xFFFFFFFFull);
  return s + 1u + 32u * q * (q - 1u) + q * (r + 1u);
}
__device__ __forceinline__ uint32_t search_step(uint32_t k) { return k == 0 ? 1u : (63u + k) >> 6; }
// p(k) for k >= 1 (chunks after the first: k >= 61), no k == 0 case to select
template <bool kWide>
__device__ __forceinline__ uint32_t search_pos_nz(uint32_t s, uint32_t k) {
  const uint32_t nn = 62u + k, q = nn >> 6, r = nn & 63u;
  if (kWide) return (uint32_t)min((uint64_t)s + 1u + 32ull * q * (q - 1u) + (uint64_t)q * (r + 1u), 0xFFFFFFFFull);
  return s + 1u + 32u * q * (q - 1u) + q * (r + 1u);
}

__device__ __forceinline__ uint32_t hash16(uint32_t seq) { return (seq * 2654435761u) >> 19; }
// lz4.cc:373-379: byU16 hashes to 13 bits, byU32 to 12
template <bool kWide>
__device__ __forceinline__ uint32_t hashp(uint32_t seq) { return (seq * 2654435761u) >> (kWide ? 20 : 19); }


// ---------------------------------------------------------------- hash tables
//
// A search chunk evaluates 64 iterations of the search loop at once, and
// iteration k's get must see every put of iterations < k (lz4.cc:505-523: get
// then put, per iteration).  gfx950's LDS resolves the lanes of ONE
// instruction that hit the same dword in ascending lane order -- a
// read-modify-write with return gives lane i the word as lanes < i left it
// (measured: tools/probe/lds_order.hip, 0 exceptions in 128 000 lanes).  So a
// single ds_mskor_rtn_b32 per table plane is the whole get+put of a chunk:
// lane i reads the entry of its slot as the nearest lower lane of the same
// slot wrote it -- or as the chunk found it -- and writes its own position.
// That is the sequential table, up to the lane that matches; the puts of the
// lanes after it (which the sequential loop never makes) are undone by
// restore(), by the one lane per slot whose entry came from before them.
//
// mskor: D = (D & ~mask) | data, on the dword holding the slot's field; a
// lane with on = false passes mask 0 AND data 0 (no change) and still reads.

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// LDS byte offset of a (generic) pointer into LDS, made opaque so the
// compiler keeps it in an SGPR instead of redoing the generic-to-LDS
// conversion (a null test and a select) at every use inside the parse loop.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  uint32_t o = (uint32_t)(uintptr_t)(const lds_u8*)p;
  asm volatile("" : "+s"(o));
  return o;
}

__device__ __forceinline__ uint32_t mskor_rtn(uint32_t a, uint32_t m, uint32_t d) {
  uint32_t r;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=&v"(r) : "v"(a), "v"(m), "v"(d)
               : "memory");
  return r;
}
__device__ __forceinline__ void mskor(uint32_t a, uint32_t m, uint32_t d) {
  asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(a), "v"(m), "v"(d) : "memory");
}

// byU16 table for values <= 4 KiB, whose positions fit 12 bits: two planes,
// the low bytes (8192 x u8) and the high nibbles (4096 x u8, two per byte),
// 12 KiB instead of 16 -- 16 KiB of LDS per value with its bytes, so 10
// values per CU in ten-wave workgroups of 160 KiB (the hardware allocates LDS
// per workgroup in 1 280-byte steps: one-wave workgroups of 16 KiB hold 9;
// the parse is latency-bound: occupancy is speed).  Cleared per
// value (12 x 16 B stores per lane).  The layout is fixed (the kernels that
// use it have one static LDS array, at LDS address 0): the value at [0, 4096),
// the low bytes at kT12Lo, the high nibbles at kT12Hi -- both planes are
// addressed through the instructions' offset fields, and the value's bytes
// need no base, so no address of the parse carries an add for a region base.
#define KDB_T12_LO 4096
#define KDB_T12_HI 12288
constexpr uint32_t kT12Lo = KDB_T12_LO, kT12Hi = KDB_T12_HI;
static_assert(kT12Lo == 4096u && kT12Hi == kT12Lo + 8192u, "value, then the 8 KiB low-byte plane, then the nibbles");
#define KDB_STR2(x) #x
#define KDB_STR(x) KDB_STR2(x)
// An off lane's address bits in a workgroup of several waves, each with its
// 16 KiB region at base = wave x 16 KiB (lz4_compress_kernel<..., kWaves>):
// 163 840, the whole 160 KiB past LDS address 0, so `base | h` for an off
// lane lands past the workgroup's allocation from every wave's region (its
// bits, 15 and 17, are clear in every slot index and nibble address).
constexpr uint32_t kOffLaneWG = 0x28000u;
// kBased: the table of wave `base >> 14` of a multi-wave workgroup -- its
// planes at base + kT12Lo / base + kT12Hi.  The base rides in the off-lane
// select the exchange makes anyway (on ? base : kOffLaneWG), so no address
// of the parse carries an add for it.
template <bool kBased>
struct Table12T {
  static constexpr bool kTagged = false;
  uint32_t base = 0;   // kBased: this wave's region (a multiple of 16 KiB)
  // a lane's slot as the exchange addressed it, kept for restore(): the low
  // byte's index, the high nibble's dword address (in its plane) and shift
  struct Slot { uint32_t lo, hi, sh, mh; };
  // get-then-put of every lane of the chunk, in lane order (see above)
  __device__ __forceinline__ uint32_t xchg(uint32_t h, uint32_t p, bool on, Slot& s) const {
    const uint32_t sl = (h & 3u) << 3;
    s.sh = (h & 7u) << 2;
    // A lane whose exchange is off addresses LDS past the kernel's allocation
    // (reads return 0, writes are dropped: it neither gets nor puts, and its
    // restore is dropped too) instead of carrying a zero mask and zero data:
    // one select for the address instead of four on the masks and data
    // (compress 9.07 -> 9.00 ms, profiles/r04_d/r04_e_ab_exchange_oor.txt)
    const uint32_t oor = kBased ? (on ? base : kOffLaneWG) : (on ? 0u : 0x10000u);
    s.lo = h | oor;
    s.hi = ((h >> 1) & ~3u) | oor;
    const uint32_t ml = 0xffu << sl;
    s.mh = 15u << s.sh;
    const uint32_t dl = (p & 0xffu) << sl, dh = ((p >> 8) & 15u) << s.sh;
    const uint32_t al = (h & ~3u) | oor;
    uint32_t ol, oh;
    asm volatile(
        "ds_mskor_rtn_b32 %0, %2, %3, %4 offset:" KDB_STR(KDB_T12_LO) "\n\t"
        "ds_mskor_rtn_b32 %1, %5, %6, %7 offset:" KDB_STR(KDB_T12_HI) "\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(ol), "=&v"(oh)
        : "v"(al), "v"(ml), "v"(dl), "v"(s.hi), "v"(s.mh), "v"(dh)
        : "memory");
#if KDB_ABL_DUP_XCHG
    // attribution build (tools/gpurun/lds_attr.sh): the same two exchanges
    // again as reads (mask 0, data 0), so their LDS bank conflicts count twice
    uint32_t d0, d1;
    asm volatile(
        "ds_mskor_rtn_b32 %0, %2, %4, %4 offset:" KDB_STR(KDB_T12_LO) "\n\t"
        "ds_mskor_rtn_b32 %1, %3, %4, %4 offset:" KDB_STR(KDB_T12_HI) "\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(d0), "=&v"(d1) : "v"(h & ~3u), "v"(s.hi), "v"(0u) : "memory");
    asm volatile("" ::"v"(d0), "v"(d1));
#endif
    return (__builtin_amdgcn_ubfe(oh, s.sh, 4) << 8) | __builtin_amdgcn_ubfe(ol, sl, 8);
  }
  // v: a position < 4096; only lanes whose exchange was on (mh = their nibble mask)
  __device__ __forceinline__ void restore(const Slot& s, uint32_t v) const {
    ((lds_u8*)(uintptr_t)(s.lo + kT12Lo))[0] = (uint8_t)v;
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:" KDB_STR(KDB_T12_HI) ::"v"(s.hi), "v"(s.mh), "v"((v >> 8) << s.sh)
                 : "memory");
  }
};
using Table12 = Table12T<false>;
constexpr uint32_t kTable12Bytes = 8192u + 4096u;
// The off-lane addresses of the exchanges (Table12/16/32::xchg) rely on the
// hardware dropping LDS accesses past the kernel's allocation: they start at
// 0x10000 past the table's base, so every kernel that uses these tables must
// allocate less LDS than that (gfx950 allows up to 160 KiB per workgroup).
// Checked statically for the fixed layouts below and at launch for the
// dynamically sized one (launch_one, the 4-8 KiB class).
constexpr uint32_t kOffLaneLds = 0x10000u;

// byU16 table, 8192 x u16 (values up to 65 546 bytes; positions < 65 536).
// kWG: the table of one wave of a multi-wave workgroup (its 16 KiB region at
// `off`): an off lane's index gets bits that put it past the whole 160 KiB
// (kOffLaneWG) instead of 64 KiB past the table, which would be another
// wave's region.
template <bool kWG>
struct Table16T {
  static constexpr bool kTagged = false;
  uint32_t off;
  struct Slot { uint32_t h; };
  __device__ Table16T(uint16_t* p) : off(lds_off(p)) {}
  __device__ Table16T() : off(0) {}
  __device__ __forceinline__ uint32_t xchg(uint32_t h, uint32_t p, bool on, Slot& s) const {
    // an off lane addresses past the allocation (see Table12::xchg): mixed
    // batch compress 5.510 -> 5.494 ms (profiles/r04_d/r04_f_ab_exchange_oor16.txt)
    const uint32_t oor = on ? 0u : (kWG ? kOffLaneWG >> 1 : 0x8000u);
    s.h = h | oor;
    const uint32_t sh = (h & 1u) << 4;
    const uint32_t o = mskor_rtn(off + ((s.h & ~1u) << 1), 0xffffu << sh, (p & 0xffffu) << sh);
    return (o >> sh) & 0xffffu;
  }
  __device__ __forceinline__ void restore(const Slot& s, uint32_t v) const {
    ((lds_u16*)(uintptr_t)off)[s.h] = (uint16_t)v;
  }
};
using Table16 = Table16T<false>;

// byU32 table (values >= 65547 bytes): 4096 x u32 positions (lz4.cc:383-410).
struct Table32 {
  static constexpr bool kTagged = false;
  uint32_t off;
  struct Slot { uint32_t h; };
  __device__ Table32(uint32_t* p) : off(lds_off(p)) {}
  __device__ Table32() : off(0) {}
  __device__ __forceinline__ uint32_t xchg(uint32_t h, uint32_t p, bool on, Slot& s) const {
    s.h = h | (on ? 0u : 0x4000u);      // an off lane: past the allocation (see Table12::xchg)
    return mskor_rtn(off + (s.h << 2), 0xffffffffu, p);
  }
  __device__ __forceinline__ void restore(const Slot& s, uint32_t v) const { ((lds_u32*)(uintptr_t)off)[s.h] = v; }
};

// byU32 table with word tags (values of at most kTagMaxLen bytes: positions fit
// 20 bits).  An entry is position | tag << 20, the tag 12 more bits of the
// entry's 4-byte word (bits 8-19 of the hash product; the hash takes bits
// 20-31).  Two words with different tags differ, so a candidate whose tag is
// not the searched word's -- or whose position is past the 64 KiB window --
// cannot match (lz4.cc:526-527), and its 4 bytes are not read: the reads left
// are mostly true matches near the search, hits in this wave's cache lines,
// instead of stale entries scattered over the value's past (L2/MALL misses on
// 1 MiB parts).  The same decisions and the same table contents, positions-
// wise, as Table32.  An empty entry is position 0 with position 0's tag
// (empty()): the reference's empty slots read as position 0, whose word may
// match.
constexpr uint32_t kTagMaxLen = 1u << 20;
__device__ __forceinline__ uint32_t word_tag(uint32_t seq) { return ((seq * 2654435761u) >> 8) & 0xfffu; }
struct Table32T {
  static constexpr bool kTagged = true;
  uint32_t off;
  struct Slot { uint32_t h, e; };
  __device__ Table32T(uint32_t* p) : off(lds_off(p)) {}
  __device__ Table32T() : off(0) {}
  __device__ __forceinline__ static uint32_t empty(uint32_t word0) { return word_tag(word0) << 20; }
  __device__ __forceinline__ static uint32_t tag(uint32_t seq) { return word_tag(seq); }
  // every entry empty: the 16 KiB at t (the table's base), as 16-byte stores
  __device__ __forceinline__ static void clear(uint32_t* t, uint32_t word0) {
    const uint32_t f = empty(word0);
    for (uint32_t i = lane_id(); i < 4096u / 4u; i += 64u) reinterpret_cast<uint4*>(t)[i] = make_uint4(f, f, f, f);
  }
  // get + put with the tag; *maybe: the old entry's tag is tg (the lane is on)
  __device__ __forceinline__ uint32_t xchg_tagged(uint32_t h, uint32_t p, uint32_t tg, bool on, Slot& s,
                                                  bool& maybe) const {
    s.h = h | (on ? 0u : 0x4000u);      // an off lane: past the allocation (see Table12::xchg)
    s.e = mskor_rtn(off + (s.h << 2), 0xffffffffu, p | (tg << 20));
    maybe = on && (s.e >> 20) == tg;
    return s.e & 0xfffffu;
  }
  // the entry as this lane read it (v, its position, is implied)
  __device__ __forceinline__ void restore(const Slot& s, uint32_t) const { ((lds_u32*)(uintptr_t)off)[s.h] = s.e; }
};

// The same tagged byU32 table in 12 KiB, for launches whose values are all at
// most kTagMaxLen bytes: two planes, the positions' low halves (4096 x u16) and
// one byte per entry of position bits 16-19 and a 4-bit tag (bits 16-19 of the
// hash product).  With the 2 KiB ring next to it a wave needs 14.1 KiB of LDS
// instead of 20.1: 10 waves per CU instead of 7 (tools/probe/lds_occupancy --
// the hardware admits 10 workgroups of 14.1 or 15 KiB per CU but only 9 of
// 16 KiB, and 7 of 20.1), so KingDB's 1 MiB parts of a batch (2 560 per GPU in
// `--workload big`) all run in one round: compress 14.2 -> 11.15 ms.  The
// planes are exchanged together as Table12's are (one ds_mskor_rtn each, in
// lane order).  Per wave it is slower than Table32T (at 7 waves per CU, ~9.4
// against 7.1 ms per round: 1 in 16 stale far entries pass a 4-bit tag and cost
// a global read each), and more tag bits measured no better overall
// (profiles/r05/r05_c*: a 6-bit tag in a third, 2-bit plane 11.3 ms -- one more
// LDS atomic per exchange; an 8-bit tag in 14 KiB needs 16 KiB with the ring,
// 9 waves per CU, 17.2 ms; the same with a 1 KiB ring 17.6-19.9 ms).
struct Table24T {
  static constexpr bool kTagged = true;
  static constexpr uint32_t kBytes = 8192u + 4096u;
  uint32_t off;                         // the u16 plane; the byte plane at off + 8192
  struct Slot { uint32_t h, e; };       // h: the index (| the off-lane bit); e: the old entry, 24 bits
  __device__ Table24T(uint32_t* p) : off(lds_off(p)) {}
  __device__ Table24T() : off(0) {}
  __device__ __forceinline__ static uint32_t tag(uint32_t seq) { return ((seq * 2654435761u) >> 16) & 15u; }
  // every entry empty: position 0 with position 0's tag
  __device__ __forceinline__ static void clear(uint32_t* t, uint32_t word0) {
    const uint32_t b = tag(word0) << 4, f = b * 0x01010101u;
    for (uint32_t i = lane_id(); i < kBytes / 16u; i += 64u)
      reinterpret_cast<uint4*>(t)[i] = i < 512u ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(f, f, f, f);
  }
  __device__ __forceinline__ uint32_t xchg_tagged(uint32_t h, uint32_t p, uint32_t tg, bool on, Slot& s,
                                                  bool& maybe) const {
    s.h = h | (on ? 0u : 0x8000u);      // an off lane: past the allocation (see Table12::xchg)
    const uint32_t sl = (h & 1u) << 4, sb = (h & 3u) << 3;
    const uint32_t al = off + ((s.h << 1) & ~3u), ab = off + 8192u + (s.h & ~3u);
    uint32_t ol, ob;
    asm volatile(
        "ds_mskor_rtn_b32 %0, %2, %3, %4\n\t"
        "ds_mskor_rtn_b32 %1, %5, %6, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(ol), "=&v"(ob)
        : "v"(al), "v"(0xffffu << sl), "v"((p & 0xffffu) << sl), "v"(ab), "v"(0xffu << sb),
          "v"(((p >> 16) | (tg << 4)) << sb)
        : "memory");
    const uint32_t lo = __builtin_amdgcn_ubfe(ol, sl, 16), by = __builtin_amdgcn_ubfe(ob, sb, 8);
    s.e = lo | (by << 16);
    maybe = on && (by >> 4) == tg;
    return lo | ((by & 15u) << 16);
  }
  __device__ __forceinline__ void restore(const Slot& s, uint32_t) const {
    ((lds_u16*)(uintptr_t)off)[s.h] = (uint16_t)s.e;
    ((lds_u8*)(uintptr_t)(off + 8192u))[s.h] = (uint8_t)(s.e >> 16);
  }
};

// The per-sequence register window (compress_block's kWin) for tagged byU32
// values too: with the table's tags most candidate reads are near matches, so
// the window's bytes serve the count, the literals and the next input words
// (1 MiB parts: compress 22.3-22.7 -> 20.0 ms; untagged, it measured slower,
// profiles/r04_d/r04_y2_ab_window_byu32.txt).
#ifndef KDB_LZ4_WIDE_WINDOW
#define KDB_LZ4_WIDE_WINDOW 1
#endif
// byU32 values with the tagged table read through an LDS ring (RingSrc)
// instead of in place with the register window: 1 MiB parts compress
// 20.0 -> 15.3 ms (profiles/r05/r05_rg*: a 4 KiB ring refilled 1 KiB at a
// time when the search comes within 512 bytes of its front; a 2 KiB ring
// measured the same, 8 KiB or a 2 KiB front slower, and loading the next
// chunk a refill ahead slower too -- its loads, in flight, then sat in front
// of every other global access's in-order wait).
#ifndef KDB_LZ4_WIDE_RING
#define KDB_LZ4_WIDE_RING 1
#endif
#ifndef KDB_LZ4_RING_AHEAD
#define KDB_LZ4_RING_AHEAD 0
#endif
#ifndef KDB_LZ4_RING_BYTES
#define KDB_LZ4_RING_BYTES 4096u
#endif
#ifndef KDB_LZ4_RING_FRONT
#define KDB_LZ4_RING_FRONT 512u
#endif

// Value bytes staged in LDS (byte i at p[i]).  kUnclamped: a read outside the
// value cannot fault (LDS), so the parse's reads whose result a lane mask
// discards need no clamp into [0, S).
struct LdsSrc {
  static constexpr bool kUnclamped = true;
  static constexpr bool kWindow = false;
  const uint8_t* p;
  __device__ __forceinline__ uint32_t u8(uint32_t i) const { return p[i]; }
  __device__ __forceinline__ uint32_t rd32(uint32_t i) const { return lds_rd32(p, i); }
  // rd32 in two halves: the loads (issued early), then the realignment
  struct Word { uint32_t lo, hi, sh; };
  __device__ __forceinline__ Word rd32_issue(uint32_t i) const {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    return Word{w[i >> 2], w[(i >> 2) + 1u], i & 3u};
  }
  __device__ __forceinline__ static uint32_t word(const Word& w) { return __builtin_amdgcn_alignbyte(w.hi, w.lo, w.sh); }
  __device__ __forceinline__ void step(uint32_t) {}
};

// Value bytes read in place from global memory (any alignment).
struct GlobalSrc {
  static constexpr bool kUnclamped = false;
  static constexpr bool kWindow = true;    // compress_block's per-sequence register window
  const uint8_t* g;
  uint32_t S;
  uint32_t keep;   // the frontier touch in flight (see step)
  __device__ __forceinline__ uint32_t u8(uint32_t i) const { return g[i]; }
  // one unaligned dword load (gfx950's global loads take any alignment): every
  // caller's 4 bytes lie inside the value (positions <= mflimit, or clamped
  // to S - 4), so the load never touches a page past it
  typedef uint32_t __attribute__((aligned(1))) u32u;
  __device__ __forceinline__ uint32_t rd32(uint32_t i) const { return *reinterpret_cast<const u32u*>(g + i); }
  struct Word { uint32_t v; };
  __device__ __forceinline__ Word rd32_issue(uint32_t i) const { return Word{rd32(i)}; }
  __device__ __forceinline__ static uint32_t word(const Word& w) { return w.v; }
  // Touches the 256 bytes from p + 256 (one aligned dword per lane, clamped
  // into the value) so the search frontier is in L1/L2 before it is parsed;
  // the previous touch's dword is consumed here -- one sequence later, when
  // it has long arrived -- so the compiler keeps the load.
  __device__ __forceinline__ void step(uint32_t p) {
    asm volatile("" ::"v"(keep));
    const uint32_t a = min(p + 256u + 4u * lane_id(), S - 1u);
    keep = *reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(g + a) & ~(uintptr_t)3);
  }
};

__device__ __forceinline__ uint4 funnel16(const uint4& a, const uint4& b, uint32_t sh);
// Value bytes of a long value read through an LDS ring of its last kR bytes
// (byU32 values with the tagged table): every read the parse makes near the
// search -- the input words, the count's bytes, the literals, the near
// candidates the tags leave -- is an LDS read; positions outside the ring
// (far candidates, a long count past the front) fall back to global loads.
// Global loads return in issue order (vmcnt), so with the value read in place
// each sequence waited for its own frontier's HBM miss (the frontier touch
// only moved the wait); here the value comes in 1 KiB refills, one wait per
// ~10 G1 sequences.  The ring holds positions [hi - kR, hi) at ring + (p mod
// kR), with a kMirror-byte copy of its first bytes after its end so a 4-byte
// read never wraps.
template <uint32_t kRingBytes>
struct RingSrcT {
  static constexpr bool kUnclamped = false;   // compress_block clamps (the fallback reads global memory)
  static constexpr bool kWindow = false;
  static constexpr uint32_t kR = kRingBytes, kMirror = 64u, kChunk = 1024u, kFront = KDB_LZ4_RING_FRONT;
  typedef uint32_t __attribute__((aligned(1))) u32u;
  const uint8_t* g;
  uint32_t S;
  uint8_t* ring;        // LDS: kR + kMirror bytes, 16-byte aligned
  uint32_t hi;          // positions below hi are staged (the last kR of them are in the ring)
  __device__ __forceinline__ bool in(uint32_t i, uint32_t n) const { return i - (hi - kR) <= kR - n; }
  // The fallback's load is waited for inside its branch (the compiler
  // otherwise waits at the join, on every read: vmcnt(0), in order, so also
  // for every earlier global store; measured neutral on 1 MiB parts, kept for
  // reads that do fall back)
  __device__ __forceinline__ uint32_t u8(uint32_t i) const {
    uint32_t v = ring[i & (kR - 1u)];
    const bool ok = in(i, 1u);
    if (ballot(!ok)) {
      uint32_t gv = 0;
      if (!ok) gv = g[i];
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      v = ok ? v : gv;
    }
    return v;
  }
  __device__ __forceinline__ uint32_t rd32(uint32_t i) const {
    uint32_t v = lds_rd32(ring, i & (kR - 1u));
    const bool ok = in(i, 4u);
    if (ballot(!ok)) {
      uint32_t gv = 0;
      if (!ok) gv = *reinterpret_cast<const u32u*>(g + i);
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      v = ok ? v : gv;
    }
    return v;
  }
  struct Word { uint32_t v; };
  __device__ __forceinline__ Word rd32_issue(uint32_t i) const { return Word{rd32(i)}; }
  __device__ __forceinline__ static uint32_t word(const Word& w) { return w.v; }
  // Before a sequence's search from p: the ring filled to kFront past p (or
  // the value's end), 1 KiB at a time -- whole aligned 16-byte loads (an
  // aligned chunk never crosses a page, so reading around the value cannot
  // fault), realigned in registers.  With KDB_LZ4_RING_AHEAD the next chunk's
  // loads go out at the end of each refill and land in registers (na, nb)
  // until the front needs them, so a refill rarely waits.
  uint4 na, nb;
  bool npend;
  // Only aligned chunks that hold a byte of the value are loaded (a chunk past
  // its end may lie past the allocation: zeros instead); the ring's bytes past
  // S are never used (compress_block clamps its reads into the value).
  __device__ __forceinline__ void fetch(uint32_t at, uint4& a, uint4& b) const {
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
    const uint4* base = reinterpret_cast<const uint4*>(g - head);
    const uint32_t c = (at >> 4) + lane_id();   // this lane's 16 bytes: positions at + 16 lane ..
    const uint32_t end = head + S;               // chunk k holds value bytes iff 16 k < end
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    a = 16u * c < end ? base[c] : z;
    b = head ? (16u * (c + 1u) < end ? base[c + 1u] : z) : a;
  }
  __device__ __forceinline__ void put(const uint4& a, const uint4& b) {
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
    const uint4 w = funnel16(a, b, head);
    const uint32_t o = (hi & (kR - 1u)) + 16u * lane_id();
    reinterpret_cast<uint4*>(ring)[o >> 4] = w;
    if (o < kMirror) reinterpret_cast<uint4*>(ring)[(kR + o) >> 4] = w;
    hi += kChunk;
  }
  __device__ __forceinline__ void step(uint32_t p) {
#pragma unroll 1
    while (hi < S && p + kFront > hi) {
#if KDB_LZ4_RING_AHEAD
      if (npend) {
        put(na, nb);
        npend = false;
        continue;
      }
#endif
      uint4 a, b;
      fetch(hi, a, b);
      put(a, b);
    }
#if KDB_LZ4_RING_AHEAD
    if (!npend && hi < S) {
      fetch(hi, na, nb);
      npend = true;
    }
#endif
  }
};

using RingSrc = RingSrcT<KDB_LZ4_RING_BYTES>;
// the compact launch's ring (Table24T): 2 KiB, measured as fast as 4 KiB with the 16 KiB table
#ifndef KDB_LZ4_COMPACT_RING
#define KDB_LZ4_COMPACT_RING 2048u
#endif
using RingSrcC = RingSrcT<KDB_LZ4_COMPACT_RING>;

// out chunk = bytes [sh, sh+16) of the 32 bytes (a, b); sh in 0..15 (uniform)
__device__ __forceinline__ uint4 funnel16(const uint4& a, const uint4& b, uint32_t sh) {
  if (sh == 0) return a;
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const uint32_t q = sh >> 2, r = sh & 3u;
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t lo = w[k], hi = w[k + 1];
    // select w[k+q], w[k+q+1] with a uniform q (0..3)
    if (q == 1) { lo = w[k + 1]; hi = w[k + 2]; }
    else if (q == 2) { lo = w[k + 2]; hi = w[k + 3]; }
    else if (q == 3) { lo = w[k + 3]; hi = w[k + 4]; }
    o[k] = __builtin_amdgcn_alignbyte(hi, lo, r);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Output: bytes go straight to HBM at out[0..).  kGuard (LZ4_compress_limitedOutput
// with a caller cap below the bound): never write at or past out_cap -- the
// reference may, on limitedOutput failures; the return value is what parity is
// about (see oracle/lz4_oracle.c).  Without kGuard the slot holds the bound,
// which the block never exceeds.
//
// Writes the encoding of one sequence at out[pos .. pos+total): token, the
// literal-length run (nl1 bytes: 255s then remL; none iff lit < 15), the
// literals in[anchor .. anchor+lit), and -- when has_match -- the offset (LE16)
// and the match-length run (nm1 bytes: 255s then remM; none iff ml < 15).
// One global_store_byte per 64 bytes.  Returns total.
//
// Run lengths: a run of n >= 15 is (n-15)/255 bytes of 255 and one of
// (n-15) % 255 (lz4.cc:539-545, 582-590), i.e. nl1 = (n+240)/255 bytes ending
// in n+240-255*nl1; for n < 15 the same formulas give nl1 = 0.
__device__ __forceinline__ uint32_t run_bytes(uint32_t n) { return (n + 240u) / 255u; }
__device__ __forceinline__ uint32_t run_last(uint32_t n, uint32_t nb) { return n + 240u - 255u * nb; }

template <bool kGuard, class Src>
__device__ __forceinline__ int emit_seq(uint8_t* __restrict__ out, int out_cap, int pos, uint32_t token,
                                        uint32_t lit, uint32_t nl1, uint32_t remL, const Src& src,
                                        uint32_t S, uint32_t anchor, bool has_match, uint32_t off,
                                        uint32_t nm1, uint32_t remM) {
  const uint32_t lane = lane_id();
  const uint32_t a = 1u + nl1;                                     // first literal byte
  const uint32_t b = a + lit;                                      // offset low byte
  const uint32_t total = has_match ? b + 2u + nm1 : b;
  // One pass per 64 bytes; every byte class is a compare-select: token,
  // 255-run bytes, remL, literals (one LDS byte read), offset, 255-run, remM.
  // Without a run its "last byte" index falls on a byte of higher precedence
  // (the token, resp. the offset's high byte or a literal).
  const uint32_t remL_at = a - 1u;
  const uint32_t remM_at = total - 1u;
  const int lbase = (int)anchor - (int)a;
#pragma clang loop unroll(disable)
  for (uint32_t i = 0; i < total; i += 64u) {
    const uint32_t j = i + lane;
    const uint32_t lb = src.u8((uint32_t)min(max(lbase + (int)j, 0), (int)S - 1));
    const uint32_t h = j == 0 ? token : (j == remL_at ? remL : 255u);
    const uint32_t t = j == b ? (off & 255u) : j == b + 1u ? (off >> 8) : (j == remM_at ? remM : 255u);
    const uint32_t val = j < a ? h : (j < b ? lb : t);
    if (j < total && (!kGuard || pos + (int)j < out_cap)) out[pos + (int)j] = (uint8_t)val;
  }
  return (int)total;
}

// x in a VGPR (every lane the same value): arithmetic on it is VALU
__device__ __forceinline__ uint32_t vgpr_u32(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Inclusive sum over the wave's 64 lanes (DPP: row shifts inside each row of
// 16, then the row totals broadcast into the rows above).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
  return x;
}


// LZ4_compress_generic (byU16, limitedOutput).  `in` = LDS, value byte i at
// in[i], i < S (every read is clamped into [0, S)).  Returns the block size
// or 0 (limitedOutput failure, checked against `cap` at the reference's check
// points), like the reference.
template <bool kWide, bool kGuard, bool kBatchE = false, bool kLdsOut = false, class Src, class Tab>
__device__ __forceinline__ int compress_block(Src& src, uint32_t S, const Tab& tab,
                                              uint8_t* __restrict__ out, int out_cap, int cap) {
  const uint32_t lane = lane_id();
  int op = 0;
  uint32_t anchor = 0;
  // reads whose result a lane mask discards: clamped into the value only
  // where an out-of-range read could fault (in-place values in HBM)
  constexpr bool kFree = Src::kUnclamped;
#define RD32(p) src.rd32(p)

  if (S >= kMinLength) {                                    // lz4.cc:483
    const uint32_t mflimit = S - kMfLimit;
    const uint32_t matchlimit = S - kLastLiterals;
    const uint32_t last4 = S - 4u;                          // highest position a u32 read may start
    auto clamp4 = [&](uint32_t p) { return kFree ? p : min(p, last4); };
    auto clamp1 = [&](uint32_t p) { return kFree ? p : min(p, S - 1u); };
    // lz4.cc:486: put(0) stores position 0 -- what an empty slot already reads as.
    //
    // After a match ending at ip the reference puts ip-2 (lz4.cc:600), then
    // tests ip (lz4.cc:603-618: get(ip), put(ip), compare; the distance check
    // there always holds for byU16 sizes) -- a search iteration at ip without
    // the skip counter -- and, when that fails, searches afresh from ip+1,
    // whose first 65 iterations advance by 1.  So all of it is the next
    // search chunk, positions ip-2 .. ip+60 ("lead" chunk): lane 0 = ip-2,
    // put only (never a match; later same-slot lanes take it as their
    // reference like any earlier lane); lane 1 = ip-1, dead (no get, no put);
    // lane 2 = ip, the test, valid unconditionally (ip <= mflimit was
    // checked); lanes >= 3 = search iterations 0..60.  A lane-2 match is
    // _next_match: no catch-up, no literals.
    // the search starts at anchor + 1 (lz4.cc:487, 623): no variable of its own
    // the input words of the next sequence's first chunk, read as soon as
    // its start is known (at the end of the sequence before), so the read
    // overlaps that sequence's byte store
    typename Src::Word seq0 = src.rd32_issue(clamp4(1u + lane));
    // In-place values (HBM/L2): a 256-byte register window of the value from
    // each match's start (one dword per lane, loaded with the count's bytes),
    // from which the next sequence's input words and -- one sequence later --
    // its literals come by ds_bpermute instead of two more global round trips
    // per sequence (the chain is then: exchange, candidate word, count).
    // A base of 2^31 marks "no window" (positions stay below 2^31).  byU16
    // values only: for byU32 ones (1 MiB parts) it measured slower (8.47 ->
    // 9.01 ms per 600 x 1 MiB).
    constexpr bool kWin = !kFree && Src::kWindow && (!kWide || (KDB_LZ4_WIDE_WINDOW && Tab::kTagged));
#ifndef KDB_LZ4_SEQ_WINDOW
#define KDB_LZ4_SEQ_WINDOW 1
#endif
#if !KDB_LZ4_SEQ_WINDOW
    uint32_t win = 0, wbase = 0x80000000u, pwin = 0, pbase = 0x80000000u;
#endif
#if KDB_LZ4_SEQ_WINDOW
    // Round 4 (KDB_LZ4_SEQ_WINDOW, the default; 0 = the round-3 window
    // above): one 256-byte window per sequence, loaded at the sequence's
    // start from 64 bytes before its first search position -- an address
    // known before the search -- so it lands with the candidate words, and
    // the count's bytes, the literals and the next sequence's input words
    // come out of it by ds_bpermute whenever they lie in it (near matches:
    // all of G1's).  The sequence's chain is then one global round trip
    // (candidate words and window together) instead of two (the candidate
    // words, then the window's newest line, an HBM miss).  64 KiB x 10 486
    // compress 3.71 -> 3.37 ms, mixed batch 5.34 -> 5.04 ms
    // (profiles/r04_d/r04_u_ab_sequence_window.txt, digest-gated).
    uint32_t sw = 0, sbase = 0x80000000u;
#endif
    // One sequence per call.  The sequence loop runs while anchor < lim_end:
    // mflimit + 1 (lz4.cc:597: a match that ends past mflimit leaves for the
    // last literals), or 0 once a search finds no match (the last literals)
    // or limitedOutput fails (guard_fail) -- a bound, not a status word, so
    // the loop's test is one scalar compare and no flag is carried.  kLead:
    // the search starts with a lead chunk (every sequence but a value's
    // first), so its lane masks are constants.
    uint32_t lim_end = mflimit + 1u;
    bool guard_fail = false;
    // the search's lane bound mflimit - 1 - s + o3 (s = anchor + 1) is
    // kbound - anchor: one scalar subtract (the constants are opaque, or the
    // compiler rebuilds it as two)
    uint32_t kbound0 = mflimit - 2u, kbound1 = mflimit + 1u;
    asm volatile("" : "+s"(kbound0), "+s"(kbound1));
    // the block's bytes, as a buffer resource whose range (2^31 - 1 bytes)
    // only the "past the sequence" offset 2^31 leaves
    const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    // the lead chunk's compare keys (see the search below): lane 0 and 2
    // always valid, lane 1 never; for a match lanes 0 and 1 never
    const int key_put = lane == 1u ? INT32_MAX : (lane == 0u || lane == 2u) ? INT32_MIN : (int)lane;
    const int key_match = lane <= 1u ? INT32_MAX : lane == 2u ? INT32_MIN : (int)lane;
    // Batched emission (round 5; LDS-staged values, no limitedOutput cap):
    // the parse only records each sequence -- lit | ml << 16 and the offset
    // in lane `nseq` of two VGPRs (v_writelane from the SGPRs the search and
    // the count leave) -- and flush_batch() encodes up to 64 sequences at
    // once: one lane per sequence computes its exact run lengths and encoded
    // size, a wave prefix sum gives every sequence's output and input
    // positions, each lane stores its token, run bytes and offset, and the
    // literal runs are copied LDS -> HBM one sequence per wave-wide store.
    // The encoding's ~40 vector instructions per sequence leave the parse's
    // chain.  (lz4.cc:535-592: the same bytes.)
#ifndef KDB_LZ4_BATCH_EMIT
#define KDB_LZ4_BATCH_EMIT 1
#endif
    constexpr bool kBatch = KDB_LZ4_BATCH_EMIT && kBatchE && kFree && !kGuard && !kWide;
    uint32_t rlm = 0, roff = 0;       // lane k: sequence k of the batch (lit | ml << 16, offset)
    uint32_t nseq = 0, banchor = 0;   // sequences recorded; the batch's first anchor
    auto flush_batch = [&]() {
      const bool on = lane < nseq;
      const uint32_t L = on ? (rlm & 0xffffu) : 0u, M = on ? (rlm >> 16) : 0u;
      const uint32_t nl1 = run_bytes(L), nm1 = run_bytes(M);
      // encoded bytes | input bytes << 16 (each total < 2^16: S <= 8 KiB here)
      const uint32_t x = on ? (L + nl1 + nm1 + 3u) | ((L + kMinMatch + M) << 16) : 0u;
      const uint32_t xi = wave_incl_sum(x);
      const uint32_t ex = xi - x;
      const uint32_t o = (uint32_t)op + (ex & 0xffffu);   // the token
      const uint32_t a = banchor + (ex >> 16);             // the literals in the value
      const uint32_t lp = o + 1u + nl1;                    // the literals in the block
      const uint32_t po = lp + L;                          // the offset (LE16)
      auto st8 = [&](uint32_t v, bool w, uint32_t pos) {
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, out_rsrc, w ? (int)pos : (int)0x80000000, 0, 0);
      };
      st8((min(L, kRunMask) << 4) | min(M, kMlMask), on, o);
      st8(roff, on, po);
      st8(roff >> 8, on, po + 1u);
      // the length runs: 255s, then run_last (lz4.cc:539-545, 582-590)
#pragma unroll 1
      for (uint32_t j = 0; ballot(j < max(nl1, nm1)) != 0; ++j) {
        st8(j + 1u == nl1 ? run_last(L, nl1) : 255u, j < nl1, o + 1u + j);
        st8(j + 1u == nm1 ? run_last(M, nm1) : 255u, j < nm1, po + 2u + j);
      }
      // the literals: one wave-wide byte store per sequence (its first 64),
      // in passes of G sequences with their LDS reads issued together (eight
      // while eight are left, then two: a sequence past nseq has L = 0 and
      // stores nothing); the block position goes in the store's scalar
      // offset.  Positions < 2^16: packed.
      const uint32_t la = lp | (a << 16);
      auto lit_pass = [&](uint32_t s0, auto g_c) {
        constexpr uint32_t G = decltype(g_c)::value;
        uint32_t b[G], vo[G], so[G];
#pragma unroll
        for (uint32_t k = 0; k < G; ++k) {
          const uint32_t Ls = readlane(L, s0 + k), pk = readlane(la, s0 + k);
          b[k] = src.u8((pk >> 16) + lane);
          vo[k] = lane < Ls ? lane : 0x80000000u;
          so[k] = pk & 0xffffu;
        }
#pragma unroll
        for (uint32_t k = 0; k < G; ++k)
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b[k], out_rsrc, (int)vo[k], (int)so[k], 0);
      };
      uint32_t s0 = 0;
#pragma unroll 1
      for (; s0 + 8u <= nseq; s0 += 8u) lit_pass(s0, std::integral_constant<uint32_t, 8>{});
#pragma unroll 1
      for (; s0 < nseq; s0 += 2u) lit_pass(s0, std::integral_constant<uint32_t, 2>{});   // s0 + 1 <= 63
      // literal runs longer than 64 bytes (rare): the rest, sequence by sequence
      for (uint64_t lng = ballot(L > 64u); lng; lng &= lng - 1u) {
        const uint32_t s = (uint32_t)__builtin_ctzll(lng);
        const uint32_t Ls = readlane(L, s), pk = readlane(la, s);
#pragma unroll 1
        for (uint32_t j = 64u; j < Ls; j += 64u)
          st8(src.u8((pk >> 16) + j + lane), j + lane < Ls, (pk & 0xffffu) + j + lane);
      }
      op += (int)(readlane(xi, 63) & 0xffffu);
      banchor = anchor;
      nseq = 0;
    };
    // The rest of a sequence once its search found a match (mm: the matching
    // lanes, pk/refk/slot: the chunk's positions, entries and table slots).
    auto finish = [&](uint64_t mm, uint32_t pk, uint32_t refk, const typename Tab::Slot& slot) {
      const uint32_t ks = (uint32_t)__builtin_ctzll(mm);
      uint32_t ip = readlane(pk, ks);
      uint32_t ref = readlane(refk, ks);
      // undo the puts of the lanes after ks (the sequential loop stops at ks):
      // per slot, the lowest such lane holds the entry as lanes <= ks left it
      // -- its refk is a position <= ip (positions grow with the lane; entries
      // from before the chunk are smaller still).  The lanes after ks are the
      // ones with pk > ip, and every lane's refk < pk, so the test is
      // refk <= ip < pk, one unsigned compare: (ip - refk) < (pk - refk).
      // Lanes whose exchange was off (invalid, dead) pass it too: one that
      // read an entry <= ip writes back what the slot holds as of ks (a later
      // lane that overwrote it restores the same entry), and its nibble mask
      // is 0.
      if constexpr (kFree) {
        if (ip - refk < pk - refk) tab.restore(slot, refk);
      }

      // ======== catch up (lz4.cc:531) and LZ4_count (lz4.cc:562-578), issued together
      uint32_t c, ml, ip_end;
      {
        // catch-up bound (lz4.cc:531: ip > anchor, ref > base): 0 for a
        // lane-2 match of a lead chunk (ip == anchor), the _next_match path
        const uint32_t lim = min(ip - anchor, ref);
        const uint32_t rem = matchlimit - (ip + kMinMatch);
        // the reads go out first (lanes past lim / rem read something
        // harmless, clamped into the value only in HBM); the masks are
        // built while they are in flight
        const uint32_t ia = ip - 1u - lane, ra = ref - 1u - lane, ib = ip + kMinMatch + lane;
#if KDB_LZ4_SEQ_WINDOW
        uint32_t a0, b0, a1, b1;
        uint32_t lim_w = lim;
        const uint32_t iw = ip - sbase, rw = ref - sbase;
        if (kWin && max(iw, rw) <= 188u) {
          // the catch-up's ref side has rw bytes before it in the window
          auto wbyte = [&](uint32_t d) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(d & ~3u), (int)sw);
            return (w >> ((d & 3u) << 3)) & 0xffu;
          };
          a0 = wbyte(iw - 1u - lane);
          b0 = wbyte(rw - 1u - lane);
          a1 = wbyte(iw + kMinMatch + lane);
          b1 = wbyte(rw + kMinMatch + lane);
          lim_w = min(lim, rw);
        } else {
          a0 = src.u8(clamp1(ia));
          b0 = src.u8(clamp1(ra));
          a1 = src.u8(clamp1(ib));
          b1 = src.u8(clamp1(ref + kMinMatch + lane));
        }
#else
        const uint32_t lim_w = lim;
        const uint32_t a0 = src.u8(clamp1(ia)), b0 = src.u8(clamp1(ra));
        const uint32_t a1 = src.u8(clamp1(ib));
        const uint32_t b1 = src.u8(clamp1(ref + kMinMatch + lane));
#endif
        // in-place values: the restore (table writes) goes out behind the
        // count's reads (value bytes in HBM, no overlap), so their issue does
        // not wait behind it; it lands before the next sequence's exchange
        // all the same (measured: mixed batch compress -2 %; LDS-staged
        // values restore first, below the search: +1.7 % the other way)
#if !KDB_LZ4_SEQ_WINDOW
        if constexpr (kWin) {
          pwin = win;
          pbase = wbase;
          wbase = ip;
          win = src.rd32(min(ip + 4u * lane, last4));
        }
#endif
        if constexpr (!kFree) {
          if (ip - refk < pk - refk) tab.restore(slot, refk);
        }
        // compares straight into lane masks; lanes past lim / rem vote false:
        // their byte is replaced by 256, which no byte equals.  lane < lim is
        // ia >= anchor and ra >= 0, lane < rem is ib < matchlimit: compares of
        // the read addresses on the vector unit, selects rather than an AND of
        // masks on the CU's one scalar unit (the 256 is opaque so the compiler
        // does not fold the selects back into one)
        uint32_t k256 = 256u, k257 = 257u;           // two, so the nested selects stay two
        asm volatile("" : "+v"(k256), "+v"(k257));
        // (in-place values, whose reads are clamped, compare the lane with
        // lim and rem: measured a little faster there)
        const uint32_t x0 = kFree ? ((int)ra >= 0 ? ((int)ia >= (int)anchor ? a0 : k256) : k257)
                                  : (lane < lim_w ? a0 : k256);
        const uint32_t x1 = kFree ? (ib < matchlimit ? a1 : k256) : (lane < rem ? a1 : k256);
        const int c0 = first_zero_or_neg(__builtin_amdgcn_uicmp(x0, b0, 32 /*EQ*/));
        const int ml0 = first_zero_or_neg(__builtin_amdgcn_uicmp(x1, b1, 32 /*EQ*/));
        c = (uint32_t)c0;
        ml = (uint32_t)ml0;
        // one scalar test for the rare continuations of either count
        if (__builtin_expect((c0 | ml0) < 0 || lim_w < lim, 0)) {
        if (ml0 < 0) {
          ml = 64u;
#pragma unroll 1
          for (;;) {
            const bool l2 = lane < rem - ml;
            const uint32_t x = src.u8(l2 ? ip + kMinMatch + ml + lane : 0u);
            const uint32_t y = src.u8(l2 ? ref + kMinMatch + ml + lane : 0u);
            const uint32_t d = first_zero(ballot(l2 && x == y));
            ml += d;
            if (d < 64u) break;
          }
        }
        const uint32_t cs_ = c0 < 0 ? 64u : (uint32_t)c0;
        c = cs_;
        if (cs_ < lim && (c0 < 0 || cs_ == lim_w)) {
#pragma unroll 1
          for (;;) {
            const bool l2 = lane < lim - c;
            const uint32_t x = src.u8(l2 ? ip - c - 1u - lane : 0u), y = src.u8(l2 ? ref - c - 1u - lane : 0u);
            const uint32_t d = first_zero(ballot(l2 && x == y));
            c += d;
            if (d < 64u) break;
          }
        }
        }
        // the match ends at ip_end whatever the catch-up; the next search
        // starts at ip_end + 1 (lz4.cc:623), i.e. anchor + 1
        ip_end = ip + kMinMatch + ml;
      }
      ip -= c;
      ref -= c;
      ml += c;
      const uint32_t moff = ip - ref;

      // ======== token + literals (lz4.cc:535-550), offset (554), match length (580-592)
      const uint32_t lit = ip - anchor;
      const bool long_ml = ml >= kMlMask;
      if (kGuard) {
        // With cap >= compressBound these checks cannot fire (each sequence's
        // encoding is at most its input + lit/255 bytes, so op stays below
        // anchor + anchor/255 and both sides stay under the bound's 16 spare
        // bytes); the unguarded instantiation omits them.
        const int op_off = op + 1 + (lit >= kRunMask ? (int)((lit - kRunMask) / 255u) + 1 : 0) + (int)lit;
        if (op + 1 + (int)lit + (int)(2 + 1 + kLastLiterals) + (int)(lit / 255u) > cap ||
            (long_ml && op_off + 2 + (int)(1 + kLastLiterals) + (int)(ml >> 8) > cap)) {
          guard_fail = true;
          lim_end = 0;
          return;
        }
      }
      // at most one run byte each (almost every sequence): (n+241)>>8 is
      // (n >= 15), the byte n-15 = bits 7:0 of n+241 (the byte stores keep
      // bits 7:0, so no mask); without a run its "last byte" index falls on a
      // byte of higher precedence, so any value does.  Longer runs -- lit or
      // ml >= 270 -- take the exact run_bytes / run_last.
      if constexpr (kGuard) {
        const uint32_t token = (min(lit, kRunMask) << 4) | min(ml, kMlMask);
        uint32_t nl1 = (lit + 241u) >> 8, nm1 = (ml + 241u) >> 8, remL = lit + 241u, remM = ml + 241u;
        if (max(lit, ml) >= 270u) {
          nl1 = run_bytes(lit);
          nm1 = run_bytes(ml);
          remL = run_last(lit, nl1);
          remM = run_last(ml, nm1);
        }
        const int seq_op = op;
        op += (int)(lit + nl1 + nm1 + 3u);
        emit_seq<kGuard>(out, out_cap, seq_op, token, lit, nl1, remL, src, S, anchor, true, moff, nm1, remM);
        anchor = ip_end;
        seq0 = src.rd32_issue(clamp4(ip_end - 2u + lane));
      } else if constexpr (kBatch) {
        // record the sequence; its bytes are written by flush_batch
        anchor = ip_end;
        seq0 = src.rd32_issue(ip_end - 2u + lane);
        rlm = writelane(lit | (ml << 16), nseq, rlm);
        roff = writelane(moff, nseq, roff);
        ++nseq;
      } else {
        // The encoding's arithmetic on the vector unit, on uniform VGPR
        // copies of lit and ml (the CU's one scalar unit, shared by its
        // waves, is the dearer resource: +8 scalar instructions per sequence
        // cost 6.9 %, +8 vector ones 2.9 %), and op lives in a VGPR too.
        // One scalar test remains: a run of 2+ bytes or an encoding over 64
        // bytes (rare) goes to emit_seq with the exact lengths, after the
        // one-store path has written its first <= 64 bytes (some wrong, all
        // rewritten: the one-store total never exceeds the exact one, and
        // each lane's later store to the same address lands after its
        // earlier one).
        const uint32_t vlit = vgpr_u32(lit), vml = vgpr_u32(ml);
        const uint32_t remL = vlit + 241u, remM = vml + 241u;
        const uint32_t nl1 = remL >> 8, nm1 = remM >> 8;
        const uint32_t etot = vlit + nl1 + nm1 + 3u;  // 1 + nl1 + lit + 2 + nm1
        const int seq_op = op;
        const uint32_t seq_anchor = anchor;
        op = seq_op + (int)etot;
        anchor = ip_end;
        // the next sequence's input words go out before this sequence's
        // bytes, whose literal read shares their round trip
        // byte j of the encoding on lane j: token (0), remL (1 if nl1),
        // literals [a, b) with a = 1 + nl1, b = a + lit, the offset LE16 at
        // b, b+1, remM at b+2 (if nm1); lanes past etot are dropped
        const uint32_t da = (lane - 1u) - nl1;        // lane - a: the lane's literal index
        uint32_t lb;
        if constexpr (!kWin) {
          seq0 = src.rd32_issue(clamp4(ip_end - 2u + lane));
          lb = src.u8(clamp1(seq_anchor + da));
        } else {
          // next input words: bytes ip_end - 2 + lane .. +3, at window offset
          // ml + 2 + lane (ml before the catch-up); covered while ml <= 187
#if KDB_LZ4_SEQ_WINDOW
          const uint32_t pw = ip_end - sbase;
          if (pw <= 190u) {
            const uint32_t d = pw - 2u + lane;
            const uint32_t w0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((d >> 2) << 2), (int)sw);
            const uint32_t w1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((d >> 2) + 1u) << 2), (int)sw);
            seq0 = typename Src::Word{__builtin_amdgcn_alignbyte(w1, w0, d & 3u)};
          } else {
            seq0 = src.rd32_issue(clamp4(ip_end - 2u + lane));
          }
          const uint32_t lo = seq_anchor - sbase;
          if (lo + lit <= 256u) {
            const uint32_t o = lo + da;
            const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((o >> 2) << 2), (int)sw);
            lb = w >> ((o & 3u) << 3);
          } else {
            lb = src.u8(clamp1(seq_anchor + da));
          }
#else
          const uint32_t mw = ip_end - wbase;               // 4 + ml
          if (mw <= 191u) {
            const uint32_t d = mw - 2u + lane;
            const uint32_t w0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((d >> 2) << 2), (int)win);
            const uint32_t w1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((d >> 2) + 1u) << 2), (int)win);
            seq0 = typename Src::Word{__builtin_amdgcn_alignbyte(w1, w0, d & 3u)};
          } else {
            seq0 = src.rd32_issue(clamp4(ip_end - 2u + lane));
          }
          // literals [seq_anchor, seq_anchor + lit): in the previous match's
          // window when they end inside it
          const uint32_t lo = seq_anchor - pbase;
          if (lo + lit <= 256u) {
            const uint32_t o = lo + da;
            const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((o >> 2) << 2), (int)pwin);
            lb = w >> ((o & 3u) << 3);
          } else {
            lb = src.u8(clamp1(seq_anchor + da));
          }
#endif
        }
        const uint32_t head = ((min(vlit, kRunMask) << 4) | min(vml, kMlMask)) | (remL << 8);
        const uint32_t tail = moff | (remM << 16);
        const uint32_t d = da - vlit;                 // lane - b
        uint32_t val = lane < 2u ? head >> (lane << 3) : 255u;
        val = d < 3u ? tail >> (d << 3) : val;
        val = da < vlit ? lb : val;
        if constexpr (kLdsOut) {   // out is LDS (the compress service's result buffer)
          if (lane < etot) ((lds_u8*)(uintptr_t)(lds_off(out) + (uint32_t)seq_op + lane))[0] = (uint8_t)val;
        } else {
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)val, out_rsrc,
                                               lane < etot ? seq_op + (int)lane : (int)0x80000000, 0, 0);
        }
        const int rare = unii((int)(510u - max(remL, remM)) | (64 - (int)etot));
        if (__builtin_expect(rare < 0, 0)) {
          const uint32_t xl = run_bytes(lit), xm = run_bytes(ml);
          const int pos = unii(seq_op);
          emit_seq<false>(out, out_cap, pos, (min(lit, kRunMask) << 4) | min(ml, kMlMask), lit, xl,
                          run_last(lit, xl), src, S, seq_anchor, true, moff, xm, run_last(ml, xm));
          op = pos + (int)(lit + xl + xm + 3u);
        }
      }
    };
    auto sequence = [&](auto lead_c) {
      constexpr uint32_t t0 = decltype(lead_c)::value ? 1u : 0u;
      // the frontier touch (GlobalSrc::step) only for byU32 values: for the
      // byU16 in-place class its load, issued ahead of the search's reads,
      // cost more than it saved (64 KiB 6.51 -> 6.36 ms without it; 1 MiB
      // byU32 9.84 -> 10.71 ms without it, profiles/r02_e40_ab_touch.txt)
      if constexpr (kWide) src.step(anchor + 1u);
#if KDB_LZ4_SEQ_WINDOW
      if constexpr (kWin) {
        const uint32_t cs = anchor + 1u - 3u * (decltype(lead_c)::value ? 1u : 0u);   // the first chunk's start
        sbase = cs >= 64u ? cs - 64u : 0u;
        sw = src.rd32(min(sbase + 4u * lane, last4));
      }
#endif
      // ================= search (lz4.cc:494-527), 64 iterations per step
      // (the loop exits with the chunk that matched; a chunk that runs past
      // mflimit without a match goes to the last literals)
      uint32_t pk, refk;
      typename Tab::Slot slot;
      uint64_t mm, vm;
      const uint32_t o3 = 3u * t0;
      // First chunk (nearly every sequence's only one): step(k) = 1 for k <= 64,
      // so its positions are s-o3+lane.
      // valid lanes (lz4.cc:510): pk + 1 <= mflimit, a compare of the lane
      // index with a scalar bound (no pk in the chain: s <= mflimit + 1, so
      // it is >= -2).  A lead chunk's lanes 0 and 2 are valid whatever the
      // bound (lane 0 puts, lane 2 tests), lane 1 never (dead), and only
      // lanes >= 2 may match: their compare keys (key_put, key_match) make
      // each mask one vector compare, with no scalar mask arithmetic.
      const int bound = (int)((t0 ? kbound1 : kbound0) - anchor);
      {
        pk = anchor + 1u - o3 + lane;
        vm = __builtin_amdgcn_sicmp(t0 ? key_put : (int)lane, bound, 41 /*SLE*/);
        const bool valid = __builtin_amdgcn_inverse_ballot_w64(vm);   // my bit of vm, no VALU
        const uint32_t seq = Src::word(seq0);
        const uint32_t h = hashp<kWide>(seq);
        // get + put of every valid lane at once, in lane order: refk is the
        // entry as the sequential loop's get at this iteration reads it
        bool maybe = true;
        if constexpr (Tab::kTagged) {
          refk = tab.xchg_tagged(h, pk, Tab::tag(seq), valid, slot, maybe);
          maybe = maybe && pk <= refk + kMaxDistance;
        } else {
          refk = tab.xchg(h, pk, valid, slot);
        }
#if KDB_ABL_DUP_CAND
        {  // attribution build: the candidate word read twice (opaque address, so both loads stay)
          uint32_t r2 = refk;
          asm volatile("" : "+v"(r2));
          const uint32_t x = RD32(r2);
          asm volatile("" ::"v"(x));
        }
#endif
        // the lanes whose reference matches (lz4.cc:527, 610-616), as a
        // compare straight into a lane mask (a ballot of a bool would be
        // materialised in a VGPR and compared again); byU32 adds the
        // distance check (lz4.cc:526, 614), byU16 sizes never need it.
        // refk is a position <= mflimit of this value (the table holds
        // nothing else), so its 4 bytes need no clamp.
        uint32_t cw;
        if constexpr (Tab::kTagged) {   // only candidates that may match are read
          cw = ~seq;
          if (maybe) cw = RD32(refk);
        } else {
          cw = RD32(refk);
        }
        mm = __builtin_amdgcn_uicmp(cw, seq, 32 /*EQ*/) &
             (t0 ? __builtin_amdgcn_sicmp(key_match, bound, 41 /*SLE*/) : vm);
        if (kWide) mm &= __builtin_amdgcn_uicmp(pk, refk + kMaxDistance, 37 /*ULE*/);
      }
      // later chunks: no match yet and every lane valid, i.e. lane 63 (else:
      // last literals); the two tests nested, so the common path is one
      // scalar compare and branch
      if (__builtin_expect(mm == 0, 0)) {
       if (bound >= 63) {
        uint32_t kb = 0;
#pragma unroll 1
        for (;;) {
          kb += 64u;
          // k >= 61: the closed form with no k == 0 case
          const uint32_t k = kb + lane - o3;
          pk = search_pos_nz<kWide>(anchor + 1u, k);
          vm = __builtin_amdgcn_uicmp(pk + ((63u + k) >> 6), mflimit, 37 /*ULE*/);
          const bool valid = __builtin_amdgcn_inverse_ballot_w64(vm);
          const uint32_t seq = RD32(clamp4(pk));
          const uint32_t h = hashp<kWide>(seq);
          uint32_t cw;
          if constexpr (Tab::kTagged) {
            bool maybe;
            refk = tab.xchg_tagged(h, pk, Tab::tag(seq), valid, slot, maybe);
            cw = ~seq;
            if (maybe && pk <= refk + kMaxDistance) cw = RD32(refk);
          } else {
            refk = tab.xchg(h, pk, valid, slot);
            cw = RD32(refk);
          }
          mm = __builtin_amdgcn_uicmp(cw, seq, 32 /*EQ*/) & vm;
          if (kWide) mm &= __builtin_amdgcn_uicmp(pk, refk + kMaxDistance, 37 /*ULE*/);
          if ((mm | ~vm) != 0) break;                // a match, or past mflimit
        }
       }
       if (!mm) {
         lim_end = 0;
         return;
       }
       // a later chunk matched: the sequence's rest, a copy of its own (were
       // the paths to join, the compiler would carry a flag across the join)
       finish(mm, pk, refk, slot);
       return;
      }
      finish(mm, pk, refk, slot);
    };
    sequence(std::false_type{});
    // lz4.cc:597 (the match ended past mflimit: the last literals); else the
    // table fill of ip-2 (lz4.cc:600) and the test of ip run as the next
    // (lead) chunk, positions ip-2+lane (seq0 above).  The test is made here,
    // at the branch, so no flag carries it across the sequence's byte store.
#pragma unroll 1
    while (anchor < lim_end) {
      sequence(std::true_type{});
      if constexpr (kBatch) {
        if (nseq == 64u) flush_batch();
      }
    }
    if constexpr (kBatch) {
      if (nseq) flush_batch();
    }
    if (kGuard && guard_fail) return 0;
  }

  {  // the last literals (lz4.cc:625-637)
    const uint32_t run = S - anchor;
    if (kGuard && op + (int)run + 1 + (int)((run + 255u - kRunMask) / 255u) > cap) return 0;
    const uint32_t nl1 = run_bytes(run);
    op += emit_seq<kGuard>(out, out_cap, op, min(run, kRunMask) << 4, run, nl1, run_last(run, nl1), src, S, anchor,
                           false, 0u, 0u, 0u);
  }
#undef RD32
  return unii(op);
}

constexpr uint32_t kSmallMax = 4096u;     // tagged table + register prefetch
// Values from here on take compress_block's batched emission; shorter ones
// (a few sequences: 100-byte values have one or two) emit each sequence as
// it goes -- the batch flush's fixed cost (a prefix sum, the run-byte loop, a
// pass of eight literal stores) is more than their per-sequence emission.
// Two instances of the parse in one kernel, picked per value (a runtime
// choice per sequence inside one instance moved ~12 instructions per
// sequence to the scalar unit: headline compress 8.48 -> 8.83 ms).
#ifndef KDB_LZ4_BATCH_MIN
#define KDB_LZ4_BATCH_MIN 512
#endif
constexpr uint32_t kBatchMin = KDB_LZ4_BATCH_MIN;
constexpr uint32_t kMidLdsMax = 8192u;    // LDS-staged values up to here, in place above
constexpr uint32_t kPrefetch = 4u;        // output chunks per lane: 4096 / 16 / 64

// Stages value bytes g[0 .. n) into LDS at offset 0 (16B-aligned), whatever
// g's alignment: whole aligned 16-byte loads of the chunks that hold value
// bytes (such a chunk never crosses a page, so the over-read cannot fault; the
// funnel's second chunk is loaded only when it holds one too), realigned in
// registers.
__device__ __forceinline__ void stage_aligned(const uint8_t* g, uint32_t n, uint8_t* lds) {
  const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
  const uint4* base = reinterpret_cast<const uint4*>(g - head);
  const uint32_t chunks = (n + 15u) >> 4;
  const uint32_t end = head + n;                 // chunk k holds value bytes iff 16 k < end
  uint4* l = reinterpret_cast<uint4*>(lds);
  for (uint32_t c = lane_id(); c < chunks; c += 64u)
    l[c] = head ? funnel16(base[c], 16u * (c + 1u) < end ? base[c + 1u] : make_uint4(0u, 0u, 0u, 0u), head)
                : base[c];
}

// kFrame = false: LZ4_compress_limitedOutput per value; ret[v] = size or 0,
//   dst slot capacity = cap[v].
// kFrame = true : CompressorLZ4::Compress per value; the slot must hold
//   8 + compress_bound(S) bytes; frame_len[v] = frame bytes, ret[v] = 0 or -1.
//
// The values of [min_len, in_cap] bytes, staged in LDS at `smem` (kSmall:
// the fixed 16 KiB layout -- Table12, then the value; else Table16, then the
// value), taken from the WorkQueue on `work`.
// kEmit: how compress_block emits its sequences -- kEmitDirect (each as it
// goes), kEmitBatch (batched), or kEmitPerValue (two instances of the parse,
// batched for values of kBatchMin bytes and more).
constexpr uint32_t kEmitDirect = 0, kEmitBatch = 1, kEmitPerValue = 2;
// kWaves > 1 (kSmall only): `smem` is this wave's 16 KiB region of a workgroup
// of kWaves independent waves (lz4_compress_kernel), so the workgroup's
// barrier is no business of the value loop: LDS ordering within the wave is
// all it needs (a wave's LDS instructions execute in order).
template <uint32_t kWaves>
__device__ __forceinline__ void value_sync() {
  if constexpr (kWaves == 1) __syncthreads();
  else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
template <bool kFrame, bool kSmall, uint32_t kEmit, uint32_t kWaves = 1>
__device__ __forceinline__ void values_loop(
    uint8_t* const smem, const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t min_len, uint32_t in_cap,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ dst_cap, uint32_t* __restrict__ frame_len,
    int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch, uint32_t nq, uint32_t guide) {
  const uint32_t lane = lane_id();
  uint16_t* tab16 = reinterpret_cast<uint16_t*>(smem);
  constexpr uint32_t kTabBytes = kSmall ? kTable12Bytes : kTableBytes;
  // kSmall: the value at [0, 4 KiB), Table12 after it (see Table12); else
  // Table16, then the value
  uint8_t* s_in = kSmall ? smem : smem + kTabBytes;      // value bytes [0, S), 16B-aligned
  uint8_t* s_tab = kSmall ? smem + kT12Lo : smem;
  const uint4 z4 = make_uint4(0, 0, 0, 0);

  static_assert(kWaves == 1 || kSmall, "multi-wave workgroups: the Table12 class");
  using Tab = typename std::conditional<kSmall, Table12T<(kWaves > 1)>, Table16>::type;
  Tab tab;
  if constexpr (!kSmall) tab = Table16(tab16);
  if constexpr (kSmall && kWaves > 1) tab.base = lds_off(smem);
  // this wave among the launch's (claims spread over the work queues by it)
  const uint32_t vb = kWaves > 1 ? blockIdx.x * kWaves + uni(threadIdx.x >> 6) : blockIdx.x;
  if (kSmall) {
    for (uint32_t i = lane; i < kTabBytes / 16u; i += 64u) reinterpret_cast<uint4*>(s_tab)[i] = z4;
  }

  // register prefetch (kSmall): the next value's realigned 16-byte chunks.
  // (Round 4 tried waiting for them with an explicit vmcnt that leaves the
  // value's last 16 byte stores in flight -- loads into accumulation
  // registers the compiler does not track: digest-identical and no faster,
  // 8.80 -> 8.83 ms, profiles/r04_d/r04_n_ab_counted_wait.txt.)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 pa[kPrefetch], pb[kPrefetch];
  uint32_t p_head = 0, p_chunks = 0;
  WorkQueue wq = WorkQueue::make(work, n, batch, nq, guide, vb, gridDim.x * kWaves);
  uint32_t v = uni(wq.next());
  auto prefetch = [&](uint32_t w) {
    if (w < n) {
      const uint8_t* gp = src + sload(src_off, w);
      p_head = uni((uint32_t)(reinterpret_cast<uintptr_t>(gp) & 15u));
      const uint4* base = reinterpret_cast<const uint4*>(__builtin_assume_aligned(gp - p_head, 16));
      const uint32_t len = sload(src_len, w);
      p_chunks = (len >= min_len && len <= in_cap) ? (len + 15u) >> 4 : 0u;   // other launches' values: none
      // whole-wave 16-byte loads (no per-lane exec masks, so global_load_dwordx4),
      // indices clamped to the last aligned chunk holding value bytes; lanes
      // past p_chunks load data the staging ignores
      if (p_chunks) {
        const uint32_t last = (p_head + len - 1u) >> 4;
#pragma unroll
        for (uint32_t i = 0; i < kPrefetch; ++i) {
          const uint32_t c = lane + 64u * i;
          const uint4 a = base[min(c, last)], b = base[min(c + 1u, last)];
          pa[i] = u32x4{a.x, a.y, a.z, a.w};
          pb[i] = u32x4{b.x, b.y, b.z, b.w};
        }
      }
    }
  };
  if (kSmall) prefetch(v);

  while (v < n) {
    const uint32_t vn = uni(wq.next());    // the next value, one ahead
    const uint32_t S = sload(src_len, v);
    const uint8_t* g = src + sload(src_off, v);
    uint8_t* o = dst + sload(dst_off, v);
    const bool mine = S >= min_len && S <= in_cap;   // else another size class's launch owns it
    if (kSmall) {
      // staging, then the next value's prefetch at ONE place on every path:
      // with two prefetch sites the compiler joined their registers with
      // copies at the loop's latch, and a copy of a register a load is
      // still filling waits for it -- and, vmcnt being in order, for every
      // byte store of the value just compressed
      if (mine) {
#pragma unroll
        for (uint32_t i = 0; i < kPrefetch; ++i) {
          const uint32_t c = lane + 64u * i;
          if (c < p_chunks)
            reinterpret_cast<uint4*>(s_in)[c] =
                funnel16(make_uint4(pa[i].x, pa[i].y, pa[i].z, pa[i].w), make_uint4(pb[i].x, pb[i].y, pb[i].z, pb[i].w),
                         p_head);
        }
      }
      prefetch(vn);                  // the next value's loads fly while this one is parsed
    }
    if (!mine) {
      v = vn;
      continue;
    }
    if (!kSmall) {
      stage_aligned(g, S, s_in);
      for (uint32_t i = lane; i < kTableBytes / 16u; i += 64u) reinterpret_cast<uint4*>(tab16)[i] = z4;
    }
    value_sync<kWaves>();

    const uint32_t bound = compress_bound(S);
    if (!kFrame) {
      const uint32_t cap = uni(dst_cap[v]);
      LdsSrc ls{s_in};
      const bool batch = kEmit == kEmitBatch || (kEmit == kEmitPerValue && S >= kBatchMin);
      const int r = cap < bound ? compress_block<false, true>(ls, S, tab, o, (int)cap, (int)cap)
                    : batch     ? compress_block<false, false, kEmit != kEmitDirect>(ls, S, tab, o, (int)bound, (int)cap)
                                : compress_block<false, false, kEmit == kEmitBatch>(ls, S, tab, o, (int)bound, (int)cap);
      if (lane == 0) ret[v] = r;
    } else {
      LdsSrc ls{s_in};
      const bool batch = kEmit == kEmitBatch || (kEmit == kEmitPerValue && S >= kBatchMin);
      const int r = batch ? compress_block<false, false, kEmit != kEmitDirect>(ls, S, tab, o + 8, (int)bound, (int)bound)
                          : compress_block<false, false, kEmit == kEmitBatch>(ls, S, tab, o + 8, (int)bound, (int)bound);
      if (r <= 0) {                              // compressor.cc:31-34
        if (lane == 0) { ret[v] = -1; frame_len[v] = 0; }
      } else {
        const bool raw = (uint32_t)r > S;        // raw fallback (compressor.cc:40-48)
        const uint32_t stored = raw ? 0u : (uint32_t)r + 8u;
        const uint32_t flen = raw ? S + 8u : stored;
        if (raw) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // block stores land before the raw bytes
          flush_lds_to_global(o + 8, s_in, 0, S);
        }
        if (lane < 8u) {                         // compressor.cc:53-54
          const uint32_t w = lane < 4u ? stored : S;
          o[lane] = (uint8_t)(w >> (8u * (lane & 3u)));
        }
        if (lane == 0) { ret[v] = 0; frame_len[v] = flen; }
      }
    }
    if (kSmall) {                                // a zeroed table per value (lz4.cc:669)
#pragma unroll
      for (uint32_t k = 0; k < kTabBytes / 1024u; ++k) reinterpret_cast<uint4*>(s_tab)[lane + 64u * k] = z4;
    }
    value_sync<kWaves>();
    v = vn;
  }
}

// kWaves (kSmall): waves per workgroup, each compressing its own values in its
// own 16 KiB region.  LDS is handed out in 1 280-byte steps per workgroup
// (tools/probe/lds_occupancy, profiles/r05/r05_occ.txt): a one-wave workgroup
// of 16 KiB takes 13 steps, so 9 fit a CU's 160 KiB; ten waves in one
// workgroup of exactly 160 KiB hold 10 values per CU.
template <bool kFrame, bool kSmall, uint32_t kEmit, uint32_t kWaves = 1>
__global__ __launch_bounds__(64 * kWaves) void lz4_compress_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t min_len, uint32_t in_cap,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ dst_cap, uint32_t* __restrict__ frame_len,
    int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch, const uint32_t* __restrict__ census,
    uint32_t cls, uint32_t nq, uint32_t guide) {
  if (census && census[cls] == 0) return;      // no value of this size class in the batch
  // kSmall: a fixed LDS layout at LDS address 0 (the kernel's only LDS
  // array), so every LDS address is a constant offset (a dynamic
  // allocation's base costs a v_add per address); with several waves, wave w's
  // region at w x 16 KiB
  constexpr uint32_t kStaticLds = kSmall ? (kTable12Bytes + 4096u) * kWaves : 16u;
  static_assert(kStaticLds <= 163840u, "gfx950: 160 KiB of LDS per workgroup");
  __shared__ __attribute__((aligned(16))) uint8_t smem_s[kStaticLds];
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_d[];
  uint8_t* smem = smem_d;
  if constexpr (kSmall) smem = kWaves > 1 ? smem_s + (kTable12Bytes + 4096u) * uni(threadIdx.x >> 6) : smem_s;
  values_loop<kFrame, kSmall, kEmit, kWaves>(smem, src, src_off, src_len, n, min_len, in_cap, dst, dst_off,
                                             dst_cap, frame_len, ret, work, batch, nq, guide);
}

// ---------------------------------------------------------------------------
// The resident compress service (service.h; lz4_decompress.hip has its decode
// twin): one wave serving per-call LZ4_compress_limitedOutput requests
// (lz4.cc:664-682) of values up to kSmallMax bytes from a mailbox in pinned
// host memory -- the value staged at LDS address 0 next to the Table12 planes,
// as lz4_compress_kernel<false, true> stages it, the block written straight to
// the slot in host memory.  Every wave reaches an exit: idle_ticks without a
// request, life_ticks in all, or the host's stop.
// Values up to this size are compressed into LDS first in the compress
// service (a block that fits a reply goes back without waiting for host-memory
// writes: 100 B Compress 3.87-4.13 -> 3.54-3.74 us); longer ones write the slot
// directly (4 KiB through LDS measured 21.7 -> 23.3 us, profiles/r05/r05_sab4_*).
constexpr uint32_t kSvcLdsOutMax = 256u;
__global__ __launch_bounds__(64) void lz4_compress_service_kernel(const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks,
                                                                  uint64_t life_ticks) {
  __shared__ __attribute__((aligned(16))) uint8_t smem_s[kTable12Bytes + kSmallMax];
  // the block, written here first: a short one (<= kSvcInline bytes) goes back
  // in the slot's reply (no wait for host-memory writes to be acknowledged
  // before the done word), a longer one is copied to the slot
  __shared__ __attribute__((aligned(16))) uint8_t s_cout[(kSmallMax + kSmallMax / 255u + 16u + 64u + 15u) & ~15u];
  const uint32_t lane = lane_id();
  uint8_t* s_tab = smem_s + kT12Lo;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  for (uint32_t i = lane; i < kTable12Bytes / 16u; i += 64u) reinterpret_cast<uint4*>(s_tab)[i] = z4;
  __syncthreads();
  Table12 tab;
  const bool reply_on = __hip_atomic_load(&ibox->no_reply, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u;
  // the value staged at LDS [0, S) by svc_loop
  svc_loop(ibox, obox, gen, idle_ticks, life_ticks, smem_s, kSmallMax,
           [&](uint32_t sidx, const SvcArgs& a, const uint8_t** res) -> int {
    const uint32_t S = a.csize, cap = a.osize;
    int rc = (int)kUnsupported;
    if (S <= kSmallMax && cap <= kSvcOutBytes) {
      __syncthreads();
      const uint32_t bound = compress_bound(S);
      LdsSrc ls{smem_s};
      if (S <= kSvcLdsOutMax) {
        // a block that may fit the reply: written to LDS (it never exceeds
        // min(cap, bound) <= sizeof s_cout), then replied, or copied to the slot
        rc = cap < bound ? compress_block<false, true, false, true>(ls, S, tab, s_cout, (int)cap, (int)cap)
                         : compress_block<false, false, false, true>(ls, S, tab, s_cout, (int)bound, (int)cap);
        if (rc > 0 && !(reply_on && svc_replies(sidx, rc)))
          flush_lds_to_global(obox->slot[sidx].out, s_cout, 0, (uint32_t)rc);
        *res = s_cout;   // the reply reads it before the next request's staging
      } else {
        // a longer one straight to the slot, its stores overlapping the parse
        SvcSlot* sl = &obox->slot[sidx];
        rc = cap < bound ? compress_block<false, true>(ls, S, tab, sl->out, (int)cap, (int)cap)
                         : compress_block<false, false>(ls, S, tab, sl->out, (int)bound, (int)cap);
      }
#pragma unroll
      for (uint32_t k = 0; k < kTable12Bytes / 1024u; ++k) reinterpret_cast<uint4*>(s_tab)[lane + 64u * k] = z4;
      __syncthreads();
    }
    return rc;
  });
}

hipError_t launch_compress_service(hipStream_t st, const SvcBox* ibox, SvcBox* obox, uint32_t gen,
                                   uint64_t idle_ticks, uint64_t life_ticks) {
  hipLaunchKernelGGL(lz4_compress_service_kernel, dim3(1), dim3(64), 0, st, ibox, obox, gen, idle_ticks, life_ticks);
  return hipGetLastError();
}

static_assert(kTable12Bytes + kSmallMax <= kOffLaneLds, "Table12 kernels: off lanes must address past the LDS");
static_assert(kTableBytes + kMidLdsMax <= kOffLaneLds, "the LDS-staged class: off lanes must address past the LDS");
static_assert(4096u * 4u <= kOffLaneLds, "Table32 kernels: off lanes must address past the LDS");
// the compact byU32 kernel: Table24T's off lanes address its byte plane at
// off + 8192 + (h | 0x8000), 40 KiB past the table's base, and the ring
// follows the table: everything must stay below that
static_assert(Table24T::kBytes + RingSrcC::kR + RingSrcC::kMirror <= 8192u + 0x8000u,
              "Table24T kernels: off lanes must address past the LDS");
// LDS bytes a launch needs for values up to max_len bytes.
size_t compress_lds_bytes(uint32_t max_len) {
  // 16 KiB: 10 per CU in ten-wave workgroups
  if (max_len <= kSmallMax) return kTable12Bytes + kSmallMax;
  return kTableBytes + (((size_t)max_len + 15u) & ~(size_t)15u);
}

// ---------------------------------------------------------------------------
// Values of 65 547 bytes and more: LZ4_compress_generic(byU32) (lz4.cc:673-676;
// 12-bit hash, u32 positions, distance check).  KingDB's default part size is
// 1 MB (util/options.h:171), so whole parts land here.  The value is read in
// place from global memory (L2), the 16 KiB table lives in LDS; one wave per
// value.  Waves claim up to 16 values at a time and compress the ones of this class.
// kCompact (byU32 launches whose values are all at most kTagMaxLen bytes):
// Table24T and the 2 KiB ring in 14.1 KiB of LDS (10 waves per CU).
template <bool kFrame, bool kWide, bool kCompact = false, uint32_t kWaves = 1>
__device__ __forceinline__ void big_values(
    uint32_t* const tab32, uint8_t* const ring, const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t min_len, uint32_t max_len,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ frame_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch) {
  const uint32_t lane = lane_id();
  // byU32 (kWide): 4096 x u32; byU16: the same 16 KiB as 8192 x u16
  static_assert(kWaves == 1 || !kWide, "multi-wave workgroups: the byU16 table");
  using Tab = typename std::conditional<kWide, Table32, Table16T<(kWaves > 1)>>::type;
  Tab tab;
  if constexpr (kWide) tab = Table32(tab32);
  else tab = Tab(reinterpret_cast<uint16_t*>(tab32));
  const Table32T tabt(tab32);
  const Table24T tabc(tab32);
  static_assert(!kCompact || kWide, "the compact table is byU32's");
  if constexpr (kCompact) max_len = min(max_len, kTagMaxLen);   // every value tagged
  bool direct_done = false;
#pragma unroll 1
  for (;;) {
    uint32_t c0 = 0;
    if (!work) {                                 // direct launch: value <this wave's index>, once
      if (direct_done) break;
      c0 = kWaves > 1 ? blockIdx.x * kWaves + uni(threadIdx.x >> 6) : blockIdx.x;
      direct_done = true;
    } else {
      if (lane == 0) c0 = atomicAdd(work, batch);
      c0 = uni(c0);
    }
    if (c0 >= n) break;
    const uint32_t vi = c0 + lane;
    const bool in_claim = lane < batch && vi < n;
    const uint32_t len = in_claim ? src_len[vi] : 0u;
    uint64_t big = ballot(in_claim && len >= min_len && len <= max_len);
#pragma unroll 1
    while (big) {
      const uint32_t l = (uint32_t)__builtin_ctzll(big);
      big &= big - 1ull;
      const uint32_t v = c0 + l;
      const uint32_t S = readlane(len, l);
      const uint8_t* g = src + src_off[v];
      uint8_t* o = dst + dst_off[v];
      // byU32 values of at most kTagMaxLen bytes (KingDB's 1 MB parts) take the
      // tagged table, whose empty entries hold position 0's tag
      const bool tagged = kWide && S <= kTagMaxLen && S >= 4u;
      if constexpr (kCompact) {
        Table24T::clear(tab32, uni(*reinterpret_cast<const GlobalSrc::u32u*>(g)));
      } else {
        const uint32_t fill = tagged ? Table32T::empty(uni(*reinterpret_cast<const GlobalSrc::u32u*>(g))) : 0u;
        for (uint32_t i = lane; i < 4096u / 4u; i += 64u) reinterpret_cast<uint4*>(tab32)[i] = make_uint4(fill, fill, fill, fill);
      }
      const uint32_t bound = compress_bound(S);                   // 0 past LZ4_MAX_INPUT_SIZE
      GlobalSrc ws{g, S, 0u};
      // compress_block over the value with source R and table T (cap: the
      // caller's; out: o + skip)
      auto run = [&](auto& rsrc, const auto& t, uint32_t skip, int cap, int b) -> int {
        return cap < b ? compress_block<kWide, true>(rsrc, S, t, o + skip, cap, cap)
                       : compress_block<kWide, false>(rsrc, S, t, o + skip, b, cap);
      };
      auto run_any = [&](uint32_t skip, int cap, int b) -> int {
        if constexpr (kCompact) {
          RingSrcC rs{g, S, ring, 0u, {}, {}, false};
          return run(rs, tabc, skip, cap, b);
        } else if constexpr (kWide) {
          if (tagged) {
#if KDB_LZ4_WIDE_RING
            RingSrc rs{g, S, ring, 0u, {}, {}, false};
            return run(rs, tabt, skip, cap, b);
#else
            return run(ws, tabt, skip, cap, b);
#endif
          }
        }
        return run(ws, tab, skip, cap, b);
      };
      if (!kFrame) {
        const uint32_t cap = uni(dst_cap[v]);
        int r = 0;
        if (bound != 0) r = run_any(0u, (int)cap, (int)bound);
        if (lane == 0) ret[v] = r;
      } else {
        const int r = bound == 0 ? 0 : run_any(8u, (int)bound, (int)bound);
        if (r <= 0) {                                             // compressor.cc:31-34
          if (lane == 0) { ret[v] = -1; frame_len[v] = 0; }
        } else {
          const bool raw = (uint32_t)r > S;                       // compressor.cc:40-48
          const uint32_t stored = raw ? 0u : (uint32_t)r + 8u;
          if (raw) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll 1
            for (uint32_t i = lane; i < S; i += 256u) {           // 4 loads in flight per lane
              uint8_t b[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) b[k] = i + 64u * k < S ? g[i + 64u * k] : 0;
#pragma unroll
              for (int k = 0; k < 4; ++k) if (i + 64u * k < S) o[8u + i + 64u * k] = b[k];
            }
          }
          if (lane < 8u) {                                        // compressor.cc:53-54
            const uint32_t w = lane < 4u ? stored : S;
            o[lane] = (uint8_t)(w >> (8u * (lane & 3u)));
          }
          if (lane == 0) { ret[v] = 0; frame_len[v] = raw ? S + 8u : stored; }
        }
      }
    }
  }
}

template <bool kFrame, bool kWide>
__global__ __launch_bounds__(64) void lz4_compress_big_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t min_len, uint32_t max_len,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ frame_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch,
    const uint32_t* __restrict__ census, uint32_t cls, uint32_t prio) {
  if (census && census[cls] == 0) return;      // no value of this size class in the batch
  // the big class is a mixed batch's critical path: its waves win issue
  // arbitration over the small classes' waves that fill the GPU beside them
  if (prio) __builtin_amdgcn_s_setprio(2);
  __shared__ __attribute__((aligned(16))) uint32_t tab32[4096];
  // byU32 values' LDS ring (RingSrc); 16 + 4.06 KiB: 7 waves per CU (LDS)
  __shared__ __attribute__((aligned(16))) uint8_t ring[kWide && KDB_LZ4_WIDE_RING ? RingSrc::kR + RingSrc::kMirror : 16u];
  big_values<kFrame, kWide>(tab32, ring, src, src_off, src_len, n, min_len, max_len, dst, dst_off, dst_cap, frame_len,
                            ret, work, batch);
}

// byU32 launches whose values are all at most kTagMaxLen bytes (KingDB's 1 MiB
// parts): Table24T + the 2 KiB ring, 12 + 2.06 KiB: 10 waves per CU (LDS;
// hipOccupancy says 11, the hardware admits 10: tools/probe/lds_occupancy)
template <bool kFrame>
__global__ __launch_bounds__(64) void lz4_compress_big_compact_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t min_len, uint32_t max_len,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ frame_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch,
    const uint32_t* __restrict__ census, uint32_t cls, uint32_t prio) {
  if (census && census[cls] == 0) return;
  if (prio) __builtin_amdgcn_s_setprio(2);
  __shared__ __attribute__((aligned(16))) uint32_t tab[Table24T::kBytes / 4u];
  __shared__ __attribute__((aligned(16))) uint8_t ring[RingSrcC::kR + RingSrcC::kMirror];
  big_values<kFrame, true, true>(tab, ring, src, src_off, src_len, n, min_len, max_len, dst, dst_off, dst_cap, frame_len,
                                 ret, work, batch);
}

// A batch with values on both sides of 4 KiB .. 8 KiB (a mixed batch): ONE
// persistent launch, in the 16 KiB the small class needs.  Each wave first
// takes the in-place values (8 KiB .. 65 546 B: Table16 over the whole 16
// KiB), which are the long ones, then -- when they are all claimed -- the
// small values (<= 4 KiB, Table12 + staging).  Waves leave the in-place pass
// one by one as its claims run out and go straight to small values, so the
// small class fills the in-place tail instead of competing with its start
// (two concurrent launches split the CUs from the start and left the
// in-place values' last rounds alone on the GPU).
// kWaves: waves per workgroup, each in its own 16 KiB region (10 per CU
// instead of 9, as lz4_compress_kernel).
template <bool kFrame, uint32_t kWaves = 1>
__global__ __launch_bounds__(64 * kWaves) void lz4_compress_mixed_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t big_min, uint32_t big_max,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off, const uint32_t* __restrict__ dst_cap,
    uint32_t* __restrict__ frame_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work_big,
    uint32_t batch_big, uint32_t* __restrict__ work_small, uint32_t batch_small, uint32_t nq) {
  constexpr uint32_t kRegion = kTable12Bytes + kSmallMax;
  static_assert(kRegion * kWaves <= 163840u, "gfx950: 160 KiB of LDS per workgroup");
  __shared__ __attribute__((aligned(16))) uint32_t smem32_all[kRegion * kWaves / 4u];
  uint32_t* smem32 = kWaves > 1 ? smem32_all + kRegion / 4u * uni(threadIdx.x >> 6) : smem32_all;
  big_values<kFrame, false, false, kWaves>(smem32, nullptr, src, src_off, src_len, n, big_min, big_max, dst, dst_off,
                                           dst_cap, frame_len, ret, work_big, batch_big);
  value_sync<kWaves>();
#ifndef KDB_LZ4_MIXED_EMIT
#define KDB_LZ4_MIXED_EMIT kEmitPerValue
#endif
  // the small pass: 100-byte and 4 KiB values together, each its own form
  values_loop<kFrame, true, KDB_LZ4_MIXED_EMIT, kWaves>(reinterpret_cast<uint8_t*>(smem32), src, src_off, src_len, n, 0u,
                                                        kSmallMax, dst, dst_off, dst_cap, frame_len, ret, work_small,
                                                        batch_small, nq, 0u);
}

// Values per size class (len <= b0, <= b1, <= b2, above), so that a class
// launch with nothing to do returns at once instead of scanning the batch.
__global__ void class_census_kernel(const uint32_t* __restrict__ len, uint32_t n, uint32_t b0, uint32_t b1,
                                    uint32_t b2, uint32_t* __restrict__ counts) {
  uint32_t c[4] = {0, 0, 0, 0};
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const uint32_t L = len[v];
    c[L <= b0 ? 0 : L <= b1 ? 1 : L <= b2 ? 2 : 3]++;
  }
  // per block: the waves' sums in LDS, then one atomic per class (one per
  // wave and class, on a grid of 1 024 blocks -- 16 Ki same-address atomics
  // for 1 Mi values -- took 92 us of a mixed batch's compress step)
  __shared__ uint32_t part[4][4];
  const uint32_t w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t x = c[k];
    for (int d = 32; d >= 1; d >>= 1) x += (uint32_t)__shfl_xor((int)x, d);
    if (lane_id() == 0) part[w][k] = x;
  }
  __syncthreads();
  if (threadIdx.x < 4u) {
    uint32_t x = 0;
    for (uint32_t i = 0; i < (blockDim.x >> 6); ++i) x += part[i][threadIdx.x];
    if (x) atomicAdd(&counts[threadIdx.x], x);
  }
}

template <bool F, bool Sm, uint32_t Em, uint32_t W = 1>
static hipError_t launch_one(hipStream_t st, size_t lds, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* src_len, uint32_t n, uint32_t min_len, uint32_t in_cap, uint8_t* dst,
                             const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                             int32_t* ret, const uint32_t* census = nullptr, uint32_t cls = 0,
                             uint32_t guide = 0) {
  static_assert(W == 1 || Sm, "multi-wave workgroups: the <= 4 KiB class");
  auto kern = lz4_compress_kernel<F, Sm, Em, W>;
  // see kOffLaneLds: the off lanes' first address (Table12 at kT12Lo in the
  // static 16 KiB; Table16 at the dynamic allocation, after the 16 static
  // bytes) must lie past the whole allocation
  const size_t alloc = (Sm ? kTable12Bytes + kSmallMax : 16u) + lds;
  const size_t off_lane = Sm ? kOffLaneLds + kT12Lo : 16u + kOffLaneLds;
  if (W == 1 && alloc > off_lane) return hipErrorInvalidValue;
  if (W > 1 && lds != 0) return hipErrorInvalidValue;   // static LDS only (kOffLaneWG: nothing past 160 KiB)
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), lds, n, W);
  uint32_t* work = nullptr;
  hipError_t e = launch_counter(st, n, grid * W, &work);   // (waves >= values: wave b takes value b)
  if (e != hipSuccess) return e;
  const uint32_t batch = claim_batch(n, grid * W);
  // the rocprof (demangled) name
  static const char* const names[2][2][3] = {
      {{"lz4_compress_kernel<false, false, 0u, 1u>", "lz4_compress_kernel<false, false, 1u, 1u>",
        "lz4_compress_kernel<false, false, 2u, 1u>"},
       {"lz4_compress_kernel<false, true, 0u, 1u>", "lz4_compress_kernel<false, true, 1u, 1u>",
        "lz4_compress_kernel<false, true, 2u, 1u>"}},
      {{"lz4_compress_kernel<true, false, 0u, 1u>", "lz4_compress_kernel<true, false, 1u, 1u>",
        "lz4_compress_kernel<true, false, 2u, 1u>"},
       {"lz4_compress_kernel<true, true, 0u, 1u>", "lz4_compress_kernel<true, true, 1u, 1u>",
        "lz4_compress_kernel<true, true, 2u, 1u>"}}};
  static const std::string multi = std::string("lz4_compress_kernel<") + (F ? "true" : "false") + ", true, " +
                                   std::to_string(Em) + "u, " + std::to_string(W) + "u>";
  launch_note(W > 1 ? multi.c_str() : names[F][Sm][Em]);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * W), lds, st, src, src_off, src_len, n, min_len, in_cap, dst, dst_off,
                     dst_cap, frame_len, ret, work, batch, census, cls, work_queues(in_cap), guide);
  e = hipGetLastError();
  const hipError_t r = work_counter_release(st, work);   // the slot is fenced even when the launch failed
  return e != hipSuccess ? e : r;
}

template <bool F, bool W>
static hipError_t launch_big(hipStream_t st, const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                             uint32_t n, uint32_t min_len, uint32_t max_len, uint8_t* dst, const uint64_t* dst_off,
                             const uint32_t* dst_cap, uint32_t* frame_len, int32_t* ret,
                             const uint32_t* census = nullptr, uint32_t cls = 0) {
  // byU32 values all within the tagged table's reach: the compact kernel
  static const bool compact_on = kdb_tune("KDB_LZ4_COMPACT", 1) != 0;   // 0: the 16 KiB table (A/B)
  const bool compact = W && compact_on && max_len <= kTagMaxLen;
  auto kern = compact ? lz4_compress_big_compact_kernel<F> : lz4_compress_big_kernel<F, W>;
  static const uint32_t prio = env_prio();
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), 0, n);
  uint32_t* work = nullptr;
  hipError_t e = launch_counter(st, n, grid, &work);
  if (e != hipSuccess) return e;
  const uint32_t batch = work ? claim_batch(n, grid) : 1u;   // values per claim; lanes >= batch idle
  launch_note(compact ? (F ? "lz4_compress_big_compact_kernel<true>" : "lz4_compress_big_compact_kernel<false>")
              : F ? (W ? "lz4_compress_big_kernel<true, true>" : "lz4_compress_big_kernel<true, false>")
                : (W ? "lz4_compress_big_kernel<false, true>" : "lz4_compress_big_kernel<false, false>"));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, st, src, src_off, src_len, n, min_len, max_len, dst, dst_off,
                     dst_cap, frame_len, ret, work, batch, census, cls, prio);
  e = hipGetLastError();
  const hipError_t r = work_counter_release(st, work);
  return e != hipSuccess ? e : r;
}

#ifndef KDB_LZ4_MIXED_WAVES
#define KDB_LZ4_MIXED_WAVES 10
#endif
template <bool F>
static hipError_t launch_mixed(hipStream_t st, const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                               uint32_t n, uint32_t big_min, uint32_t big_max, uint8_t* dst, const uint64_t* dst_off,
                               const uint32_t* dst_cap, uint32_t* frame_len, int32_t* ret) {
  constexpr uint32_t W = KDB_LZ4_MIXED_WAVES;
  auto kern = lz4_compress_mixed_kernel<F, W>;
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), 0, n, W);
  uint32_t *wb = nullptr, *ws = nullptr;
  hipError_t e = launch_counter(st, n, grid * W, &wb);
  if (e == hipSuccess) e = launch_counter(st, n, grid * W, &ws);
  if (e == hipSuccess) {
    const uint32_t bb = wb ? claim_batch(n, grid * W) : 1u, bs = claim_batch(n, grid * W);
    static_assert(W == 1 || W == 10, "the rocprof names below");
    launch_note(W > 1 ? (F ? "lz4_compress_mixed_kernel<true, 10u>" : "lz4_compress_mixed_kernel<false, 10u>")
                      : (F ? "lz4_compress_mixed_kernel<true, 1u>" : "lz4_compress_mixed_kernel<false, 1u>"));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * W), 0, st, src, src_off, src_len, n, big_min, big_max, dst, dst_off,
                       dst_cap, frame_len, ret, wb, bb, ws, bs, work_queues(kSmallMax));
    e = hipGetLastError();
  }
  const hipError_t r1 = work_counter_release(st, wb), r2 = work_counter_release(st, ws);
  return e != hipSuccess ? e : r1 != hipSuccess ? r1 : r2;
}

// One launch per size class that [min_len, max_len] (the launch's bounds on
// its values' lengths; the batch API passes min_len 0) intersects: <= 4 KiB
// (two-plane table, 16 KiB LDS), 4 KiB .. 8 KiB (LDS-staged), 8 KiB .. 65 546 B
// (in place, byU16), >= 65 547 B (byU32, in place).  Each launch skips the
// other classes' values; with several classes a census kernel lets a class
// launch with nothing to do return at once.
hipError_t launch_compress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                           const uint32_t* src_len, uint32_t n, uint32_t min_len, uint32_t max_len, uint8_t* dst,
                           const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                           int32_t* ret) {
  launch_notes_reset();
  if (n == 0) return hipSuccess;
  if (min_len > max_len) min_len = 0;
  // the exchange tables' lane order, verified on this device before its first
  // frame (selftest.hip); a device without it compresses nothing
  hipError_t e = lane_order_ok();
  if (e != hipSuccess) return e;
  static const uint32_t mid_split = (uint32_t)kdb_tune("KDB_LZ4_CSPLIT", kMidLdsMax);
  // top of the LDS-staged class; at most 48 KiB: Table16's off lanes address
  // 64 KiB past the table, which must lie past the staged value too (a
  // tuning split of 65 546 measured wrong frames, profiles/r04_d/r04_cs_*)
  const uint32_t b1 = min(max(mid_split, kSmallMax), min(k64KLimit - 1u, 65536u - kTableBytes));
  // class c covers lengths [lo[c], hi[c]]
  const uint32_t lo[4] = {0u, kSmallMax + 1u, b1 + 1u, k64KLimit};
  const uint32_t hi[4] = {kSmallMax, b1, k64KLimit - 1u, 0xFFFFFFFFu};
  bool on[4];
  uint32_t classes = 0;
  for (int c = 0; c < 4; ++c) {
    on[c] = lo[c] <= hi[c] && max_len >= lo[c] && min_len <= hi[c];
    classes += on[c] ? 1u : 0u;
  }
  uint32_t* census = nullptr;            // per-class counts, when more than one class launches
  if (classes > 1) {
    e = work_counter(st, &census);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(class_census_kernel, dim3(min((n + 255u) / 256u, 256u)), dim3(256), 0, st, src_len, n,
                       kSmallMax, b1, k64KLimit - 1u, census);
  }
  // The in-place classes (8 KiB .. 65 546 B, and byU32) go first, on a
  // forked stream when smaller classes follow: their values take longest,
  // and the small classes fill the GPU around their tail.  With both the
  // small and the byU16 in-place class, one launch takes both
  // (lz4_compress_mixed_kernel: in-place values first, then the small ones).
  static const bool combo_on = kdb_tune("KDB_LZ4_CMIXED", 1) != 0;   // 0: separate class launches (A/B)
  const bool combo = combo_on && on[0] && on[2];
  hipStream_t aux = st;
  const bool fork = combo ? on[3] : ((on[2] || on[3]) && (on[0] || on[1]));
  // The class launches stop at the first error, but the join of the forked
  // stream and the census slot's fence always follow: a caller that reuses
  // its buffers after an error must not race a kernel still queued on aux.
  auto classes_run = [&]() -> hipError_t {
    hipError_t r = hipSuccess;
    if (combo) {
      r = frame ? launch_mixed<true>(st, src, src_off, src_len, n, lo[2], hi[2], dst, dst_off, dst_cap, frame_len, ret)
                : launch_mixed<false>(st, src, src_off, src_len, n, lo[2], hi[2], dst, dst_off, dst_cap, frame_len, ret);
      if (r != hipSuccess) return r;
    }
    if (on[2] && !combo) {
      r = frame ? launch_big<true, false>(aux, src, src_off, src_len, n, lo[2], hi[2], dst, dst_off, dst_cap, frame_len,
                                          ret, census, 2)
                : launch_big<false, false>(aux, src, src_off, src_len, n, lo[2], hi[2], dst, dst_off, dst_cap,
                                           frame_len, ret, census, 2);
      if (r != hipSuccess) return r;
    }
    if (on[3]) {
      // the caller's max_len bounds this class's values (the compact kernel's
      // test).  Host code takes no min() here: HIP's host min() on uint32_t is
      // the signed one (min(x, 0xFFFFFFFFu) == 0xFFFFFFFFu)
      const uint32_t top = max_len < hi[3] ? max_len : hi[3];
      r = frame ? launch_big<true, true>(aux, src, src_off, src_len, n, lo[3], top, dst, dst_off, dst_cap,
                                         frame_len, ret, census, 3)
                : launch_big<false, true>(aux, src, src_off, src_len, n, lo[3], top, dst, dst_off, dst_cap,
                                          frame_len, ret, census, 3);
      if (r != hipSuccess) return r;
    }
    if (on[0] && !combo) {
      const size_t lds = 0;   // static LDS (compress_lds_bytes(kSmallMax) bytes)
      const uint32_t guide = claim_guide(max_len < kSmallMax ? max_len : kSmallMax);
      // batched emission when the launch may hold values of kBatchMin bytes
      // and more (a launch of short values only keeps the per-sequence form)
      const bool bat = max_len >= kBatchMin;
      // ten waves per workgroup (10 values per CU instead of 9, see
      // lz4_compress_kernel); KDB_LZ4_WG10=0 (tuning builds): one
#ifndef KDB_LZ4_WG10_DEFAULT
#define KDB_LZ4_WG10_DEFAULT 1
#endif
      // waves per workgroup: 10 (one 160 KiB workgroup per CU), or 5 for A/B:
      // two 80 KiB workgroups would make the same 10 per CU by the 1 280-byte
      // step rule, but the hardware admitted one -- compress 8.0 -> 15.1 ms
      // (profiles/r06/r06_n_w5.txt)
#ifndef KDB_LZ4_CWAVES
#define KDB_LZ4_CWAVES 10
#endif
      constexpr uint32_t CW = KDB_LZ4_CWAVES;
      static_assert(CW == 5 || CW == 10, "16 KiB regions: 5 or 10 per 160 KiB");
      static const bool wg10 = kdb_tune("KDB_LZ4_WG10", KDB_LZ4_WG10_DEFAULT) != 0;
      if (wg10)
        r = frame ? (bat ? launch_one<true, true, kEmitBatch, CW>(st, lds, src, src_off, src_len, n, 0u, kSmallMax, dst,
                                                                  dst_off, dst_cap, frame_len, ret, census, 0, guide)
                         : launch_one<true, true, kEmitDirect, CW>(st, lds, src, src_off, src_len, n, 0u, kSmallMax, dst,
                                                                   dst_off, dst_cap, frame_len, ret, census, 0, guide))
                  : (bat ? launch_one<false, true, kEmitBatch, CW>(st, lds, src, src_off, src_len, n, 0u, kSmallMax,
                                                                   dst, dst_off, dst_cap, frame_len, ret, census, 0, guide)
                         : launch_one<false, true, kEmitDirect, CW>(st, lds, src, src_off, src_len, n, 0u, kSmallMax,
                                                                    dst, dst_off, dst_cap, frame_len, ret, census, 0,
                                                                    guide));
      else
      r = frame ? (bat ? launch_one<true, true, kEmitBatch>(st, lds, src, src_off, src_len, n, 0u, kSmallMax, dst,
                                                            dst_off, dst_cap, frame_len, ret, census, 0, guide)
                       : launch_one<true, true, kEmitDirect>(st, lds, src, src_off, src_len, n, 0u, kSmallMax, dst,
                                                             dst_off, dst_cap, frame_len, ret, census, 0, guide))
                : (bat ? launch_one<false, true, kEmitBatch>(st, lds, src, src_off, src_len, n, 0u, kSmallMax, dst,
                                                             dst_off, dst_cap, frame_len, ret, census, 0, guide)
                       : launch_one<false, true, kEmitDirect>(st, lds, src, src_off, src_len, n, 0u, kSmallMax, dst,
                                                              dst_off, dst_cap, frame_len, ret, census, 0, guide));
      if (r != hipSuccess) return r;
    }
    // 4 KiB .. 8 KiB: the value staged in LDS (24 KiB with the table: 6 per CU);
    // 8 KiB .. 65 546 B: read in place from HBM/L2 with only the table in LDS
    // (10 per CU by hipOccupancy, 9 by the 1 280-byte LDS steps) -- measured
    // faster than 2-5 LDS-staged values per CU.
    if (on[1]) {
      const uint32_t top = max_len < hi[1] ? max_len : hi[1];   // (host min() is signed)
      const size_t lds = compress_lds_bytes(top);
      // Beside a byU32 launch this class queues behind it on aux: its 24 KiB
      // workgroups cannot start while the byU32 waves hold the CUs' LDS, and
      // waiting in the dispatcher next to them they cost the byU32 launch
      // 1.4 ms even with no value of their own (1 MiB parts: compress 12.6 ->
      // 11.1 ms without the fork, profiles/r05/r05_nf_*)
      hipStream_t s1 = on[3] ? aux : st;
      r = frame ? launch_one<true, false, kEmitBatch>(s1, lds, src, src_off, src_len, n, lo[1], top, dst, dst_off,
                                                      dst_cap, frame_len, ret, census, 1, claim_guide(top))
                : launch_one<false, false, kEmitBatch>(s1, lds, src, src_off, src_len, n, lo[1], top, dst, dst_off,
                                                       dst_cap, frame_len, ret, census, 1, claim_guide(top));
    }
    return r;
  };
  e = fork ? fork_begin(st, &aux) : hipSuccess;
  if (e == hipSuccess) e = classes_run();
  const hipError_t j = fork ? fork_end(st, aux) : hipSuccess;          // aux == st when fork_begin failed
  const hipError_t c = work_counter_release(st, census);                // its readers are all joined into st
  if (e == hipSuccess) e = j;
  if (e == hipSuccess) e = c;
  return e;
}

}  // namespace kdb_lz4
