// kingdb_amd/csrc/lz4_compress.hip -- gfx950 LZ4 r1.3.0 block compressor.
//
// Replaces LZ4_compress_limitedOutput (/root/reference/algorithm/lz4.cc:664-682)
// = LZ4_compress_generic(limitedOutput, byU16, noDict, noDictIssue)
// (lz4.cc:431-641), fused with CompressorLZ4::Compress's frame epilogue
// (algorithm/compressor.cc:26-59).  Output is byte-identical to the reference.
//
// Persistent launch: one wavefront (workgroup of 64) per resident slot takes
// values from a device-scope work counter, one value ahead.  LDS per workgroup: the byU16 hash table
// (8192 x u16), the staged value and the block being assembled (flushed to HBM
// with 16-byte stores).  For launches whose values are all <= 4 KiB the table
// carries a 4-bit generation tag beside each 12-bit position, so it is cleared
// once per 15 values instead of per value (a stale tag reads as the zeroed
// slot, position 0 -- lz4.cc:669 semantics), and the next value is prefetched
// into registers while the current one is parsed.
//
// The greedy parse is sequential by definition; what is parallel is:
//  * the search loop (lz4.cc:494-527): the positions it visits from a start
//    `s` are a closed-form function of the iteration index (step =
//    nb++ >> SKIPSTRENGTH), so 64 iterations are evaluated at once, one per
//    lane.  An iteration's table read must see every earlier iteration's put:
//    lanes with the same 13-bit hash are grouped with 13 ballots (bit-sliced
//    match-any) and a lane takes its reference from the nearest lower lane of
//    its group, else from the table as it stood before the chunk.  The first
//    matching lane ends the chunk; only puts of lanes up to it are committed
//    (the last lane of each group writes), exactly the table state the
//    sequential loop would leave;
//  * the catch-up loop (lz4.cc:531) and LZ4_count (lz4.cc:562-578), issued
//    together: the match length after catching up c bytes is c + the length
//    measured from the original position, so neither waits for the other;
//  * literal copies and length-byte runs.
#include <cstdio>

#include "lz4_device.h"

namespace kdb_lz4 {

// Position visited at iteration k of a search run started at s (lz4.cc:497-507):
// p(0)=s, p(k+1)=p(k)+step(k), step(0)=1, step(k)=(63+k)>>6 for k>=1, i.e.
// p(k) = s + 1 + sum_{t=64}^{62+k} floor(t/64) for k >= 1.
__device__ __forceinline__ uint32_t search_pos(uint32_t s, uint32_t k) {
  if (k == 0) return s;
  const uint32_t nn = 62u + k, q = nn >> 6, r = nn & 63u;
  return s + 1u + 32u * q * (q - 1u) + q * (r + 1u);
}
__device__ __forceinline__ uint32_t search_step(uint32_t k) { return k == 0 ? 1u : (63u + k) >> 6; }

__device__ __forceinline__ uint32_t hash16(uint32_t seq) { return (seq * 2654435761u) >> 19; }

// The byU16 table.  kTagged: entry = gen << 12 | pos (values <= 4 KiB, so
// positions < 4096); an entry of another generation is an empty slot (0).
template <bool kTagged>
struct Table {
  uint16_t* t;
  uint32_t gen;
  __device__ __forceinline__ uint32_t get(uint32_t h) const {
    const uint32_t e = t[h];
    if (kTagged) return (e >> 12) == gen ? (e & 0xfffu) : 0u;
    return e;
  }
  __device__ __forceinline__ void put(uint32_t h, uint32_t p) const {
    t[h] = (uint16_t)(kTagged ? ((gen << 12) | p) : p);
  }
};

// Output: the block is assembled in LDS (out[0..out_cap)) and flushed to HBM
// once complete.  kGuard (LZ4_compress_limitedOutput with a caller cap below
// the bound): never write at or past out_cap -- the reference may, on
// limitedOutput failures; the return value is what parity is about (see
// oracle/lz4_oracle.c).  Without kGuard the cap is the bound, which the block
// never exceeds.
template <bool kGuard>
__device__ __forceinline__ void put8(uint8_t* out, int out_cap, int pos, uint32_t b) {
  if (!kGuard || (uint32_t)pos < (uint32_t)out_cap) out[pos] = (uint8_t)b;
}

// Lanes 0..nb write a length continuation (nb 255s then `rem`) at out[pos..].
template <bool kGuard>
__device__ __forceinline__ void put_len(uint8_t* out, int out_cap, int pos, uint32_t nb, uint32_t rem) {
  const uint32_t lane = lane_id();
#pragma unroll 1
  for (uint32_t i = 0; i <= nb; i += 64u) {
    const uint32_t j = i + lane;
    if (j <= nb) put8<kGuard>(out, out_cap, pos + (int)j, j < nb ? 255u : rem);
  }
}

// out[pos .. pos+n) = in[a .. a+n), 64 bytes per step.
template <bool kGuard>
__device__ __forceinline__ void put_bytes(uint8_t* out, int out_cap, int pos, const uint8_t* in, uint32_t a,
                                          uint32_t n) {
#ifdef KDB_ABL_NO_EMIT
  return;
#endif
  const uint32_t lane = lane_id();
#pragma unroll 1
  for (uint32_t i = 0; i < n; i += 64u) {
    const uint32_t j = i + lane;
    const uint32_t b = in[a + j];
    if (j < n) put8<kGuard>(out, out_cap, pos + (int)j, b);
  }
}

// LZ4_compress_generic (byU16, limitedOutput).  `in` = LDS, value byte i at
// in[i]; in_base/head: the 16B-aligned buffer and the offset of byte 0; the
// buffer is readable well past S, so reads are issued unconditionally and
// masked afterwards.  Returns the block size or 0 (limitedOutput failure,
// checked against `cap` at the reference's check points), like the reference.
template <bool kTagged, bool kGuard>
__device__ int compress_block(const uint8_t* __restrict__ in, const uint8_t* in_base, uint32_t head,
                              uint32_t S, const Table<kTagged>& tab, uint8_t* __restrict__ out, int out_cap,
                              int cap) {
  const uint32_t lane = lane_id();
  int op = 0;
  uint32_t anchor = 0;
#define RD32(p) lds_rd32(in_base, head + (p))

  if (S >= kMinLength) {                                    // lz4.cc:483
    const uint32_t mflimit = S - kMfLimit;
    const uint32_t matchlimit = S - kLastLiterals;
    // lz4.cc:486: put(0) stores position 0 -- what an empty slot already reads as.
    uint32_t s = 1;                                         // lz4.cc:487
    for (;;) {
      // ================= search (lz4.cc:494-527), 64 iterations per step
      uint32_t ip = 0, ref = 0;
      bool found = false;
#pragma unroll 1
      for (uint32_t kb = 0;; kb += 64u) {
        const uint32_t k = kb + lane;
        const uint32_t pk = search_pos(s, k);
        const bool valid = pk + search_step(k) <= mflimit;         // lz4.cc:510
        const uint32_t seq = RD32(pk);
        const uint32_t h = hash16(seq);
        const uint32_t told = tab.get(h);
        const uint64_t vm = __ballot(valid);
        // lanes of this chunk whose iteration hashes to the same slot
        uint32_t lo = ~0u, hi = ~0u;
#pragma unroll
        for (int b = 0; b < 13; ++b) {
          const uint32_t t = (uint32_t)((int32_t)(h << (31 - b)) >> 31);   // 0 or ~0
          const uint64_t m = __ballot(t != 0u);
          lo &= ~(t ^ (uint32_t)m);
          hi &= ~(t ^ (uint32_t)(m >> 32));
        }
        const uint64_t same = (((uint64_t)hi << 32) | lo) & vm;
        const uint64_t below = same & mask_lt(lane);
        const uint32_t refk = below ? search_pos(s, kb + 63u - (uint32_t)__builtin_clzll(below)) : told;
        const bool match = valid && RD32(refk) == seq;           // lz4.cc:527
        const uint64_t mm = __ballot(match);
        if (mm) {
          const uint32_t ks = (uint32_t)__builtin_ctzll(mm);
          const uint64_t later = same & ~mask_le(lane) & mask_le(ks);
          if (valid && lane <= ks && later == 0) tab.put(h, pk);   // lz4.cc:526
          ip = readlane(pk, ks);
          ref = readlane(refk, ks);
          found = true;
          break;
        }
        if (vm != ~0ull) break;              // ran past mflimit: last literals
        if ((same & ~mask_le(lane)) == 0) tab.put(h, pk);
      }
      if (!found) break;

      bool catchup = true;
#pragma unroll 1
      for (;;) {  // one sequence per iteration; `continue` = _next_match with no literals
        // ======== catch up (lz4.cc:531) and LZ4_count (lz4.cc:562-578), issued together
        uint32_t c, ml;
        {
          const uint32_t lim = catchup ? min(ip - anchor, ref) : 0u;
          const uint32_t rem = matchlimit - (ip + kMinMatch);
          const uint32_t a0 = in[ip - 1u - lane], b0 = in[ref - 1u - lane];
          const uint32_t a1 = in[ip + kMinMatch + lane], b1 = in[ref + kMinMatch + lane];
          c = first_zero(__ballot(lane < lim && a0 == b0));      // <= lim
          ml = first_zero(__ballot(lane < rem && a1 == b1));     // <= rem
          if (c == 64u) {
#pragma unroll 1
            for (;;) {
              const uint32_t x = in[ip - c - 1u - lane], y = in[ref - c - 1u - lane];
              const uint32_t d = first_zero(__ballot(lane < lim - c && x == y));
              c += d;
              if (d < 64u) break;
            }
          }
          if (ml == 64u) {
#pragma unroll 1
            for (;;) {
              const uint32_t x = in[ip + kMinMatch + ml + lane], y = in[ref + kMinMatch + ml + lane];
              const uint32_t d = first_zero(__ballot(lane < rem - ml && x == y));
              ml += d;
              if (d < 64u) break;
            }
          }
        }
        const uint32_t ip_end = ip + kMinMatch + ml;  // independent of the catch-up
        ip -= c;
        ref -= c;
        ml += c;

        // ======== token + literals (lz4.cc:535-550), offset (554), match length (580-592)
        const uint32_t lit = ip - anchor;
        const int tok_pos = op;
        op += 1;
        if ((int64_t)op + lit + (2 + 1 + kLastLiterals) + lit / 255u > (int64_t)cap) return 0;
        uint32_t token = (lit >= kRunMask ? kRunMask : lit) << 4;
        if (lit >= kRunMask) {
          const uint32_t nb = (lit - kRunMask) / 255u;
          put_len<kGuard>(out, out_cap, op, nb, lit - kRunMask - 255u * nb);
          op += (int)nb + 1;
        }
        put_bytes<kGuard>(out, out_cap, op, in, anchor, lit);
        op += (int)lit;
        const uint32_t off = ip - ref;
        if (lane < 2u) put8<kGuard>(out, out_cap, op + (int)lane, lane ? (off >> 8) : (off & 255u));
        op += 2;
        if (ml >= kMlMask) {
          if ((int64_t)op + (1 + kLastLiterals) + (ml >> 8) > (int64_t)cap) return 0;
          token += kMlMask;
          const uint32_t nb = (ml - kMlMask) / 255u;
          put_len<kGuard>(out, out_cap, op, nb, ml - kMlMask - 255u * nb);
          op += (int)nb + 1;
        } else {
          token += ml;
        }
        if (lane == 0) put8<kGuard>(out, out_cap, tok_pos, token);
        ip = ip_end;
        anchor = ip;
        if (ip > mflimit) goto last_literals;                      // lz4.cc:597

        // ======== fill table + test next position (lz4.cc:600-624)
        const uint32_t sm2 = RD32(ip - 2u);
        const uint32_t sq = RD32(ip);
        const uint32_t hh = hash16(sq);
        if (lane == 0) tab.put(hash16(sm2), ip - 2u);
        const uint32_t r2 = uni(tab.get(hh));
        if (lane == 0) tab.put(hh, ip);
        if (r2 + kMaxDistance >= ip && RD32(r2) == sq) {
          ref = r2;
          catchup = false;
          continue;                                                  // goto _next_match
        }
        break;
      }
      s = ip + 1u;                                                   // lz4.cc:623
    }
  }

last_literals:
  {  // lz4.cc:627-637
    const uint32_t run = S - anchor;
    if ((int64_t)op + run + 1 + (run + 255u - kRunMask) / 255u > (int64_t)(uint32_t)cap) return 0;
    if (lane == 0) put8<kGuard>(out, out_cap, op, (run >= kRunMask ? kRunMask : run) << 4);
    op += 1;
    if (run >= kRunMask) {
      const uint32_t nb = (run - kRunMask) / 255u;
      put_len<kGuard>(out, out_cap, op, nb, run - kRunMask - 255u * nb);
      op += (int)nb + 1;
    }
    put_bytes<kGuard>(out, out_cap, op, in, anchor, run);
    op += (int)run;
  }
#undef RD32
  return op;
}

constexpr uint32_t kSmallMax = 4096u;     // tagged table + register prefetch
constexpr uint32_t kPrefetch = 5u;        // 16-byte loads per lane: (15 + 4096 + 15) / 16 / 64 < 5

// Staged-input region: value bytes + 16-byte-load slack; the register prefetch
// of small launches writes kPrefetch whole KiB.
__host__ __device__ __forceinline__ uint32_t in_region_bytes(bool small, uint32_t in_cap) {
  const uint32_t a = ((in_cap + 15u) & ~15u) + 48u;
  const uint32_t b = small ? kPrefetch * 64u * 16u + 16u : 0u;
  return a > b ? a : b;
}

// kFrame = false: LZ4_compress_limitedOutput per value; ret[v] = size or 0,
//   dst slot capacity = cap[v].
// kFrame = true : CompressorLZ4::Compress per value; the slot must hold
//   8 + compress_bound(S) bytes; frame_len[v] = frame bytes, ret[v] = 0 or -1.
template <bool kFrame, bool kSmall>
__global__ __launch_bounds__(64) void lz4_compress_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t in_cap,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ dst_cap, uint32_t* __restrict__ frame_len,
    int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  uint16_t* tab16 = reinterpret_cast<uint16_t*>(smem);
  uint8_t* s_in = smem + kTableBytes;
  const uint32_t in_bytes = in_region_bytes(kSmall, in_cap);
  uint8_t* s_out = s_in + in_bytes;       // [8-byte frame header][block]
  const uint4 z4 = make_uint4(0, 0, 0, 0);

  Table<kSmall> tab{tab16, 1u};
  if (kSmall) {
    for (uint32_t i = lane; i < kTableBytes / 16u; i += 64u) reinterpret_cast<uint4*>(tab16)[i] = z4;
  }
  // register prefetch (kSmall): the next value's 16-byte chunks, lane-strided
  uint4 pf[kPrefetch];
  WorkQueue wq{work, n, batch, 0u, 0u};
  uint32_t v = wq.next();
  auto prefetch = [&](uint32_t w) {
    if (w < n) {
      const uint8_t* gp = src + src_off[w];
      const uint32_t hd = (uint32_t)(reinterpret_cast<uintptr_t>(gp) & 15u);
      const uint4* base = reinterpret_cast<const uint4*>(gp - hd);
      const uint32_t chunks = (hd + min(src_len[w], kSmallMax) + 15u) >> 4;
#pragma unroll
      for (uint32_t i = 0; i < kPrefetch; ++i) {
        const uint32_t c = lane + 64u * i;
        pf[i] = c < chunks ? base[c] : z4;
      }
    }
  };
  if (kSmall) prefetch(v);

  while (v < n) {
    const uint32_t vn = wq.next();         // the next value, one ahead
    const uint32_t S = uni(src_len[v]);
    const uint8_t* g = src + src_off[v];
    uint8_t* o = dst + dst_off[v];
    if (S > in_cap || S >= k64KLimit) {             // byU32 sizes: not this kernel
      if (lane == 0) { ret[v] = kUnsupported; if (kFrame) frame_len[v] = 0; }
      if (kSmall) prefetch(vn);
      v = vn;
      continue;
    }
    uint32_t head;
    if (kSmall) {
      head = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
#pragma unroll
      for (uint32_t i = 0; i < kPrefetch; ++i) reinterpret_cast<uint4*>(s_in)[lane + 64u * i] = pf[i];
      prefetch(vn);                  // the next value's loads fly while this one is parsed
    } else {
      head = stage_to_lds(g, S, s_in);
#ifndef KDB_ABL_NO_ZERO
      for (uint32_t i = lane; i < kTableBytes / 16u; i += 64u) reinterpret_cast<uint4*>(tab16)[i] = z4;
#endif
    }
    __syncthreads();

    const uint8_t* in = s_in + head;
    const uint32_t bound = compress_bound(S);
    if (!kFrame) {
      const uint32_t cap = uni(dst_cap[v]);
      // the block never needs more than `bound` bytes; a larger cap changes nothing
      const int r = cap < bound
                        ? compress_block<kSmall, true>(in, s_in, head, S, tab, s_out + 8, (int)cap, (int)cap)
                        : compress_block<kSmall, false>(in, s_in, head, S, tab, s_out + 8, (int)bound, (int)cap);
      if (r > 0) flush_lds_to_global(o, s_out, 8, (uint32_t)r);
      if (lane == 0) ret[v] = r;
    } else {
      const int r = compress_block<kSmall, false>(in, s_in, head, S, tab, s_out + 8, (int)bound, (int)bound);
      if (r <= 0) {                              // compressor.cc:31-34
        if (lane == 0) { ret[v] = -1; frame_len[v] = 0; }
      } else {
        const bool raw = (uint32_t)r > S;        // raw fallback (compressor.cc:40-48)
        const uint32_t stored = raw ? 0u : (uint32_t)r + 8u;
        const uint32_t flen = raw ? S + 8u : stored;
        if (lane < 8u) {                         // compressor.cc:53-54
          const uint32_t w = lane < 4u ? stored : S;
          s_out[lane] = (uint8_t)(w >> (8u * (lane & 3u)));
        }
        if (raw) {
          flush_lds_to_global(o, s_out, 0, 8u);
          flush_lds_to_global(o + 8, s_in, head, S);
        } else {
          flush_lds_to_global(o, s_out, 0, flen);
        }
        if (lane == 0) { ret[v] = 0; frame_len[v] = flen; }
      }
    }
    if (kSmall) {
      if (++tab.gen == 16u) {                    // tags exhausted: clear (lz4.cc:669)
        tab.gen = 1u;
#ifndef KDB_ABL_NO_ZERO
        for (uint32_t i = lane; i < kTableBytes / 16u; i += 64u) reinterpret_cast<uint4*>(tab16)[i] = z4;
#endif
      }
    }
    __syncthreads();
    v = vn;
  }
}

// LDS bytes a launch needs for values up to max_len bytes.
size_t compress_lds_bytes(uint32_t max_len) {
  const bool small = max_len <= kSmallMax;
  const uint32_t m = small ? kSmallMax : max_len;
  const size_t in_bytes = in_region_bytes(small, m);
  const size_t out_bytes = ((8u + (size_t)compress_bound(m) + 15u) & ~(size_t)15u) + 16u;
  return kTableBytes + in_bytes + out_bytes;
}

template <bool F, bool Sm>
static hipError_t launch_one(hipStream_t st, size_t lds, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* src_len, uint32_t n, uint32_t in_cap, uint8_t* dst,
                             const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                             int32_t* ret) {
  auto kern = lz4_compress_kernel<F, Sm>;
  uint32_t* work = nullptr;
  hipError_t e = work_counter(st, &work);
  if (e != hipSuccess) return e;
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), lds, n);
  const uint32_t batch = claim_batch(n, grid);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, st, src, src_off, src_len, n, in_cap, dst, dst_off,
                     dst_cap, frame_len, ret, work, batch);
  return hipGetLastError();
}

hipError_t launch_compress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                           const uint32_t* src_len, uint32_t n, uint32_t max_len, uint8_t* dst,
                           const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                           int32_t* ret) {
  if (n == 0) return hipSuccess;
  const bool small = max_len <= kSmallMax;
  const uint32_t in_cap = small ? kSmallMax : max_len;
  size_t lds = compress_lds_bytes(max_len);
#ifdef KDB_ABL_OCC
  lds = 163840 / KDB_ABL_OCC;   // diagnostic: force KDB_ABL_OCC workgroups per CU
#endif
  if (frame) {
    return small ? launch_one<true, true>(st, lds, src, src_off, src_len, n, in_cap, dst, dst_off, dst_cap,
                                          frame_len, ret)
                 : launch_one<true, false>(st, lds, src, src_off, src_len, n, in_cap, dst, dst_off, dst_cap,
                                           frame_len, ret);
  }
  return small ? launch_one<false, true>(st, lds, src, src_off, src_len, n, in_cap, dst, dst_off, dst_cap,
                                         frame_len, ret)
               : launch_one<false, false>(st, lds, src, src_off, src_len, n, in_cap, dst, dst_off, dst_cap,
                                          frame_len, ret);
}

}  // namespace kdb_lz4
