// kingdb_amd/csrc/lz4_compress.hip -- gfx950 LZ4 r1.3.0 block compressor.
//
// Replaces LZ4_compress_limitedOutput (/root/reference/algorithm/lz4.cc:664-682)
// = LZ4_compress_generic(limitedOutput, byU16, noDict, noDictIssue)
// (lz4.cc:431-641), fused with CompressorLZ4::Compress's frame epilogue
// (algorithm/compressor.cc:26-59).  Output is byte-identical to the reference.
//
// One wavefront per value.  LDS per workgroup: the byU16 hash table (8192 x u16,
// zeroed per value -- lz4.cc:669's zeroed context) + the value staged from HBM.
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
//  * LZ4_count (lz4.cc:412-428) and the catch-up loop (lz4.cc:531): 64-byte
//    compares, ballot, first-mismatch;
//  * literal copies and length-byte runs.
#include "lz4_device.h"

namespace kdb_lz4 {

#ifdef KDB_LZ4_STAMPS
// Diagnostic build only (never the shipped .so): per-phase shader-clock sums.
__device__ unsigned long long g_stamps[16];
struct Stamps {
  unsigned long long last, acc[12];
  __device__ void start() { last = __builtin_amdgcn_s_memtime(); for (int i = 0; i < 12; ++i) acc[i] = 0; }
  __device__ void mark(int i) { unsigned long long t = __builtin_amdgcn_s_memtime(); acc[i] += t - last; last = t; }
  __device__ void count(int i) { acc[i] += 1; }
  __device__ void flush() { if (__lane_id() == 0) for (int i = 0; i < 12; ++i) atomicAdd(&g_stamps[i], acc[i]); }
};
#define ST_MARK(i) st.mark(i)
#define ST_COUNT(i) st.count(i)
#else
struct Stamps { __device__ void start() {} __device__ void flush() {} };
#define ST_MARK(i) ((void)0)
#define ST_COUNT(i) ((void)0)
#endif

// Position visited at iteration k of a search run started at s (lz4.cc:497-507):
// p(0)=s, p(k+1)=p(k)+step(k), step(0)=1, step(k)=(63+k)>>6 for k>=1, i.e.
// p(k) = s + 1 + sum_{t=64}^{62+k} floor(t/64) for k >= 1.
__device__ __forceinline__ uint32_t search_pos(uint32_t s, uint32_t k) {
  if (k == 0) return s;
  const uint32_t nn = 62u + k, q = nn >> 6, r = nn & 63u;
  return s + 1u + 32u * q * (q - 1u) + q * (r + 1u);
}

__device__ __forceinline__ uint32_t hash16(uint32_t seq) { return (seq * 2654435761u) >> 19; }

// Output sink: global bytes at o[0..cap); never writes at or past cap (the
// reference may, on limitedOutput failures -- the return value is what parity
// is about, see oracle/lz4_oracle.c).
struct Sink {
  uint8_t* o;
  int cap;
  __device__ __forceinline__ void put(int pos, uint32_t b) const {
    if (pos >= 0 && pos < cap) o[pos] = (uint8_t)b;
  }
};

// Emits `run` as a length continuation (nb 255s + remainder) at o[pos..];
// returns the number of bytes written.  Wave-cooperative.
__device__ __forceinline__ int emit_len(const Sink& sk, int pos, uint32_t run) {
  const uint32_t nb = run / 255u, rem = run - nb * 255u;
  for (uint32_t i = lane_id(); i <= nb; i += 64u) sk.put(pos + (int)i, i < nb ? 255u : rem);
  return (int)nb + 1;
}

// Copies n input bytes (value position a..a+n) to o[pos..pos+n).
__device__ __forceinline__ void emit_bytes(const Sink& sk, int pos, const uint8_t* in,
                                           uint32_t a, uint32_t n) {
  for (uint32_t i = lane_id(); i < n; i += 64u) sk.put(pos + (int)i, in[a + i]);
}

// LZ4_compress_generic (byU16, limitedOutput).  `in` = LDS, value byte i at
// in[i] (caller passes the head-adjusted base), readable 8 bytes past S.
// Returns the block size or 0 (limitedOutput failure), like the reference.
__device__ int compress_block(const uint8_t* __restrict__ in, const uint8_t* in_base,
                              uint32_t head, uint32_t S, uint16_t* __restrict__ tab,
                              const Sink& sk, Stamps& st) {
  const uint32_t lane = lane_id();
  const int cap = sk.cap;
  int op = 0;
  uint32_t anchor = 0;
#define RD32(p) lds_rd32(in_base, head + (p))

  if (S >= kMinLength) {                                    // lz4.cc:483
    const uint32_t mflimit = S - kMfLimit;
    const uint32_t matchlimit = S - kLastLiterals;
    // lz4.cc:486: put(0) -- a no-op on the zeroed table.
    uint32_t s = 1;                                         // lz4.cc:487
    for (;;) {
      // ================= search (lz4.cc:494-527), 64 iterations per step
      uint32_t ip = 0, ref = 0;
      bool found = false;
      ST_MARK(7);
      for (uint32_t kb = 0;; kb += 64u) {
        ST_COUNT(8);
        const uint32_t k = kb + lane;
        const uint32_t pk = search_pos(s, k);
        const bool valid = search_pos(s, k + 1u) <= mflimit;      // lz4.cc:510
        const uint32_t seq = valid ? RD32(pk) : 0u;
        const uint32_t h = hash16(seq);
        const uint32_t told = valid ? (uint32_t)tab[h] : 0u;
        const uint64_t vm = __ballot(valid);
        // lanes of this chunk whose iteration hashes to the same slot
        uint64_t same = vm;
#pragma unroll
        for (int b = 0; b < 13; ++b) {
          const uint32_t bit = (h >> b) & 1u;
          const uint64_t m = __ballot(bit);
          same &= bit ? m : ~m;
        }
        const uint64_t below = same & mask_lt(lane);
        const uint32_t refk = below ? search_pos(s, kb + 63u - (uint32_t)__builtin_clzll(below)) : told;
        const bool match = valid && RD32(refk) == seq;           // lz4.cc:527
        const uint64_t mm = __ballot(match);
        if (mm) {
          const uint32_t ks = (uint32_t)__builtin_ctzll(mm);
          const uint64_t later = same & ~mask_le(lane) & mask_le(ks);
          if (valid && lane <= ks && later == 0) tab[h] = (uint16_t)pk;   // lz4.cc:526
          ip = readlane(pk, ks);
          ref = readlane(refk, ks);
          found = true;
          break;
        }
        if (vm != ~0ull) break;              // ran past mflimit: last literals
        if ((same & ~mask_le(lane)) == 0) tab[h] = (uint16_t)pk;
      }
      ST_MARK(1);
      if (!found) break;
      ST_COUNT(9);

      // ================= catch up (lz4.cc:531)
      for (;;) {
        const uint32_t lim = min(ip - anchor, ref);
        if (lim == 0) break;
        const bool eq = lane < lim && in[ip - 1u - lane] == in[ref - 1u - lane];
        const uint32_t c = first_zero(__ballot(eq));
        ip -= c;
        ref -= c;
        if (c < 64u) break;
      }

      ST_MARK(2);
      // ================= literal length + literals (lz4.cc:535-550)
      int tok_pos = op++;
      uint32_t token;
      {
        const uint32_t lit = ip - anchor;
        if ((int64_t)op + lit + (2 + 1 + kLastLiterals) + lit / 255u > (int64_t)cap) return 0;
        if (lit >= kRunMask) {
          token = kRunMask << 4;
          op += emit_len(sk, op, lit - kRunMask);
        } else {
          token = lit << 4;
        }
        emit_bytes(sk, op, in, anchor, lit);
        op += (int)lit;
      }

      ST_MARK(3);
      for (;;) {  // _next_match (lz4.cc:552)
        // offset (lz4.cc:554)
        const uint32_t off = ip - ref;
        if (lane < 2u) sk.put(op + (int)lane, lane ? (off >> 8) : (off & 255u));
        op += 2;
        // match length (lz4.cc:557-592)
        uint32_t ml = 0;
        {
          const uint32_t a = ip + kMinMatch, b = ref + kMinMatch;
          for (;;) {
            const uint32_t rem = matchlimit - (a + ml);
            const bool eq = lane < rem && in[a + ml + lane] == in[b + ml + lane];
            const uint32_t c = first_zero(__ballot(eq));
            ml += c;
            if (c < 64u) break;
          }
        }
        ip += kMinMatch + ml;
        if (ml >= kMlMask) {
          if ((int64_t)op + (1 + kLastLiterals) + (ml >> 8) > (int64_t)cap) return 0;
          token += kMlMask;
          op += emit_len(sk, op, ml - kMlMask);
        } else {
          token += ml;
        }
        if (lane == 0) sk.put(tok_pos, token);
        ST_MARK(4);
        anchor = ip;
        if (ip > mflimit) goto last_literals;                      // lz4.cc:597

        // fill table + test next position (lz4.cc:600-624)
        const uint32_t hm2 = hash16(RD32(ip - 2u));
        if (lane == 0) tab[hm2] = (uint16_t)(ip - 2u);
        const uint32_t sq = RD32(ip);
        const uint32_t hh = hash16(sq);
        const uint32_t r2 = uni(tab[hh]);
        if (lane == 0) tab[hh] = (uint16_t)ip;
        if (r2 + kMaxDistance >= ip && RD32(r2) == sq) {
          ref = r2;
          tok_pos = op++;
          token = 0;
          ST_MARK(5);
          continue;                                                  // goto _next_match
        }
        ST_MARK(5);
        break;
      }
      s = ip + 1u;                                                   // lz4.cc:623
    }
  }

last_literals:
  ST_MARK(7);
  {  // lz4.cc:627-637
    const uint32_t run = S - anchor;
    if ((int64_t)op + run + 1 + (run + 255u - kRunMask) / 255u > (int64_t)(uint32_t)cap) return 0;
    if (run >= kRunMask) {
      if (lane == 0) sk.put(op, kRunMask << 4);
      op += 1;
      op += emit_len(sk, op, run - kRunMask);
    } else {
      if (lane == 0) sk.put(op, run << 4);
      op += 1;
    }
    emit_bytes(sk, op, in, anchor, run);
    op += (int)run;
  }
#undef RD32
  ST_MARK(6);
  return op;
}

// kFrame = false: LZ4_compress_limitedOutput per value; ret[v] = size or 0,
//   dst slot capacity = cap[v].
// kFrame = true : CompressorLZ4::Compress per value; the slot must hold
//   8 + compress_bound(S) bytes; frame_len[v] = frame bytes, ret[v] = 0 or -1.
template <bool kFrame>
__global__ __launch_bounds__(64) void lz4_compress_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ src_len, uint32_t n, uint32_t in_cap,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ dst_cap, uint32_t* __restrict__ frame_len,
    int32_t* __restrict__ ret) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t v = blockIdx.x;
  if (v >= n) return;
  const uint32_t lane = lane_id();
  uint16_t* tab = reinterpret_cast<uint16_t*>(smem);
  uint8_t* s_in = smem + kTableBytes;

  const uint32_t S = uni(src_len[v]);
  const uint8_t* g = src + src_off[v];
  uint8_t* o = dst + dst_off[v];
  if (S > in_cap || S >= k64KLimit) {             // byU32 sizes: not this kernel
    if (lane == 0) { ret[v] = kUnsupported; if (kFrame) frame_len[v] = 0; }
    return;
  }
  Stamps st;
  st.start();
  const uint32_t head = stage_to_lds(g, S, s_in);
  {  // zero the table (lz4.cc:669)
    uint4* t4 = reinterpret_cast<uint4*>(tab);
    const uint4 z = make_uint4(0, 0, 0, 0);
    for (uint32_t i = lane; i < kTableBytes / 16u; i += 64u) t4[i] = z;
  }
  __syncthreads();
  ST_MARK(0);

  const uint8_t* in = s_in + head;
  if (!kFrame) {
    Sink sk{o, (int)dst_cap[v]};
    const int r = compress_block(in, s_in, head, S, tab, sk, st);
    if (lane == 0) ret[v] = r;
    st.flush();
  } else {
    const uint32_t bound = compress_bound(S);
    Sink sk{o + 8, (int)bound};
    const int r = compress_block(in, s_in, head, S, tab, sk, st);
    // compressor.cc:31-59
    uint32_t stored, flen;
    if (r <= 0) {
      if (lane == 0) { ret[v] = -1; frame_len[v] = 0; }
      return;
    }
    if ((uint32_t)r > S) {                    // raw fallback (compressor.cc:40-48)
      emit_bytes(Sink{o + 8, (int)S}, 0, in, 0, S);
      stored = 0;
      flen = S + 8u;
    } else {
      stored = (uint32_t)r + 8u;
      flen = stored;
    }
    if (lane < 8u) {
      const uint32_t w = lane < 4u ? stored : S;
      o[lane] = (uint8_t)(w >> (8u * (lane & 3u)));
    }
    if (lane == 0) { ret[v] = 0; frame_len[v] = flen; }
    ST_MARK(10);
    st.flush();
  }
}

template __global__ void lz4_compress_kernel<false>(const uint8_t*, const uint64_t*, const uint32_t*,
                                                    uint32_t, uint32_t, uint8_t*, const uint64_t*,
                                                    const uint32_t*, uint32_t*, int32_t*);
template __global__ void lz4_compress_kernel<true>(const uint8_t*, const uint64_t*, const uint32_t*,
                                                   uint32_t, uint32_t, uint8_t*, const uint64_t*,
                                                   const uint32_t*, uint32_t*, int32_t*);

// LDS bytes a launch needs for values up to max_len bytes.
size_t compress_lds_bytes(uint32_t max_len) {
  return kTableBytes + (((size_t)max_len + 15u) & ~(size_t)15u) + 48u;
}

#ifdef KDB_LZ4_STAMPS
extern "C" int kdb_lz4_stamps_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -2;
}
extern "C" int kdb_lz4_stamps_reset() {
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif

hipError_t launch_compress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                           const uint32_t* src_len, uint32_t n, uint32_t max_len, uint8_t* dst,
                           const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                           int32_t* ret) {
  if (n == 0) return hipSuccess;
  const size_t lds = compress_lds_bytes(max_len);
  if (frame) {
    hipLaunchKernelGGL(lz4_compress_kernel<true>, dim3(n), dim3(64), lds, st, src, src_off, src_len,
                       n, max_len, dst, dst_off, dst_cap, frame_len, ret);
  } else {
    hipLaunchKernelGGL(lz4_compress_kernel<false>, dim3(n), dim3(64), lds, st, src, src_off,
                       src_len, n, max_len, dst, dst_off, dst_cap, frame_len, ret);
  }
  return hipGetLastError();
}

}  // namespace kdb_lz4
