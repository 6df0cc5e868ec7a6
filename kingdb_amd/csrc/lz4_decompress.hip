// kingdb_amd/csrc/lz4_decompress.hip -- gfx950 LZ4 r1.3.0 block decoder.
//
// Replaces LZ4_decompress_safe_partial (/root/reference/algorithm/lz4.cc:1050-1053)
// = LZ4_decompress_generic(endOnInputSize, partial, target, noDict)
// (lz4.cc:876-1042), and -- in frame mode -- CompressorLZ4::Uncompress's frame
// handling (algorithm/compressor.cc:75-137).  Successful decodes are bit-exact;
// malformed blocks return the reference's exact code -(consumed)-1.
//
// Persistent launch; one wavefront per value at a time, values taken from a
// device-scope work counter.  The compressed block
// is staged HBM -> LDS with aligned 16-byte loads; the value is rebuilt in an
// LDS window (a match source is always earlier output) and written back with
// 16-byte stores.
//
// The decoder is instruction-issue bound, so its token stream is read from a
// 256-byte register window (one dword per lane, refilled by one ds_read_b32):
// four consecutive block bytes are two v_readlane + one 64-bit shift, with no
// LDS round trip per token/offset/length byte.  Literal runs and match copies
// are lane-parallel; an overlapping match (offset < length) is a periodic
// extension of the `offset` bytes before it, so lane i reads
// out[ref + (i mod offset)] -- every source byte is already final and one pass
// suffices (the same bytes as the reference's dec32/dec64 copy, lz4.cc:1008-1018).
#include <cstdio>
#include <cstdlib>
#include <string>

#include "lz4_device.h"
#include "service.h"

namespace kdb_lz4 {

// A uniform value moved to (and kept in) a VGPR: the compiler treats inline
// asm VGPR results as divergent, so arithmetic on it stays on the vector unit
// instead of the CU's single scalar unit.
__device__ __forceinline__ int vgpr(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint32_t vgpr(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Unaligned u32 at an absolute LDS byte address (two aligned dwords +
// v_alignbyte): the base is folded into the address, so no add of the LDS
// buffer's (link-time) base per read.
__device__ __forceinline__ uint32_t lds_rd32_at(uint32_t a) {
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
  const lds_cu32* w = (lds_cu32*)(uintptr_t)(a & ~3u);
  // v_alignbyte reads bits 1:0 of its shift operand only: no `& 3` (with the
  // multiplies in header()/eval(), decompress 2.89 -> 2.79 ms at 1 Mi x 4 KiB,
  // profiles/r04_d/r04_i_ab_decoder_best.txt)
  return __builtin_amdgcn_alignbyte(w[1], w[0], a);
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  uint32_t o = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
  asm volatile("" : "+s"(o));
  return o;
}

// 256-byte window over the staged block (LDS byte coordinates).
struct Window {
  const uint32_t* w32;   // LDS buffer as dwords
  uint32_t base;         // LDS byte offset of lane 0's dword (multiple of 4)
  uint32_t win;          // this lane's dword
  __device__ __forceinline__ void load(uint32_t p) {   // window covering p..p+251
    base = uni(p & ~3u);
    win = w32[(base >> 2) + lane_id()];
  }
  // four bytes at LDS byte offset p (little endian)
  __device__ __forceinline__ uint32_t get4(uint32_t p) {
    if (p + 8u > base + 256u) load(p);
    const uint32_t i = (p - base) >> 2;
    const uint64_t q = ((uint64_t)readlane(win, i + 1u) << 32) | readlane(win, i);
    return uni((uint32_t)(q >> (8u * (p & 3u))));
  }
};

// Decodes the block at LDS bytes [in_off, in_off + csize) of `lds_in` into
// out[0..osize) (LDS).  The 16 bytes after the block are zero (bytes read at or
// past csize read as 0, see oracle/lz4_oracle.c).
__device__ int decode_block(const uint8_t* __restrict__ lds_in, uint32_t in_off, int csize,
                            uint8_t* __restrict__ out, int osize, int target) {
  const uint32_t lane = lane_id();
  in_off = uni(in_off);
  const int iend = unii(csize), oend = unii(osize);
  const int oexit = unii(min(target, oend - (int)kMfLimit));    // lz4.cc:908-910
  // fast-path bounds, per sequence and exact (lz4.cc:930-933, 1024): it is not
  // the last if its literals end at ip <= iend8 and op <= oexit; its match
  // must end at or before oend5
  const int iend8 = iend - (int)(2 + 1 + kLastLiterals);
  const int oend5 = oend - (int)kLastLiterals;
  const uint8_t* in = lds_in + in_off;
  Window wd{reinterpret_cast<const uint32_t*>(lds_in), 0u, 0u};
  wd.load(in_off);
  if (osize == 0) return (csize == 1 && (wd.get4(in_off) & 0xffu) == 0) ? 0 : -1;   // lz4.cc:911
  const float lanef = (float)lane;
  int ip = 0, op = 0;
  // q: the block bytes at ip (only the token and the byte after it are used);
  // have_q: q was taken from the previous sequence's literal load
  uint32_t q = 0;
  int have_q = 0;
#pragma unroll 1
  for (;;) {
    ip = unii(ip);
    op = unii(op);
    if (have_q == 0) q = wd.get4(in_off + (uint32_t)ip);
    have_q = 0;
    {
      // Fast path: sequences that are not the last, with at most one length
      // byte per run, <= 60 literals and no error.  One 64-lane load of the
      // literals also yields the offset, the match-length byte and the next
      // token (v_readlane), instead of scalar window reads.  Anything else --
      // and every error, so its exact code -- leaves the loop and goes
      // through the general path below from the same token.
      //
      // The decoder is bound by the CU's one scalar unit (about one scalar
      // instruction per CU cycle with ~19 waves per CU), while the vector
      // units idle, so this loop keeps its uniform state -- ip, op, the
      // token word and the length arithmetic -- in VGPRs (vgpr(): every lane
      // holds the same value) and only the loop and copy decisions go
      // through the scalar unit (readfirstlane + one compare).  The bounds
      // are the reference's own not-last and match-end conditions for this
      // sequence (so only the true last sequence leaves the fast path; a
      // worst-case "far from both ends" test had sent the last ~330 output
      // bytes of every value through the general path), folded with the
      // rest into sign bits of plain integer expressions, one decision.
      //
      // The next sequence's literal load goes out as soon as its token is
      // known (v_readlane of this one's load), before this sequence's match
      // copy, so the two LDS round trips of a sequence overlap.
      // The match half of a sequence (token low nibble, offset, match-length
      // byte, next token's lane) is computed from SGPRs -- the v_readlane
      // results are scalar already -- and only the literal half and the
      // positions stay on the VALU: 3.60 -> 3.56 ms at 1 Mi x 4 KiB (the whole
      // sequence on the scalar unit measured 4.44, the header too 3.87).
      // Positions are kept as per-lane absolute LDS addresses (lane i: the
      // byte at position + i), so the literal store, the match read and the
      // match store need no address add; the bounds are per-lane constants
      // shifted the same way, and lane 0 (readfirstlane) sees the plain
      // differences.  The token's fields come out of its SGPR with v_bfe.
      typedef __attribute__((address_space(3))) uint8_t lds_b;
      const uint32_t in_abs = lds_addr(lds_in) + in_off;
      const int ob = (int)lds_addr(out);
      const int obl = vgpr(ob + (int)lane), ibl = vgpr((int)in_abs + (int)lane);
      const int oexit_l = oexit + obl, oend5_l = oend5 + obl, iend8_l = iend8 + ibl;
      int avip = ibl + ip, aop = obl + op;
      uint32_t sq = q;                     // the token word in an SGPR
      // a sequence's literal-run header from its token word tq (SGPR) at
      // als-address atip: lx (a literal-length byte follows), xl (its value
      // or 0), lit, als (the first literal's per-lane address)
      int lx, xl, lit, als;
      auto header = [&](uint32_t tq, int atip) {
        int ln, b1;
        asm("v_bfe_u32 %0, %1, 4, 4" : "=v"(ln) : "s"(tq));
        asm("v_bfe_u32 %0, %1, 8, 8" : "=v"(b1) : "s"(tq));
        lx = (ln + 1) >> 4;
        xl = (int)__umul24((uint32_t)b1, (uint32_t)lx);   // lx is 0 or 1: one v_mul_u32_u24 (full
                                                                           // rate), not v_mul_lo_u32, not a negate + and
        lit = ln + xl;                                            // <= 60 iff !lx || b1 <= 45
        als = atip + 1 + lx;
      };
      header(sq, avip);
      // lane i holds the block's 4 bytes from ls + i: byte 0 is literal i,
      // and one readlane gives the offset + match-length byte, another the
      // next token and the byte after it.  The load goes out before the
      // fast-path test (its address is inside the staged block plus the
      // window slack for any token; a sequence that fails the test never
      // uses it), so both tests are one scalar decision.
      uint32_t v = lds_rd32_at((uint32_t)als);
      // The sequence's match half and the fast-path test; evaluated before
      // the loop and at the end of each pass, so the loop is a do-while on
      // one scalar compare (a mid-loop break had the structurizer carry an
      // exit flag around the loop: 4 scalar instructions per sequence).
      int mn, slit, aopl, off, mx, xm, mlen, aref, tst;
      auto eval = [&]() {
        mn = (int)(sq & 0xffu) & (int)kMlMask;
        slit = unii(lit);
        aopl = aop + lit;
        const uint32_t w = readlane(v, (uint32_t)slit & 63u);   // offset, match-length byte
        const int e = (int)((w >> 16) & 0xffu);
        off = (int)(w & 0xffffu);
        mx = (mn + 1) >> 4;                                      // a match-length byte follows
        xm = e * mx;                                             // mx is 0 or 1: one s_mul
        mlen = mn + xm + (int)kMinMatch;
        aref = aopl - off;
        // far from both ends, <= 60 literals, ref >= 0, one match-length byte
        tst = unii((iend8_l - als - lit) | (oexit_l - aopl) | (45 - xl) | (aref - obl) | ((oend5_l - mlen) - aopl)) |
              (254 - xm);
      };
      eval();
      if (tst >= 0) {
#pragma unroll 1
      do {
#if !KDB_ABL_DEC_NOLIT   // (attribution build: the fast path's literal stores left out -- timing only)
        ((lds_b*)(uintptr_t)(uint32_t)aop)[0] = (uint8_t)v;       // lz4.cc:947 (lanes past lit: not-yet-produced output)
#endif
        const int nt = slit + 2 + mx;                             // next token's lane (<= 63)
        sq = readlane(v, (uint32_t)nt);
        avip = als + nt;
        header(sq, avip);
        v = lds_rd32_at((uint32_t)als);                           // the next sequence's literals
        asm volatile("" ::: "memory");
        // the match's first 64-byte step as a plain copy, unconditionally
        // (mlen >= 4; lanes past mlen write the not-yet-produced tail); only
        // an overlapping match (offset < its first step: periodic, or offset
        // 0) or one longer than a step takes the branch, which for an
        // overlapping match rewrites the whole match (a plain copy may have
        // read bytes of this step before they were written)
#if !KDB_ABL_DEC_NOMATCH   // (attribution build: the first match step left out -- timing only)
        const uint8_t b0 = ((const lds_b*)(uintptr_t)(uint32_t)aref)[0];
        ((lds_b*)(uintptr_t)(uint32_t)aopl)[0] = b0;
#endif
        asm volatile("" ::: "memory");
        if (((off - min(mlen, 64)) | (64 - mlen)) < 0) {
          const int steps = unii(mlen);
          const int opl = unii(aopl) - ob, ref = opl - off;
          if (off - min(mlen, 64) < 0) {
            if (off > 0) {                        // periodic (see the general path)
              const int r0 = (int)lane - off * (int)((lanef + 0.5f) * __builtin_amdgcn_rcpf((float)off));
              const int rr = r0 < 0 ? r0 + off : (r0 >= off ? r0 - off : r0);
#pragma unroll 1
              for (int i = 0; i < steps; i += 64) {
                const uint8_t b = out[ref + i + rr];
                out[opl + i + (int)lane] = b;
              }
            } else {                              // offset 0: zeros (see the general path)
#pragma unroll 1
              for (int i = 0; i < steps; i += 64) out[opl + i + (int)lane] = 0;
            }
          } else {
#pragma unroll 1
            for (int i = 64; i < steps; i += 64) {
              const uint8_t b = out[ref + i + (int)lane];
              out[opl + i + (int)lane] = b;
              asm volatile("" ::: "memory");
            }
          }
        }
        asm volatile("" ::: "memory");
        aop = aopl + mlen;
        eval();
      } while (tst >= 0);
      }
      ip = unii(avip) - (int)in_abs;
      op = unii(aop) - ob;
      q = sq;
    }
    const uint32_t token = q & 0xffu;
    ip++;
    int length = (int)(token >> 4);
    if (length == (int)kRunMask) {                                // lz4.cc:917-925
      uint32_t s = (q >> 8) & 0xffu;
      ip++;
      length += (int)s;
#pragma unroll 1
      while (ip < iend - (int)kRunMask && s == 255u) {
        s = wd.get4(in_off + (uint32_t)ip) & 0xffu;
        ip++;
        length += (int)s;
      }
    }
    const int cpy = op + length;                                  // lz4.cc:930-952
    const bool last = cpy > oexit || ip + length > iend - (int)(2 + 1 + kLastLiterals);
    if (last && (cpy > oend || ip + length > iend)) return -ip - 1;
    // Whole 64-byte steps, no lane mask: the bytes written past the run land
    // in output the decoder has not produced yet (overwritten before anything
    // reads them; the window has 64 bytes of slack) -- no exec-mask juggling
    // on the scalar unit, which is what this loop is bound by.
#pragma unroll 1
    for (int i = 0; i < length; i += 64) out[op + i + (int)lane] = in[ip + i + (int)lane];
    ip += length;
    op = cpy;
    if (last) break;
    // offset (lz4.cc:955-956) and the first match-length byte
    q = wd.get4(in_off + (uint32_t)ip);
    const int off = (int)(q & 0xffffu);
    ip += 2;
    const int ref = op - off;
    if (ref < 0) return -ip - 1;
    length = (int)(token & kMlMask);                              // lz4.cc:959-968
    if (length == (int)kMlMask) {
      if (ip > iend - (int)kLastLiterals) return -ip - 1;
      uint32_t s = (q >> 16) & 0xffu;
      ip++;
      length += (int)s;
#pragma unroll 1
      while (s == 255u) {
        if (ip > iend - (int)kLastLiterals) return -ip - 1;
        s = wd.get4(in_off + (uint32_t)ip) & 0xffu;
        ip++;
        length += (int)s;
      }
    }
    const int mlen = length + (int)kMinMatch;
    if (op + mlen > oend - (int)kLastLiterals) return -ip - 1;    // lz4.cc:1024
    asm volatile("" ::: "memory");
    if (off >= mlen || off >= 64) {
      // plain forward copy in 64-byte steps: every source byte a lane < mlen
      // reads is < the step (lanes past mlen write the not-yet-produced tail)
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) {
        const uint8_t b = out[ref + i + (int)lane];
        out[op + i + (int)lane] = b;
        asm volatile("" ::: "memory");
      }
    } else if (off > 0) {
      // periodic: out[op+i+l] = out[ref + i + (l mod off)] -- the same byte as
      // out[ref + (i+l) mod off], read from the step before (always written)
      const int r0 = (int)lane - off * (int)((lanef + 0.5f) * __builtin_amdgcn_rcpf((float)off));
      const int rr = r0 < 0 ? r0 + off : (r0 >= off ? r0 - off : r0);
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) {
        const uint8_t b = out[ref + i + rr];
        out[op + i + (int)lane] = b;
      }
    } else {
      // offset 0: the reference copies its destination onto itself, bytes it
      // never wrote (new[] memory: undefined).  Here they are zeros, never the
      // previous value decoded in this LDS window.
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) out[op + i + (int)lane] = 0;
    }
    asm volatile("" ::: "memory");
    op += mlen;
  }
  return op;
}

// kFrame = false: block mode. in_len[v] = C, out_cap[v] = S (target = max unless
//   given); ret[v] = LZ4 return code, out_len[v] = max(ret, 0).
// kFrame = true : one CompressorLZ4 frame per value at src + src_off[v]
//   (header u32 size_compressed_stored, u32 size_source); in_len[v] = bytes
//   available there; ret[v] = 0 (OK) / -1 (IOError); out_len[v] = *size_dest.
// Register prefetch: while a value is decoded, the next value's bytes (frame
// header included) are already on their way from HBM as whole aligned
// 16-byte chunks, so a value's start does not wait for two HBM round trips
// (header, then block).  Values whose bytes do not fit kDPrefetch chunks per
// lane (or the staging area) get chunks = 0 and are staged as before.
// kPF chunks of 16 B per lane: 5 hold any frame of a <= 4 KiB value (8 +
// compressBound(4096) bytes); 3 hold a frame of up to 3 057 bytes, and free 8
// VGPRs (launch_one picks 3 when the batch's max_in allows it).
template <uint32_t kPF>
__device__ __forceinline__ void prefetch_value(uint4& p0, uint4& p1, uint4& p2, uint4& p3, uint4& p4, uint32_t& head,
                                               uint32_t& chunks, uint32_t w, uint32_t n,
                                               const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                                               const uint32_t* __restrict__ in_len, uint32_t s_in_cap) {
  static_assert(kPF == 3 || kPF == 5, "3 or 5 chunks per lane");
  chunks = 0;
  if (w >= n) return;
  const uint8_t* gp = src + sload(src_off, w);
  const uint32_t len = sload(in_len, w);
  const uint32_t hd = uni((uint32_t)(reinterpret_cast<uintptr_t>(gp) & 15u));
  const uint32_t ch = (hd + len + 15u) >> 4;
  if (len == 0 || hd + len + 16u > s_in_cap || ch > 64u * kPF) return;
  head = hd;
  chunks = ch;
  const uint4* base = reinterpret_cast<const uint4*>(__builtin_assume_aligned(gp - hd, 16));
  const uint32_t lane = lane_id();
  p0 = base[min(lane, ch - 1u)];
  p1 = base[min(lane + 64u, ch - 1u)];
  p2 = base[min(lane + 128u, ch - 1u)];
  if constexpr (kPF == 5) {
    p3 = base[min(lane + 192u, ch - 1u)];
    p4 = base[min(lane + 256u, ch - 1u)];
  }
}

// Between a value's LDS staging and its decode, and between values: the
// wave's own LDS instructions execute in order, so a workgroup of several
// independent waves needs no barrier (a one-wave workgroup keeps the one it had).
__device__ __forceinline__ void value_sync(uint32_t waves) {
  if (waves > 1) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  else __syncthreads();
}

template <bool kFrame, uint32_t kPF>
__device__ __forceinline__ void small_decode_loop(
    uint8_t* const smem, const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t in_cap, uint32_t out_cap_max,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ out_cap, const uint32_t* __restrict__ target,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch,
    uint32_t skip_big, uint32_t nq, uint32_t guide = 0, uint32_t waves = 1) {
  const uint32_t lane = lane_id();
  // [staged block + 16 zero bytes][output window + 64 bytes of slack for the
  // decoder's unmasked 64-byte steps]; the register window may read 256 bytes
  // past the block, into the output window (decompress_lds_bytes).  With
  // `waves` > 1 (lz4_decompress_kernel) `smem` is this wave's region of the
  // workgroup's LDS and the waves never wait for one another.
  uint8_t* s_in = smem;
  const uint32_t s_in_cap = (in_cap + 32u + 15u) & ~15u;
  uint8_t* s_out = smem + s_in_cap;

  // the next value's bytes in flight in registers (prefetch_value)
  uint4 pf0 = {}, pf1 = {}, pf2 = {}, pf3 = {}, pf4 = {};
  uint32_t pf_head = 0, pf_chunks = 0;

  const uint32_t vb = waves > 1 ? blockIdx.x * waves + uni(threadIdx.x >> 6) : blockIdx.x;
  WorkQueue wq = WorkQueue::make(work, n, batch, nq, guide, vb, gridDim.x * waves);
  uint32_t v = uni(wq.next());
  prefetch_value<kPF>(pf0, pf1, pf2, pf3, pf4, pf_head, pf_chunks, v, n, src, src_off, in_len, s_in_cap);
#pragma unroll 1
  while (v < n) {
    const uint32_t vn = uni(wq.next());   // the next value, one ahead
    // the prefetched bytes land in LDS (byte i of the value at s_in[head + i])
    // before the registers take the next value's
    const uint32_t st_head = pf_head, st_chunks = pf_chunks;
    {
      uint4* l4 = reinterpret_cast<uint4*>(s_in);
      if (lane < st_chunks) l4[lane] = pf0;
      if (lane + 64u < st_chunks) l4[lane + 64u] = pf1;
      if (lane + 128u < st_chunks) l4[lane + 128u] = pf2;
      if constexpr (kPF == 5) {
        if (lane + 192u < st_chunks) l4[lane + 192u] = pf3;
        if (lane + 256u < st_chunks) l4[lane + 256u] = pf4;
      }
    }
    prefetch_value<kPF>(pf0, pf1, pf2, pf3, pf4, pf_head, pf_chunks, vn, n, src, src_off, in_len, s_in_cap);
    do {
      const uint8_t* g = src + sload(src_off, v);
      uint8_t* o = dst + sload(dst_off, v);
      int csize, osize, tgt;
      if (kFrame) {
        // compressor.cc:89-90 (GetFixed32 x2)
        uint32_t stored, raw;
        if (st_chunks) {
          stored = uni(lds_rd32(s_in, st_head));
          raw = uni(lds_rd32(s_in, st_head + 4u));
        } else {
          stored = uni((uint32_t)g[0] | ((uint32_t)g[1] << 8) | ((uint32_t)g[2] << 16) | ((uint32_t)g[3] << 24));
          raw = uni((uint32_t)g[4] | ((uint32_t)g[5] << 8) | ((uint32_t)g[6] << 16) | ((uint32_t)g[7] << 24));
        }
        const uint32_t avail = sload(in_len, v);
        if (raw > sload(out_cap, v)) {
          if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
          break;
        }
        if (stored == 0) {  // raw frame (compressor.cc:116-124)
          if (raw + 8u > avail) {
            if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
            break;
          }
          for (uint32_t i = lane; i < raw; i += 64u) o[i] = g[8u + i];
          if (lane == 0) { ret[v] = 0; out_len[v] = raw; }
          break;
        }
        csize = (int)(stored - 8u);          // compressor.cc:96 (u32 wrap kept: int cast)
        osize = (int)raw;
        tgt = osize;                         // compressor.cc:103-107: target = max = size_source
        g += 8;
        if (csize < 0 || (uint32_t)csize + 8u > avail) {
          // a negative size makes the reference return -2/-3 (IOError); a size past
          // the bytes supplied would have it read foreign memory: IOError as well.
          if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
          break;
        }
      } else {
        csize = (int)sload(in_len, v);
        osize = (int)sload(out_cap, v);
        tgt = target ? (int)sload(target, v) : osize;
      }
      if ((uint32_t)csize > in_cap || (uint32_t)osize > out_cap_max || csize < 0 || osize < 0) {
        // values too large for this launch's LDS: the ring decoder's (its own
        // launch, beside this one) when skip_big, else unsupported
        if (skip_big && csize >= 0 && osize >= 0) break;
        if (lane == 0) { ret[v] = kUnsupported; if (out_len) out_len[v] = 0; }
        break;
      }
      const uint32_t head = st_chunks ? st_head + (kFrame ? 8u : 0u) : stage_to_lds(g, (uint32_t)csize, s_in);
      if (lane < 16u) s_in[head + (uint32_t)csize + lane] = 0;   // OOB bytes read as 0
      value_sync(waves);
      const int r = decode_block(s_in, head, csize, s_out, osize, tgt);
      if (r > 0) flush_lds_to_global(o, s_out, 0, (uint32_t)r);
      if (lane == 0) {
        if (kFrame) {
          ret[v] = r > 0 ? 0 : -1;           // compressor.cc:109-115
          out_len[v] = r > 0 ? (uint32_t)r : 0u;
        } else {
          ret[v] = r;
          if (out_len) out_len[v] = r > 0 ? (uint32_t)r : 0u;
        }
      }
    } while (false);
    value_sync(waves);
    v = vn;
  }
}

// Workgroups of blockDim.x / 64 independent waves, each with its own `region`
// bytes of the dynamic LDS (launch_one picks the count: LDS is handed out in
// 1 280-byte steps per workgroup, so one-wave workgroups of the headline's
// 7 264 bytes held 21 waves per CU, two of eleven hold 22).
template <bool kFrame, uint32_t kPF>
__global__ __launch_bounds__(1024) void lz4_decompress_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t in_cap, uint32_t out_cap_max,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ out_cap, const uint32_t* __restrict__ target,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch,
    uint32_t skip_big, uint32_t nq, uint32_t guide, uint32_t region) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t waves = blockDim.x >> 6;
  small_decode_loop<kFrame, kPF>(smem + region * uni(threadIdx.x >> 6), src, src_off, in_len, n, in_cap, out_cap_max,
                                 dst, dst_off, out_cap, target, out_len, ret, work, batch, skip_big, nq, guide, waves);
}

// ---------------------------------------------------------------------------
// Values whose output exceeds what the LDS-resident decoder holds (> 65 546
// bytes: KingDB's 1 MB parts, byU32 blocks) or whose block exceeds its staging
// size.  Same decode rules (lz4.cc:876-1042); the value streams through two
// LDS rings instead of being staged whole:
//   * output: a 4 KiB ring, each decoded byte also written straight to its
//     place in HBM; a match from further back than the ring serves (decode_ring:
//     4 032 bytes) reads its source from there;
//   * input: an 8 KiB ring refilled 4 KiB at a time from HBM (bytes at and
//     past the block end staged as 0, like the zeroed tail of the LDS decoder),
//     plus a 512-byte mirror of its start so the 256-byte register window
//     never wraps.
// The input ring's size is kIR: 8 KiB (refilled 4 KiB at a time) where few
// values run at once (1 MiB parts), 4 KiB in the mixed launch when every
// value fits byU16 (<= 65 546 bytes): 8.7 KiB of LDS per wave instead of
// 12.8, 18 waves per CU instead of 12 (64 KiB values 1.33 -> 1.07 ms;
// 1 MiB parts 4.71 -> 4.80 ms with it, so they keep 8 KiB;
// profiles/r04_d/r04_ir_ab_input_ring.txt).
constexpr uint32_t kIMirror = 512u;
template <uint32_t kORing, uint32_t kIR>
constexpr size_t ring_lds() { return kORing + kIR + kIMirror; }

template <uint32_t kIR>
struct InRing {
  static constexpr uint32_t kIRing = kIR, kIMask = kIR - 1u, kIHalf = kIR / 2u;
  static_assert(kIHalf >= kIMirror && (kIR & kIMask) == 0u, "a power-of-two ring of two halves, each >= the mirror");
  uint8_t* lds;          // kIRing + kIMirror bytes
  const uint8_t* g;      // block start in HBM
  uint32_t csize;
  uint32_t filled;       // input bytes staged so far (multiple of kIHalf)

  // One half of the ring: every lane's loads go out before the first is
  // waited for.  Round 6 had them per dword behind a branch (P < csize, then
  // the second word when misaligned), which the compiler serialised: 16 HBM
  // round trips per 4 KiB half, ~1/4 of a 1 MiB part's decode.  Now the
  // indices are clamped to the block's last aligned dword instead, so every
  // load is unconditional (and, as before, only dwords holding a block byte
  // are read, so none can fault); bytes past the block are masked to zero.
  // (kBatch dwords per lane in flight -- 8 of an 8 KiB ring's 16, 4 of a
  // 4 KiB ring's 8 -- keeps the ring kernels' VGPRs, and so their waves per
  // SIMD, where they were: all 16 took the mixed kernel to 169 VGPRs, all 8
  // the 4 KiB one to 112.)
  __device__ void refill() {
    constexpr uint32_t kPer = kIHalf / 256u, kBatch = kPer >= 16u ? 8u : kPer / 2u;   // dwords per lane
    static_assert(kIHalf % 256u == 0u && kPer % kBatch == 0u, "a half is whole batches of every lane's dwords");
    const uint32_t lane = lane_id();
    const uint32_t rp = filled & kIMask;
    uint32_t* r32 = reinterpret_cast<uint32_t*>(lds);
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 3u);   // uniform: filled % 4 == 0
    const uint32_t* a = reinterpret_cast<const uint32_t*>(g - mis);
    const uint32_t last = (csize - 1u + mis) >> 2;                          // holds the block's last byte
#pragma unroll 1
    for (uint32_t b = 0; b < kPer; b += kBatch) {
      uint32_t w[kBatch];
      if (csize == 0u) {
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) w[k] = 0u;
      } else {
        uint32_t lo[kBatch], hi[kBatch];
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
          const uint32_t i = (filled >> 2) + lane + 64u * (b + k);
          lo[k] = a[min(i, last)];
          hi[k] = a[min(i + 1u, last)];
        }
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
          const uint32_t P = filled + 4u * (lane + 64u * (b + k));
          uint32_t x = __builtin_amdgcn_alignbyte(hi[k], lo[k], mis);
          const uint32_t have = P < csize ? csize - P : 0u;
          if (have < 4u) x &= (1u << (8u * have)) - 1u;
          w[k] = x;
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < kBatch; ++k) {
        const uint32_t d = lane + 64u * (b + k);
        r32[(rp >> 2) + d] = w[k];
        if (rp == 0 && d < kIMirror / 4u) r32[kIRing / 4u + d] = w[k];
      }
    }
    filled += kIHalf;
  }
  // bytes up to absolute input position `upto` staged (the oldest half is
  // overwritten: callers only move forward, and never need bytes more than
  // kIHalf behind the read position)
  __device__ __forceinline__ bool ensure(uint32_t upto) {
    bool any = false;
    while (filled < upto) { refill(); any = true; }
    return any;
  }
};

// 256-byte register window over the input ring (ring coordinates).
template <uint32_t kIMask>
struct RingWindow {
  const uint32_t* w32;
  uint32_t base, win;
  __device__ __forceinline__ void invalidate() { base = 0xFFFFFF00u; }
  __device__ __forceinline__ uint32_t get4(uint32_t pos) {
    const uint32_t p = uni(pos & kIMask);
    if (p < base || p + 8u > base + 256u) {
      base = uni(p & ~3u);
      win = w32[(base >> 2) + lane_id()];
    }
    const uint32_t i = (p - base) >> 2;
    const uint64_t q = ((uint64_t)readlane(win, i + 1u) << 32) | readlane(win, i);
    return uni((uint32_t)(q >> (8u * (p & 3u))));
  }
};

template <uint32_t kORing, uint32_t kIR>
__device__ int decode_ring(InRing<kIR>& in, uint8_t* __restrict__ ring, uint8_t* __restrict__ o, int csize, int osize,
                           int target) {
  constexpr uint32_t kOMask = kORing - 1u;
  constexpr uint32_t kIRing = kIR, kIMask = kIR - 1u;
  const uint32_t lane = lane_id();
  // the output ring's byte at position p: LDS address (p mod kORing) | rbase,
  // one v_and_or -- the ring starts the kernel's dynamic LDS, address 0 (the
  // ring kernels have no static LDS: checked at launch, ring_kernel_ok), so
  // its base is a multiple of kORing
  // (one VALU: the mask in a VGPR, the base in an SGPR -- gfx9's VOP3 reads
  // one SGPR at most, so the compiler left the two as an and + an or)
  typedef __attribute__((address_space(3))) uint8_t lds_r8;
  const uint32_t rbase = lds_addr(ring), vmask = vgpr(kOMask);
  // the fast path's whole-step ring stores (below): 1 MiB parts decode
  // 4.97 -> 4.23 ms; the 4 KiB input ring's launch (a mixed batch's 64 KiB
  // values) measured slower with them (decompress min of 9: 1.86 against
  // 1.68 ms masked, profiles/r06/r06_v_ab_*.txt), so it keeps the masked ones
  constexpr bool kWhole = kIR > 4096u;
  auto ring_at = [&](uint32_t p) -> uint32_t {
    uint32_t a;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(p), "v"(vmask), "s"(rbase));
    return a;
  };
#define RG(p) (((lds_r8*)(uintptr_t)ring_at((uint32_t)(p)))[0])
  const int iend = unii(csize), oend = unii(osize);
  const int oexit = unii(min(target, oend - (int)kMfLimit));    // lz4.cc:908-910
  const int far_ip = iend - (int)(2 + 1 + kLastLiterals) - 62;   // as in decode_block
  const int far_op = min(oexit - 60, oend - (int)kLastLiterals - 60 - 273);
  RingWindow<kIMask> wd{reinterpret_cast<const uint32_t*>(in.lds), 0u, 0u};
  wd.invalidate();
  in.ensure(kIRing);
  if (osize == 0) return (csize == 1 && (wd.get4(0) & 0xffu) == 0) ? 0 : -1;   // lz4.cc:911
  const float lanef = (float)lane;
  int ip = 0, op = 0;
  uint32_t q = 0;
  int have_q = 0;                          // as in decode_block
#pragma unroll 1
  for (;;) {
    ip = unii(ip);
    op = unii(op);
    if (in.ensure((uint32_t)ip + kIMirror)) wd.invalidate();
    if (have_q == 0) q = wd.get4((uint32_t)ip);
    have_q = 0;
    {
      // decode_block's fast path, over the rings, on the vector unit like
      // decode_block's (uniform state in VGPRs): the literal load reads the
      // input ring (its mirror covers the wrap; the loop runs while 512
      // bytes past ip are staged), and the match source must lie in the
      // output ring, at most kORing - 64 bytes back.  A sequence whose next
      // token sits on lane 63 (its second byte not loaded) ends the loop
      // after it, q to be re-read.
      //
      // As in decode_block, the ring stores are whole 64-lane steps with no
      // lane mask (round 6): the bytes past a run land on output not yet
      // produced, or on ring slots of positions more than kORing - 64 back,
      // which no match reads from the ring (the fast path's bound above; the
      // general path reads those from HBM).  The HBM stores stay exact: a
      // buffer store whose offset is out of range (2^31) for the lanes past
      // the run, so no exec mask and no 64-bit address per store.  The
      // match's first step is a plain copy, unconditionally; an overlapping
      // match rewrites it (its HBM bytes are stored by the rewrite only).
      const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(o, 0, 0x7fffffff, 0x00020000);
      auto ost = [&](uint8_t b, bool w, int pos) {
        __builtin_amdgcn_raw_buffer_store_b8(b, orsrc, w ? pos : (int)0x80000000, 0, 0);
      };
      const int lim_ip = min(far_ip, (int)in.filled - (int)kIMirror);
      int vip = vgpr(ip), vop = vgpr(op);
      uint32_t vq = vgpr(q);
      int qok = 1;
      // as in decode_block: the next sequence's literal load goes out before
      // this sequence's match copy
      int lx, xl, lit, ls;
      auto header = [&](uint32_t tq, int tip) {
        const int ln = (int)(tq & 0xffu) >> 4, b1 = (int)((tq >> 8) & 0xffu);
        lx = (ln + 1) >> 4;
        xl = (int)__umul24((uint32_t)b1, (uint32_t)lx);   // lx is 0 or 1 (as in decode_block)
        lit = ln + xl;
        ls = tip + 1 + lx;
      };
      header(vq, vip);
      uint32_t v = in.lds[((uint32_t)ls & kIMask) + lane];
#pragma unroll 1
      for (;;) {
        const int mn = (int)(vq & 0xffu) & (int)kMlMask;
        const int opl = vop + lit;
        const uint32_t l3 = (uint32_t)unii(lit) & 63u;
        const int e = (int)readlane(v, (l3 + 2u) & 63u);
        const int off = (int)(readlane(v, l3) | (readlane(v, (l3 + 1u) & 63u) << 8));
        const int mx = (mn + 1) >> 4;
        const int xm = e * mx;
        const int mlen = mn + xm + (int)kMinMatch;
        if (unii((lim_ip - vip) | (far_op - vop) | (45 - xl) | (opl - off) | (254 - xm) | ((int)kORing - 64 - off)) < 0)
          break;
        uint32_t nt;
        if constexpr (kWhole) {
          RG(vop + (int)lane) = (uint8_t)v;
          ost((uint8_t)v, (int)lane < lit, vop + (int)lane);
          nt = (uint32_t)unii(lit + 2 + mx);
          vq = vgpr(readlane(v, nt) | (readlane(v, min(nt + 1u, 63u)) << 8));
          vip = ls + lit + 2 + mx;
          header(vq, vip);
          v = in.lds[((uint32_t)ls & kIMask) + lane];   // the next sequence's literals (in the ring + mirror)
          const int ref = opl - off;
          asm volatile("" ::: "memory");
          const int steps = unii(mlen);
          const bool overlap = unii(off - min(mlen, 64)) < 0;
          {
            const uint8_t b0 = RG(ref + (int)lane);
            RG(opl + (int)lane) = b0;
            ost(b0, !overlap && (int)lane < mlen, opl + (int)lane);
          }
          asm volatile("" ::: "memory");
          if (unii((off - min(mlen, 64)) | (64 - mlen)) < 0) {
            if (overlap) {
              if (unii(off) > 0) {
                const int r0 = (int)lane - off * (int)((lanef + 0.5f) * __builtin_amdgcn_rcpf((float)off));
                const int rr = r0 < 0 ? r0 + off : (r0 >= off ? r0 - off : r0);
  #pragma unroll 1
                for (int i = 0; i < steps; i += 64) {
                  const int j = i + (int)lane;
                  const uint8_t b = RG(ref + i + rr);
                  RG(opl + j) = b;
                  ost(b, j < mlen, opl + j);
                }
              } else {                              // offset 0: zeros (see decode_block)
  #pragma unroll 1
                for (int i = 0; i < steps; i += 64) {
                  const int j = i + (int)lane;
                  RG(opl + j) = 0;
                  ost(0, j < mlen, opl + j);
                }
              }
            } else {
  #pragma unroll 1
              for (int i = 64; i < steps; i += 64) {
                const int j = i + (int)lane;
                const uint8_t b = RG(ref + j);
                RG(opl + j) = b;
                ost(b, j < mlen, opl + j);
                asm volatile("" ::: "memory");
              }
            }
          }
        } else {
          if ((int)lane < lit) {
            RG(vop + (int)lane) = (uint8_t)v;
            o[vop + (int)lane] = (uint8_t)v;
          }
          nt = (uint32_t)unii(lit + 2 + mx);
          vq = vgpr(readlane(v, nt) | (readlane(v, min(nt + 1u, 63u)) << 8));
          vip = ls + lit + 2 + mx;
          header(vq, vip);
          v = in.lds[((uint32_t)ls & kIMask) + lane];   // the next sequence's literals (in the ring + mirror)
          const int ref = opl - off;
          asm volatile("" ::: "memory");
          const int steps = unii(mlen);
          if (unii(off - min(mlen, 64)) < 0) {
            if (unii(off) > 0) {
              const int r0 = (int)lane - off * (int)((lanef + 0.5f) * __builtin_amdgcn_rcpf((float)off));
              const int rr = r0 < 0 ? r0 + off : (r0 >= off ? r0 - off : r0);
  #pragma unroll 1
              for (int i = 0; i < steps; i += 64) {
                const int j = i + (int)lane;
                const uint8_t b = RG(ref + i + rr);
                if (j < mlen) {
                  RG(opl + j) = b;
                  o[opl + j] = b;
                }
              }
            } else {                                // offset 0: zeros (see decode_block)
  #pragma unroll 1
              for (int i = 0; i < steps; i += 64) {
                const int j = i + (int)lane;
                if (j < mlen) {
                  RG(opl + j) = 0;
                  o[opl + j] = 0;
                }
              }
            }
          } else {
  #pragma unroll 1
            for (int i = 0; i < steps; i += 64) {
              const int j = i + (int)lane;
              const uint8_t b = RG(ref + j);
              if (j < mlen) {
                RG(opl + j) = b;
                o[opl + j] = b;
              }
              asm volatile("" ::: "memory");
            }
          }
        }
        asm volatile("" ::: "memory");
        vop = opl + mlen;
        if (nt >= 63u) {                      // the next token's second byte was not loaded
          qok = 0;
          break;
        }
      }
      ip = unii(vip);
      op = unii(vop);
      q = (uint32_t)unii((int)vq);
      if (!qok) {
        // resume at the top: re-stage if needed, re-read the token
        continue;
      }
      if (in.ensure((uint32_t)ip + kIMirror)) wd.invalidate();
    }
    const uint32_t token = q & 0xffu;
    ip++;
    int length = (int)(token >> 4);
    if (length == (int)kRunMask) {                                // lz4.cc:917-925
      uint32_t s = (q >> 8) & 0xffu;
      ip++;
      length += (int)s;
#pragma unroll 1
      while (ip < iend - (int)kRunMask && s == 255u) {
        if (in.ensure((uint32_t)ip + kIMirror)) wd.invalidate();
        s = wd.get4((uint32_t)ip) & 0xffu;
        ip++;
        length += (int)s;
      }
    }
    const int cpy = op + length;                                  // lz4.cc:930-952
    const bool last = cpy > oexit || ip + length > iend - (int)(2 + 1 + kLastLiterals);
    if (last && (cpy > oend || ip + length > iend)) return -ip - 1;
    // literals: from the input ring, in pieces of what is staged
#pragma unroll 1
    for (int done = 0; done < length;) {
      if ((uint32_t)(ip + done) >= in.filled) { in.refill(); wd.invalidate(); }
      const int piece = min(length - done, (int)(in.filled - (uint32_t)(ip + done)));
#pragma unroll 1
      for (int i = 0; i < piece; i += 64) {
        const int j = i + (int)lane;
        const uint8_t b = in.lds[(uint32_t)(ip + done + j) & kIMask];
        if (j < piece) {
          RG(op + done + j) = b;
          o[op + done + j] = b;
        }
      }
      done += piece;
    }
    ip += length;
    op = cpy;
    if (last) break;
    if (in.ensure((uint32_t)ip + kIMirror)) wd.invalidate();
    q = wd.get4((uint32_t)ip);                                    // offset (lz4.cc:955-956)
    const int off = (int)(q & 0xffffu);
    ip += 2;
    const int ref = op - off;
    if (ref < 0) return -ip - 1;
    length = (int)(token & kMlMask);                              // lz4.cc:959-968
    if (length == (int)kMlMask) {
      if (ip > iend - (int)kLastLiterals) return -ip - 1;
      uint32_t s = (q >> 16) & 0xffu;
      ip++;
      length += (int)s;
#pragma unroll 1
      while (s == 255u) {
        if (ip > iend - (int)kLastLiterals) return -ip - 1;
        if (in.ensure((uint32_t)ip + kIMirror)) wd.invalidate();
        s = wd.get4((uint32_t)ip) & 0xffu;
        ip++;
        length += (int)s;
      }
    }
    const int mlen = length + (int)kMinMatch;
    if (op + mlen > oend - (int)kLastLiterals) return -ip - 1;    // lz4.cc:1024
    asm volatile("" ::: "memory");
    if ((uint32_t)off > kORing - 64u) {
      // the source left the ring -- or may have: the fast path's whole-step
      // stores reach up to 64 bytes past its output into slots of positions
      // kORing - 63 .. kORing back: read it back from this wave's own output
      // in HBM (ordered after the stores by a workgroup-scope release/acquire)
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int j = i + (int)lane;
        const uint8_t b = j < mlen ? o[ref + j] : (uint8_t)0;
        if (j < mlen) {
          RG(op + j) = b;
          o[op + j] = b;
        }
        asm volatile("" ::: "memory");
      }
    } else if (off >= mlen || off >= 64) {
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) {
        const int j = i + (int)lane;
        const uint8_t b = RG(ref + j);
        if (j < mlen) {
          RG(op + j) = b;
          o[op + j] = b;
        }
        asm volatile("" ::: "memory");
      }
    } else if (off > 0) {
      // periodic, sourced from the previous 64-byte step (never more than 64
      // bytes behind, so never overwritten in the ring)
      const int r0 = (int)lane - off * (int)((lanef + 0.5f) * __builtin_amdgcn_rcpf((float)off));
      const int rr = r0 < 0 ? r0 + off : (r0 >= off ? r0 - off : r0);
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) {
        const int j = i + (int)lane;
        const uint8_t b = RG(ref + i + rr);
        if (j < mlen) {
          RG(op + j) = b;
          o[op + j] = b;
        }
      }
    } else {
      // off == 0: the reference copies the destination onto itself (bytes it
      // never wrote: undefined) -- zeros here, never an earlier value's bytes
#pragma unroll 1
      for (int i = 0; i < mlen; i += 64) {
        const int j = i + (int)lane;
        if (j < mlen) {
          RG(op + j) = 0;
          o[op + j] = 0;
        }
      }
    }
    asm volatile("" ::: "memory");
    op += mlen;
  }
  return op;
#undef RG
}

// Values of this launch's class: out size > out_small or block > in_small.
template <bool kFrame, uint32_t kORing, uint32_t kIR, bool kWQ>
__device__ __forceinline__ void ring_decode_loop(
    uint8_t* const smem, const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t in_small, uint32_t out_small,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ out_cap, const uint32_t* __restrict__ target,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch,
    uint32_t nq) {
  const uint32_t lane = lane_id();
  uint8_t* ring = smem;
  uint8_t* iring = smem + kORing;
  // kWQ: claims of up to `batch` values from the launch's work queues -- a
  // mixed batch's ring pass scans every index (65 536 claims for 1 Mi
  // values), which one counter serves at ~65 claims/us: mixed decompress
  // 2.29 -> 2.00 ms.  Else one counter: the queues' state, live across the
  // decode, cost 3 % on 1 MiB parts (and 2-8 % in the in-place compressor,
  // which keeps its one counter; profiles/r04_d/r04_wq_ab_ring_queues.txt).
  WorkQueue wq = WorkQueue::make(work, n, batch, nq);
  bool direct_done = false;
#pragma unroll 1
  for (;;) {
    uint32_t c0 = 0, cnt = 0;
    if constexpr (kWQ) {
      if (wq.cur >= wq.end) wq.claim();          // a direct launch: value blockIdx.x, once
      if (wq.cur >= wq.end) break;
      c0 = wq.cur;
      cnt = wq.end - wq.cur;
      wq.cur = wq.end;
    } else {
      if (!work) {                               // direct launch: value blockIdx.x, once
        if (direct_done) break;
        c0 = blockIdx.x;
        direct_done = true;
      } else {
        if (lane == 0) c0 = atomicAdd(work, batch);
        c0 = uni(c0);
      }
      if (c0 >= n) break;
      cnt = min(batch, n - c0);
    }
    const uint32_t vi = c0 + lane;
    bool mine = false;
    if (lane < cnt) {
      const uint32_t avail = in_len[vi];
      uint32_t osz = out_cap[vi], csz = avail;
      if (kFrame) {
        const uint8_t* g = src + src_off[vi];
        if (avail >= 8u) {
          const uint32_t stored = (uint32_t)g[0] | ((uint32_t)g[1] << 8) | ((uint32_t)g[2] << 16) | ((uint32_t)g[3] << 24);
          const uint32_t raw = (uint32_t)g[4] | ((uint32_t)g[5] << 8) | ((uint32_t)g[6] << 16) | ((uint32_t)g[7] << 24);
          osz = raw;
          csz = stored - 8u;
          // raw frames (stored == 0) are copied by the LDS launch at any size
          mine = stored != 0 && raw <= out_cap[vi] && (osz > out_small || csz > in_small);
        }
      } else {
        mine = osz > out_small || csz > in_small;
      }
    }
    uint64_t todo = ballot(mine);
#pragma unroll 1
    while (todo) {
      const uint32_t l = (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1ull;
      const uint32_t v = c0 + l;
      const uint8_t* g = src + src_off[v];
      uint8_t* o = dst + dst_off[v];
      int csize, osize, tgt;
      if (kFrame) {
        const uint32_t stored =
            uni((uint32_t)g[0] | ((uint32_t)g[1] << 8) | ((uint32_t)g[2] << 16) | ((uint32_t)g[3] << 24));
        const uint32_t raw =
            uni((uint32_t)g[4] | ((uint32_t)g[5] << 8) | ((uint32_t)g[6] << 16) | ((uint32_t)g[7] << 24));
        const uint32_t avail = uni(in_len[v]);
        if (stored == 0) {                                        // raw frame (compressor.cc:116-124)
          if (raw + 8u > avail) {
            if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
            continue;
          }
          for (uint32_t i = lane; i < raw; i += 64u) o[i] = g[8u + i];
          if (lane == 0) { ret[v] = 0; out_len[v] = raw; }
          continue;
        }
        csize = (int)(stored - 8u);
        osize = (int)raw;
        tgt = osize;
        g += 8;
        if (csize < 0 || (uint32_t)csize + 8u > avail) {
          if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
          continue;
        }
      } else {
        csize = (int)uni(in_len[v]);
        osize = (int)uni(out_cap[v]);
        tgt = target ? (int)uni(target[v]) : osize;
        if (csize < 0 || osize < 0) {
          if (lane == 0) { ret[v] = kUnsupported; if (out_len) out_len[v] = 0; }
          continue;
        }
      }
      InRing<kIR> in{iring, g, (uint32_t)csize, 0u};
      const int r = decode_ring<kORing, kIR>(in, ring, o, csize, osize, tgt);
      if (lane == 0) {
        if (kFrame) {
          ret[v] = r > 0 ? 0 : -1;
          out_len[v] = r > 0 ? (uint32_t)r : 0u;
        } else {
          ret[v] = r;
          if (out_len) out_len[v] = r > 0 ? (uint32_t)r : 0u;
        }
      }
    }
  }
}

template <bool kFrame, uint32_t kORing>
__global__ __launch_bounds__(64) void lz4_decompress_big_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t in_small, uint32_t out_small,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ out_cap, const uint32_t* __restrict__ target,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work, uint32_t batch,
    uint32_t prio, uint32_t nq) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  if (prio) __builtin_amdgcn_s_setprio(2);     // a mixed batch's critical path (see launch_compress)
  ring_decode_loop<kFrame, kORing, 8192u, false>(smem, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                   out_len, ret, work, batch, nq);
}

// A batch with values on both sides of the LDS decoder's limit (a mixed
// batch): ONE persistent launch in the ring decoder's LDS.  Each wave first
// takes the ring decoder's values (the long ones), then -- once they are all
// claimed -- the LDS decoder's (outputs up to out_small, which the launch
// sizes so the staged block and window fit the same LDS), so the small values
// fill the tail of the long ones instead of splitting the CUs with them from
// the start (lz4_compress_mixed_kernel does the same on the write side).
template <bool kFrame, uint32_t kIR>
__global__ __launch_bounds__(64) void lz4_decompress_mixed_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t in_small, uint32_t out_small,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ out_cap, const uint32_t* __restrict__ target,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ ret, uint32_t* __restrict__ work_big, uint32_t batch_big,
    uint32_t* __restrict__ work_small, uint32_t batch_small, uint32_t nq) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  ring_decode_loop<kFrame, 4096u, kIR, kIR == 4096u>(smem, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                  out_len, ret, work_big, batch_big, nq);
  __syncthreads();
  small_decode_loop<kFrame, 5u>(smem, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                            out_len, ret, work_small, batch_small, 1u, nq);
}

// ---------------------------------------------------------------------------
// The resident decode service (service.h): one wave that serves per-call
// LZ4_decompress_safe_partial requests (lz4.cc:1050-1053, blocks whose output
// fits kSvcMaxOut) from a mailbox in pinned host memory, with the same
// staging and decode_block as small_decode_loop above.  Every wave reaches an
// exit: after idle_ticks of no requests, after life_ticks in all, or at the
// host's stop.  Host memory is read and written with system-scope atomics
// (doorbells, arguments, results) or plain vector loads/stores ordered by them.
__global__ __launch_bounds__(64) void lz4_decode_service_kernel(const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks,
                                                                uint64_t life_ticks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  constexpr uint32_t s_in_cap = (kSvcMaxIn + 32u + 15u) & ~15u;   // small_decode_loop's layout
  uint8_t* s_in = smem;
  uint8_t* s_out = smem + s_in_cap;
  const bool reply_on = __hip_atomic_load(&ibox->no_reply, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u;
  // the block staged at s_in (head 0) by svc_loop
  svc_loop(ibox, obox, gen, idle_ticks, life_ticks, s_in, kSvcMaxIn,
           [&](uint32_t sidx, const SvcArgs& a, const uint8_t** res) -> int {
    const int csize = (int)a.csize, osize = (int)a.osize, tgt = (int)a.target;
    int rc = (int)kUnsupported;
    if (csize >= 0 && osize >= 0 && (uint32_t)csize <= kSvcMaxIn && (uint32_t)osize <= kSvcMaxOut) {
      if (lane < 16u) s_in[(uint32_t)csize + lane] = 0;   // OOB bytes read as 0
      __syncthreads();
#if KDB_ABL_SVC_NOSERVE   // (attribution build: no decode, the output claimed -- timing only)
      rc = osize;
#else
      rc = decode_block(s_in, 0u, csize, s_out, osize, tgt);
#endif
      // a short result goes back in the slot's reply (svc_loop), the rest here
      if (rc > 0 && !(reply_on && svc_replies(sidx, rc))) flush_lds_to_global(obox->slot[sidx].out, s_out, 0, (uint32_t)rc);
      *res = s_out;   // the reply reads it before the next request's staging
    }
    return rc;
  });
}

hipError_t launch_decode_service(hipStream_t st, const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks,
                                 uint64_t life_ticks);

size_t decompress_lds_bytes(uint32_t max_in, uint32_t max_out) {
  // staged block (16 B alignment head + block + 16 zero bytes) | output window
  // + 64 B slack; the register window reaches 256 B past the block
  const size_t in_bytes = ((size_t)max_in + 32u + 15u) & ~(size_t)15u;
  const size_t out_bytes = (((size_t)max_out + 15u) & ~(size_t)15u) + 64u;
  return in_bytes + (out_bytes > 272u ? out_bytes : 272u);
}

// Waves per workgroup for the LDS decoder with `region` bytes per wave: the
// count that puts the most waves on a CU, by the measured allocation rule
// (LDS in 1 280-byte steps per workgroup out of 160 KiB; tools/probe/
// lds_occupancy, profiles/r05/r05_occ.txt) and capped by what the kernel's
// registers allow (the occupancy API for one-wave workgroups without LDS).
// KDB_LZ4_DWAVES (tuning builds) forces a count.
static uint32_t decode_waves(const void* kern, size_t region) {
  static const uint32_t forced = (uint32_t)kdb_tune("KDB_LZ4_DWAVES", 0);
  if (forced) return forced > 16u ? 16u : forced;
  int regs = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&regs, kern, 64, 0) != hipSuccess || regs < 1) return 1;
  constexpr size_t kStep = 1280, kLds = 163840;
  uint32_t best = 1, best_waves = 0;
  for (uint32_t w = 1; w <= 16; ++w) {
    const size_t need = (region * w + kStep - 1) / kStep * kStep;
    if (need > kLds) break;
    const uint32_t waves = std::min<uint32_t>((uint32_t)(kLds / need) * w, (uint32_t)regs);
    if (waves > best_waves) {
      best = w;
      best_waves = waves;
    }
  }
  return best;
}

template <bool F>
static hipError_t launch_one(hipStream_t st, size_t lds, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* in_len, uint32_t n, uint32_t max_in, uint32_t max_out, uint8_t* dst,
                             const uint64_t* dst_off, const uint32_t* out_cap, const uint32_t* target,
                             uint32_t* out_len, int32_t* ret, uint32_t skip_big) {
  // the register prefetch's depth: 3 chunks per lane when every frame of the
  // launch fits them (8 fewer VGPRs: 6 waves per SIMD instead of 5)
  const bool pf3 = max_in <= 3057u;
  auto kern = pf3 ? lz4_decompress_kernel<F, 3u> : lz4_decompress_kernel<F, 5u>;
  const uint32_t W = decode_waves(reinterpret_cast<const void*>(kern), lds);
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), lds * W, n, W);
  uint32_t* work = nullptr;
  hipError_t e = launch_counter(st, n, grid * W, &work);   // (waves >= values: wave b takes value b)
  if (e != hipSuccess) return e;
  const uint32_t batch = claim_batch(n, grid * W);
  launch_note(F ? (pf3 ? "lz4_decompress_kernel<true, 3u>" : "lz4_decompress_kernel<true, 5u>")
                : (pf3 ? "lz4_decompress_kernel<false, 3u>" : "lz4_decompress_kernel<false, 5u>"));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * W), lds * W, st, src, src_off, in_len, n, max_in, max_out, dst,
                     dst_off, out_cap, target, out_len, ret, work, batch, skip_big, work_queues(max_out),
                     decode_guide(max_out), (uint32_t)lds);
  e = hipGetLastError();
  const hipError_t r = work_counter_release(st, work);   // the slot is fenced even when the launch failed
  return e != hipSuccess ? e : r;
}

// decode_ring addresses its output ring as (p mod kORing) | base: the ring
// kernels must have no static LDS, so their dynamic LDS (the ring first)
// starts at address 0.  Checked once per kernel.
static bool ring_kernel_ok(const void* kern) {
  hipFuncAttributes a{};
  return hipFuncGetAttributes(&a, kern) == hipSuccess && a.sharedSizeBytes == 0;
}

template <bool F, uint32_t R>
static hipError_t launch_big(hipStream_t st, const uint8_t* src, const uint64_t* src_off, const uint32_t* in_len,
                             uint32_t n, uint32_t in_small, uint32_t out_small, uint8_t* dst, const uint64_t* dst_off,
                             const uint32_t* out_cap, const uint32_t* target, uint32_t* out_len, int32_t* ret) {
  auto kern = lz4_decompress_big_kernel<F, R>;
  static const bool ok = ring_kernel_ok(reinterpret_cast<const void*>(kern));
  if (!ok) return hipErrorInvalidDeviceFunction;
  static const uint32_t prio = env_prio();
  const size_t lds = ring_lds<R, 8192u>();
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), lds, n);
  uint32_t* work = nullptr;
  hipError_t e = launch_counter(st, n, grid, &work);
  if (e != hipSuccess) return e;
  const uint32_t batch = work ? claim_batch(n, grid) : 1u;   // values per claim; lanes >= batch idle
  static const std::string name = std::string(F ? "lz4_decompress_big_kernel<true, " : "lz4_decompress_big_kernel<false, ") +
                                  std::to_string(R) + "u>";
  launch_note(name.c_str());
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, st, src, src_off, in_len, n, in_small, out_small, dst,
                     dst_off, out_cap, target, out_len, ret, work, batch, prio, work_queues(out_small));
  e = hipGetLastError();
  const hipError_t r = work_counter_release(st, work);
  return e != hipSuccess ? e : r;
}


template <bool F>
static hipError_t launch_ring(hipStream_t st, const uint8_t* src, const uint64_t* src_off, const uint32_t* in_len,
                              uint32_t n, uint32_t in_small, uint32_t out_small, uint8_t* dst, const uint64_t* dst_off,
                              const uint32_t* out_cap, const uint32_t* target, uint32_t* out_len, int32_t* ret) {
  static const uint32_t ring = (uint32_t)kdb_tune("KDB_LZ4_ORING", 4096);
  switch (ring) {
    case 8192u:
      return launch_big<F, 8192u>(st, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                  out_len, ret);
    case 16384u:
      return launch_big<F, 16384u>(st, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                  out_len, ret);
    case 32768u:
      return launch_big<F, 32768u>(st, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                   out_len, ret);
    case 65536u:
      return launch_big<F, 65536u>(st, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                   out_len, ret);
    default:
      return launch_big<F, 4096u>(st, src, src_off, in_len, n, in_small, out_small, dst, dst_off, out_cap, target,
                                   out_len, ret);
  }
}

template <bool F, uint32_t kIR>
static hipError_t launch_mixed(hipStream_t st, const uint8_t* src, const uint64_t* src_off, const uint32_t* in_len,
                               uint32_t n, uint32_t in_small, uint32_t out_small, uint8_t* dst,
                               const uint64_t* dst_off, const uint32_t* out_cap, const uint32_t* target,
                               uint32_t* out_len, int32_t* ret) {
  auto kern = lz4_decompress_mixed_kernel<F, kIR>;
  static const bool ok = ring_kernel_ok(reinterpret_cast<const void*>(kern));
  if (!ok) return hipErrorInvalidDeviceFunction;
  const size_t lds = ring_lds<4096u, kIR>();
  if (decompress_lds_bytes(in_small, out_small) > lds) return hipErrorInvalidValue;   // the small pass's staging
  const uint32_t grid = persistent_grid(reinterpret_cast<const void*>(kern), lds, n);
  uint32_t *wb = nullptr, *ws = nullptr;
  hipError_t e = launch_counter(st, n, grid, &wb);
  if (e == hipSuccess) e = launch_counter(st, n, grid, &ws);
  if (e == hipSuccess) {
    const uint32_t bb = wb ? claim_batch(n, grid) : 1u, bs = claim_batch(n, grid);
    launch_note(F ? "lz4_decompress_mixed_kernel<true>" : "lz4_decompress_mixed_kernel<false>");
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, st, src, src_off, in_len, n, in_small, out_small, dst,
                       dst_off, out_cap, target, out_len, ret, wb, bb, ws, bs, work_queues(out_small));
    e = hipGetLastError();
  }
  const hipError_t r1 = work_counter_release(st, wb), r2 = work_counter_release(st, ws);
  return e != hipSuccess ? e : r1 != hipSuccess ? r1 : r2;
}

// LDS-resident decoder for outputs up to 65 546 bytes (blocks up to the bound
// of that, plus a frame header); the ring decoder after it for the rest.
constexpr uint32_t kOutSmallMax = k64KLimit - 1u;
// the LDS decoder's limit inside lz4_decompress_mixed_kernel: its staged block
// and window (decompress_lds_bytes) fit the ring decoder's LDS -- 12.8 KiB with
// the 8 KiB input ring, 8.7 KiB with the 4 KiB one
constexpr uint32_t kMixedOutSmall8 = 6144u, kMixedOutSmall4 = 4096u;
static_assert(kMixedOutSmall4 + kMixedOutSmall4 / 255u + 24u + 32u + 15u + kMixedOutSmall4 + 64u <= 4096u + 4096u + kIMirror,
              "the small pass's staging fits the 4 KiB input ring's LDS");

hipError_t launch_decode_service(hipStream_t st, const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks,
                                 uint64_t life_ticks) {
  const size_t lds = decompress_lds_bytes(kSvcMaxIn, kSvcMaxOut);
  hipLaunchKernelGGL(lz4_decode_service_kernel, dim3(1), dim3(64), lds, st, ibox, obox, gen, idle_ticks, life_ticks);
  return hipGetLastError();
}

hipError_t launch_decompress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* in_len, uint32_t n, uint32_t max_in, uint32_t max_out,
                             uint8_t* dst, const uint64_t* dst_off, const uint32_t* out_cap,
                             const uint32_t* target, uint32_t* out_len, int32_t* ret) {
  launch_notes_reset();
  if (n == 0) return hipSuccess;
  // LDS-resident decoder up to `split` output bytes, the ring decoder above
  static const uint32_t split = min((uint32_t)kdb_tune("KDB_LZ4_DSPLIT", 8192), kOutSmallMax);
  const uint32_t in_split = split + split / 255u + 16u + 8u;
  const bool big = max_out > split || max_in > in_split;
  const uint32_t mi = max_in < in_split ? max_in : in_split;
  const uint32_t mo = max_out < split ? max_out : split;
  const size_t lds = decompress_lds_bytes(mi, mo);
  // the ring decoder's class first, on a forked stream (its values take
  // longest); the two launches write disjoint values
  hipStream_t aux = st;
  hipError_t e = hipSuccess;
  // one block that the ring decoder owns (a scalar call): that launch alone
  const bool ring_only = !frame && n == 1u && big;
  // both classes: one launch (lz4_decompress_mixed_kernel), the LDS decoder's
  // limit lowered so that its staging fits the ring decoder's LDS
  static const bool combo_on = kdb_tune("KDB_LZ4_DMIXED", 1) != 0;
  if (big && !ring_only && combo_on) {
    // values whose output fits byU16 only: the 4 KiB input ring (see InRing)
    if (max_out <= kOutSmallMax) {
      const uint32_t mo2 = min(mo, kMixedOutSmall4), mi2 = min(mi, kMixedOutSmall4 + kMixedOutSmall4 / 255u + 16u + 8u);
      return frame ? launch_mixed<true, 4096u>(st, src, src_off, in_len, n, mi2, mo2, dst, dst_off, out_cap, target,
                                               out_len, ret)
                   : launch_mixed<false, 4096u>(st, src, src_off, in_len, n, mi2, mo2, dst, dst_off, out_cap, target,
                                                out_len, ret);
    }
    const uint32_t mo2 = min(mo, kMixedOutSmall8), mi2 = min(mi, kMixedOutSmall8 + kMixedOutSmall8 / 255u + 16u + 8u);
    return frame ? launch_mixed<true, 8192u>(st, src, src_off, in_len, n, mi2, mo2, dst, dst_off, out_cap, target,
                                             out_len, ret)
                 : launch_mixed<false, 8192u>(st, src, src_off, in_len, n, mi2, mo2, dst, dst_off, out_cap, target,
                                              out_len, ret);
  }
  if (ring_only)
    return frame ? launch_ring<true>(st, src, src_off, in_len, n, mi, mo, dst, dst_off, out_cap, target, out_len, ret)
                 : launch_ring<false>(st, src, src_off, in_len, n, mi, mo, dst, dst_off, out_cap, target, out_len,
                                      ret);
  // the join always follows once the fork began, whatever failed after it: a
  // caller that reuses its buffers after an error must not race the aux stream
  if (big) {
    if ((e = fork_begin(st, &aux)) != hipSuccess) return e;
    e = frame ? launch_ring<true>(aux, src, src_off, in_len, n, mi, mo, dst, dst_off, out_cap, target, out_len, ret)
              : launch_ring<false>(aux, src, src_off, in_len, n, mi, mo, dst, dst_off, out_cap, target, out_len, ret);
  }
  if (e == hipSuccess)
    e = frame ? launch_one<true>(st, lds, src, src_off, in_len, n, mi, mo, dst, dst_off, out_cap, target,
                                 out_len, ret, big ? 1u : 0u)
              : launch_one<false>(st, lds, src, src_off, in_len, n, mi, mo, dst, dst_off, out_cap, target,
                                  out_len, ret, big ? 1u : 0u);
  const hipError_t j = fork_end(st, aux);
  return e != hipSuccess ? e : j;
}

}  // namespace kdb_lz4
