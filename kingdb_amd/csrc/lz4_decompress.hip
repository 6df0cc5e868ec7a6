// kingdb_amd/csrc/lz4_decompress.hip -- gfx950 LZ4 r1.3.0 block decoder.
//
// Replaces LZ4_decompress_safe_partial (/root/reference/algorithm/lz4.cc:1050-1053)
// = LZ4_decompress_generic(endOnInputSize, partial, target=max, noDict)
// (lz4.cc:876-1042), and -- in frame mode -- CompressorLZ4::Uncompress's frame
// handling (algorithm/compressor.cc:75-137).  Successful decodes are bit-exact;
// malformed blocks return the reference's exact code -(consumed)-1.
//
// One wavefront per value.  The compressed block is staged HBM -> LDS with
// aligned 16-byte loads; the value is rebuilt in an LDS window (the match
// source is always earlier output) and written back to HBM in one coalesced
// pass.  Token/length parsing is wave-uniform scalar work; literal runs and
// match copies are lane-parallel.  An overlapping match (offset < length) is a
// periodic extension of the `offset` bytes before it, so lane i reads
// out[ref + (i mod offset)] -- every source byte is already final and the copy
// is one parallel pass (equivalent to the reference's dec32/dec64 trick,
// lz4.cc:1008-1018).
#include "lz4_device.h"

namespace kdb_lz4 {

// Decodes the block at in[0..csize) into out[0..osize) (both LDS).
// Bytes read at or past csize read as 0 (see oracle/lz4_oracle.c).
__device__ int decode_block(const uint8_t* __restrict__ in, int csize, uint8_t* __restrict__ out,
                            int osize, int target) {
  const uint32_t lane = lane_id();
  const int iend = csize, oend = osize;
  const int oexit = min(target, oend - (int)kMfLimit);           // lz4.cc:908-910
#define INB(i) ((uint32_t)uni(((i) >= 0 && (i) < iend) ? (uint32_t)in[(i)] : 0u))
  if (osize == 0) return (csize == 1 && INB(0) == 0) ? 0 : -1;   // lz4.cc:911
  int ip = 0, op = 0;
  for (;;) {
    const uint32_t token = INB(ip);
    ip++;
    int length = (int)(token >> 4);
    if (length == (int)kRunMask) {                                // lz4.cc:917-925
      uint32_t s;
      do {
        s = INB(ip);
        ip++;
        length += (int)s;
      } while (ip < iend - (int)kRunMask && s == 255u);
    }
    const int cpy = op + length;                                  // lz4.cc:930-952
    const bool last = cpy > oexit || ip + length > iend - (int)(2 + 1 + kLastLiterals);
    if (last) {
      if (cpy > oend) return -ip - 1;
      if (ip + length > iend) return -ip - 1;
    }
    for (int i = (int)lane; i < length; i += 64) out[op + i] = in[ip + i];
    ip += length;
    op = cpy;
    if (last) break;
    // offset (lz4.cc:955-956)
    const int off = (int)(INB(ip) | (INB(ip + 1) << 8));
    ip += 2;
    const int ref = op - off;
    if (ref < 0) return -ip - 1;
    // match length (lz4.cc:959-968)
    length = (int)(token & kMlMask);
    if (length == (int)kMlMask) {
      uint32_t s;
      do {
        if (ip > iend - (int)kLastLiterals) return -ip - 1;
        s = INB(ip);
        ip++;
        length += (int)s;
      } while (s == 255u);
    }
    const int mlen = length + (int)kMinMatch;
    if (op + mlen > oend - (int)kLastLiterals) return -ip - 1;   // lz4.cc:1024
    asm volatile("" ::: "memory");
    if (off >= mlen) {
      for (int i = (int)lane; i < mlen; i += 64) out[op + i] = out[ref + i];
    } else if (off > 0) {
      // periodic: out[op+i] = out[ref + i mod off]
      int j = (int)lane % off;
      const int step = 64 % off;
      for (int i = (int)lane; i < mlen; i += 64) {
        out[op + i] = out[ref + j];
        j += step;
        if (j >= off) j -= off;
      }
    }  // off == 0: the reference copies the destination onto itself
    asm volatile("" ::: "memory");
    op += mlen;
  }
#undef INB
  return op;
}

// kFrame = false: block mode. in_len[v] = C, out_cap[v] = S (target = max);
//   ret[v] = LZ4 return code, out_len[v] = max(ret, 0).
// kFrame = true : one CompressorLZ4 frame per value at src + src_off[v]
//   (header u32 size_compressed_stored, u32 size_source); in_len[v] = bytes
//   available there; ret[v] = 0 (OK) / -1 (IOError); out_len[v] = *size_dest.
template <bool kFrame>
__global__ __launch_bounds__(64) void lz4_decompress_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t in_cap, uint32_t out_cap_max,
    uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
    const uint32_t* __restrict__ out_cap, const uint32_t* __restrict__ target,
    uint32_t* __restrict__ out_len, int32_t* __restrict__ ret) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t v = blockIdx.x;
  if (v >= n) return;
  const uint32_t lane = lane_id();
  const uint8_t* g = src + src_off[v];
  uint8_t* o = dst + dst_off[v];
  int csize, osize, tgt;
  if (kFrame) {
    // compressor.cc:89-90 (GetFixed32 x2)
    const uint32_t stored =
        uni((uint32_t)g[0] | ((uint32_t)g[1] << 8) | ((uint32_t)g[2] << 16) | ((uint32_t)g[3] << 24));
    const uint32_t raw =
        uni((uint32_t)g[4] | ((uint32_t)g[5] << 8) | ((uint32_t)g[6] << 16) | ((uint32_t)g[7] << 24));
    const uint32_t avail = uni(in_len[v]);
    if (raw > out_cap[v]) {
      if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
      return;
    }
    if (stored == 0) {  // raw frame (compressor.cc:116-124)
      if (raw + 8u > avail) {
        if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
        return;
      }
      for (uint32_t i = lane; i < raw; i += 64u) o[i] = g[8u + i];
      if (lane == 0) { ret[v] = 0; out_len[v] = raw; }
      return;
    }
    csize = (int)(stored - 8u);          // compressor.cc:96 (u32 wrap kept: int cast)
    osize = (int)raw;
    tgt = osize;                         // compressor.cc:103-107: target = max = size_source
    g += 8;
    if (csize < 0 || (uint32_t)csize + 8u > avail) {
      // a negative size makes the reference return -2/-3 (IOError); a size past
      // the bytes supplied would have it read foreign memory: IOError as well.
      if (lane == 0) { ret[v] = -1; out_len[v] = 0; }
      return;
    }
  } else {
    csize = (int)uni(in_len[v]);
    osize = (int)uni(out_cap[v]);
    tgt = target ? (int)uni(target[v]) : osize;
  }
  if ((uint32_t)csize > in_cap || (uint32_t)osize > out_cap_max || csize < 0 || osize < 0) {
    if (lane == 0) { ret[v] = kUnsupported; if (out_len) out_len[v] = 0; }
    return;
  }
  const uint32_t out_bytes = (out_cap_max + 15u) & ~15u;
  uint8_t* s_out = smem;
  uint8_t* s_in = smem + out_bytes + 16u;
  const uint32_t head = stage_to_lds(g, (uint32_t)csize, s_in);
  __syncthreads();
  const int r = decode_block(s_in + head, csize, s_out, osize, tgt);
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
}

size_t decompress_lds_bytes(uint32_t max_in, uint32_t max_out) {
  return (((size_t)max_out + 15u) & ~(size_t)15u) + 16u + (((size_t)max_in + 15u) & ~(size_t)15u) + 48u;
}

hipError_t launch_decompress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* in_len, uint32_t n, uint32_t max_in, uint32_t max_out,
                             uint8_t* dst, const uint64_t* dst_off, const uint32_t* out_cap,
                             const uint32_t* target, uint32_t* out_len, int32_t* ret) {
  if (n == 0) return hipSuccess;
  const size_t lds = decompress_lds_bytes(max_in, max_out);
  if (frame) {
    hipLaunchKernelGGL(lz4_decompress_kernel<true>, dim3(n), dim3(64), lds, st, src, src_off, in_len,
                       n, max_in, max_out, dst, dst_off, out_cap, target, out_len, ret);
  } else {
    hipLaunchKernelGGL(lz4_decompress_kernel<false>, dim3(n), dim3(64), lds, st, src, src_off,
                       in_len, n, max_in, max_out, dst, dst_off, out_cap, target, out_len, ret);
  }
  return hipGetLastError();
}

}  // namespace kdb_lz4
