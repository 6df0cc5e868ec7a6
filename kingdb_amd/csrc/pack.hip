// kingdb_amd/csrc/pack.hip -- packing of per-value frame slots into one dense
// frame stream, on the device, so only the frame bytes cross PCIe.
//
// The compress kernels write each value's frame into a fixed-size slot
// (frame_bound(S) bytes).  KingDB stores frames back to back (the value bytes
// of an HSTable entry, hstable_manager.h:656-673; multipart frames of one value,
// database.cc:143-248), so before the D2H copy the slots are compacted:
//   1. pack_scan_kernel: exclusive prefix sum of frame_len -> dst_off, total.
//      One workgroup; each thread owns a contiguous run (one read pass for the
//      run sums, one for the offsets) -- n*4 B in, n*8 B out, a few tens of us
//      at 1M values, against ~tens of ms of codec work.
//   2. pack_copy_kernel: one wave per value, dword-aligned stores on the
//      destination side (alignbyte of two aligned source dwords), byte stores
//      only at the ragged ends.  HBM-bound: 2*ΣF bytes.
#include "lz4_device.h"
#include "kdb_lz4.h"

namespace kdb_lz4 {

constexpr int kScanThreads = 1024;

__global__ __launch_bounds__(kScanThreads) void pack_scan_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                                 uint64_t* __restrict__ dst_off,
                                                                 uint64_t* __restrict__ total) {
  __shared__ uint64_t part[kScanThreads];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n + kScanThreads - 1) / kScanThreads;
  const uint64_t lo = (uint64_t)t * per;
  const uint64_t hi = lo + per < n ? lo + per : n;
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; i++) s += len[i];
  part[t] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan over the 1024 run sums
  for (uint32_t d = 1; d < kScanThreads; d <<= 1) {
    uint64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = part[t] - s;  // exclusive
  for (uint64_t i = lo; i < hi; i++) {
    dst_off[i] = run;
    run += len[i];
  }
  if (t == kScanThreads - 1) *total = part[t];
}

__device__ __forceinline__ uint32_t ld32a(const uint8_t* p) { return *(const uint32_t*)p; }

__global__ __launch_bounds__(256) void pack_copy_kernel(const uint8_t* __restrict__ src,
                                                        const uint64_t* __restrict__ src_off,
                                                        const uint32_t* __restrict__ len, uint32_t n,
                                                        uint8_t* __restrict__ dst,
                                                        const uint64_t* __restrict__ dst_off) {
  const uint32_t lane = lane_id();
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t v = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; v < n; v += nw) {
    const uint32_t L = len[v];
    if (L == 0) continue;
    const uint64_t so = src_off[v], d0 = dst_off[v];
    const uint64_t da = d0 & ~3ull;
    const uint64_t nd = (((d0 + L + 3) & ~3ull) - da) >> 2;
    for (uint64_t k = lane; k < nd; k += 64) {
      const uint64_t dpos = da + 4 * k;
      const int64_t rel = (int64_t)dpos - (int64_t)d0;
      if (rel >= 0 && rel + 4 <= (int64_t)L) {
        const uint64_t s = so + (uint64_t)rel;
        const uint64_t sa = s & ~3ull;
        const uint32_t sh = (uint32_t)(s & 3);
        const uint32_t w0 = ld32a(src + sa);
        const uint32_t w1 = sh ? ld32a(src + sa + 4) : 0u;
        *(uint32_t*)(dst + dpos) = __builtin_amdgcn_alignbyte(w1, w0, sh);
      } else {
        for (int b = 0; b < 4; b++) {
          const int64_t r = rel + b;
          if (r >= 0 && r < (int64_t)L) dst[dpos + b] = src[so + (uint64_t)r];
        }
      }
    }
  }
}

}  // namespace kdb_lz4

using namespace kdb_lz4;

extern "C" int kdb_lz4_pack_frames(void* stream, const uint8_t* src, const uint64_t* src_off,
                                   const uint32_t* len, uint32_t n, uint8_t* dst, uint64_t* dst_off,
                                   uint64_t* total) {
  if ((n && (!src || !src_off || !len || !dst || !dst_off)) || !total) return KDB_LZ4_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return hipMemsetAsync(total, 0, 8, st) == hipSuccess ? KDB_LZ4_OK : KDB_LZ4_EHIP;
  hipLaunchKernelGGL(pack_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, len, n, dst_off, total);
  if (hipGetLastError() != hipSuccess) return KDB_LZ4_EHIP;
  const uint32_t waves = n < 65536u ? n : 65536u;
  hipLaunchKernelGGL(pack_copy_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, src, src_off, len, n, dst,
                     dst_off);
  return hipGetLastError() == hipSuccess ? KDB_LZ4_OK : KDB_LZ4_EHIP;
}
