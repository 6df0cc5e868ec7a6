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
#include <atomic>
#include <mutex>
#include <unordered_map>

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

// ---------------------------------------------------------------------------
// Device-wide exclusive scan of u32 lengths into u64 offsets (+ total), in
// three launches: per-block sums, a scan of the block sums (one block), then
// the per-block scan with its block's base.  A block covers kScanTile
// elements (16 per thread).  The block sums live in a per-device ring of
// scratch slots (one per launch, reused after kScanSlots later launches, like
// the work counters); inputs past kScanSlotSums blocks fall back to the
// single-workgroup kernel above.
constexpr uint32_t kScanBlock = 256, kScanPer = 16, kScanTile = kScanBlock * kScanPer;
constexpr uint32_t kScanSlots = 1024, kScanSlotSums = 1024;   // <= 4 Mi elements per scan

__device__ __forceinline__ uint64_t block_exclusive(uint64_t v, uint64_t* sh, uint64_t* total) {
  // exclusive scan of one u64 per thread over the block (wave shuffles + LDS)
  const uint32_t t = threadIdx.x, lane = lane_id(), w = t / 64u;
  uint64_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint64_t base = 0, all = 0;
  for (uint32_t k = 0; k < kScanBlock / 64u; k++) {
    if (k < w) base += sh[k];
    all += sh[k];
  }
  __syncthreads();
  *total = all;
  return base + x - v;
}

__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                                 uint64_t* __restrict__ sums) {
  __shared__ uint64_t sh[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++)
    if (base + k < n) s += len[base + k];
  uint64_t tot;
  block_exclusive(s, sh, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanBlock) void scan_top_kernel(uint64_t* __restrict__ sums, uint32_t nb,
                                                                uint64_t* __restrict__ total) {
  __shared__ uint64_t sh[kScanBlock / 64];
  // nb <= kScanSlotSums: at most 4 sums per thread
  const uint32_t per = (nb + kScanBlock - 1) / kScanBlock;
  const uint32_t lo = threadIdx.x * per;
  uint64_t s = 0;
  for (uint32_t k = 0; k < per; k++)
    if (lo + k < nb) s += sums[lo + k];
  uint64_t tot;
  uint64_t run = block_exclusive(s, sh, &tot);
  for (uint32_t k = 0; k < per; k++)
    if (lo + k < nb) {
      const uint64_t v = sums[lo + k];
      sums[lo + k] = run;
      run += v;
    }
  if (threadIdx.x == 0) *total = tot;
}

__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                                  const uint64_t* __restrict__ sums,
                                                                  uint64_t* __restrict__ off) {
  __shared__ uint64_t sh[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  uint32_t v[kScanPer];
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++) {
    v[k] = base + k < n ? len[base + k] : 0u;
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = sums[blockIdx.x] + block_exclusive(s, sh, &tot);
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++)
    if (base + k < n) {
      off[base + k] = run;
      run += v[k];
    }
}

namespace {
std::mutex g_scan_mu;
std::unordered_map<int, std::pair<uint64_t*, std::atomic<uint32_t>*>> g_scan_pools;
}  // namespace

hipError_t launch_exclusive_scan(hipStream_t st, const uint32_t* len, uint32_t n, uint64_t* off, uint64_t* total) {
  const uint32_t nb = (n + kScanTile - 1) / kScanTile;
  if (n == 0) return hipMemsetAsync(total, 0, 8, st);
  if (nb > kScanSlotSums) {
    hipLaunchKernelGGL(pack_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, len, n, off, total);
    return hipGetLastError();
  }
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  uint64_t* slot;
  {
    std::lock_guard<std::mutex> l(g_scan_mu);
    auto& p = g_scan_pools[dev];
    if (!p.first) {
      e = hipMalloc(&p.first, (size_t)kScanSlots * kScanSlotSums * 8u);
      if (e != hipSuccess) return e;
      p.second = new std::atomic<uint32_t>(0);
    }
    slot = p.first + (size_t)(p.second->fetch_add(1) % kScanSlots) * kScanSlotSums;
  }
  hipLaunchKernelGGL(scan_sums_kernel, dim3(nb), dim3(kScanBlock), 0, st, len, n, slot);
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(kScanBlock), 0, st, slot, nb, total);
  hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(kScanBlock), 0, st, len, n, slot, off);
  return hipGetLastError();
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

// *out = max(*out, v[0..n)): grid-stride over 16-byte loads, a wave-wide max,
// the block's four waves through LDS, one atomicMax per block.  (One atomic
// per wave on the one address -- 4 096 of them for 1 Mi values -- serialised
// at the memory side: 50 us per call, inside every bench step.)
__global__ __launch_bounds__(256) void max_u32_kernel(const uint32_t* __restrict__ v, uint32_t n,
                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t wmax[4];
  uint32_t m = 0;
  const uint32_t n4 = n >> 2, stride = gridDim.x * blockDim.x;
  const uint4* v4 = reinterpret_cast<const uint4*>(v);
  const bool aligned = (reinterpret_cast<uintptr_t>(v) & 15u) == 0;
  if (aligned) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      const uint4 q = v4[i];
      m = max(m, max(max(q.x, q.y), max(q.z, q.w)));
    }
  }
  for (uint32_t i = (aligned ? n4 << 2 : 0u) + blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    m = max(m, v[i]);
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
  if (lane_id() == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (m) atomicMax(out, m);
  }
}

}  // namespace kdb_lz4

using namespace kdb_lz4;

extern "C" int kdb_lz4_max_u32(void* stream, const uint32_t* v, uint32_t n, uint32_t* out) {
  if ((n && !v) || !out) return KDB_LZ4_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(out, 0, 4, st) != hipSuccess) return KDB_LZ4_EHIP;
  if (n == 0) return KDB_LZ4_OK;
  const uint32_t blocks = min((n + 1023u) / 1024u, 256u);
  hipLaunchKernelGGL(max_u32_kernel, dim3(blocks), dim3(256), 0, st, v, n, out);
  return hipGetLastError() == hipSuccess ? KDB_LZ4_OK : KDB_LZ4_EHIP;
}

extern "C" int kdb_lz4_pack_frames(void* stream, const uint8_t* src, const uint64_t* src_off,
                                   const uint32_t* len, uint32_t n, uint8_t* dst, uint64_t* dst_off,
                                   uint64_t* total) {
  if ((n && (!src || !src_off || !len || !dst || !dst_off)) || !total) return KDB_LZ4_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return hipMemsetAsync(total, 0, 8, st) == hipSuccess ? KDB_LZ4_OK : KDB_LZ4_EHIP;
  if (launch_exclusive_scan(st, len, n, dst_off, total) != hipSuccess) return KDB_LZ4_EHIP;
  const uint32_t waves = n < 65536u ? n : 65536u;
  hipLaunchKernelGGL(pack_copy_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, src, src_off, len, n, dst,
                     dst_off);
  return hipGetLastError() == hipSuccess ? KDB_LZ4_OK : KDB_LZ4_EHIP;
}
