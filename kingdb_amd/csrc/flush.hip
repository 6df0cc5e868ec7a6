// kingdb_amd/csrc/flush.hip -- the write-buffer flush batch (include/kdb_flush.h,
// SURVEY.md §8 row f3): PutPartValidSize's compression, disable rule, offsets
// and running CRC32C for parts that client threads queued raw, each thread's
// state carried across batches.
//
// Reference (/root/reference/interface/database.cc:143-267), per part, over
// the thread's ThreadStorage slots (thread/threadstorage.h:23-46):
//   first part (offset 0): compression enabled, ts_offset 0 (:159-162)
//   disabled: offset = ts_offset, ts_offset += chunk (:164-171)
//   non-empty and enabled: the compressor's total restarts at a first part
//     (:177-179), offset = that total (:182), Compress (:185-189), and the
//     disable rule (:196-209) swaps the frame for 8 zero bytes + the chunk
//   last part: size_value_compressed (:237-248)
//   CRC32C restarts at a first part with the key, then every chunk_final (:251-257)
//   the allocation check (:261-266) rejects the part (IOError) after all that
//
// Pipeline (stream-ordered):
//   flush_prep_kernel     thread per part: frame slot sizes
//   scan                  slot offsets
//   frame compress        every part (launch_compress): a part the policy then
//                         takes raw simply ignores its frame
//   flush_policy_kernel   thread per run: the rules above, in order
//   pack                  the frames the policy kept, back to back (kdb_lz4_pack_frames)
//   flush_crc_small_kernel  thread per segment of one part that starts a value
//                         and whose key + chunk_final fit 512 bytes: one pass
//   flush_crc_kernel      wave per other segment: crc::extend_wave per piece
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/kdb_flush.h"
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

constexpr uint32_t kSmallSeg = 512;     // key + chunk_final bytes a thread takes alone

__host__ __device__ __forceinline__ uint64_t padding_size(uint64_t size_value) {   // format.h:63-71
  return (size_value / 65536u + 1u) * 8u;
}

__global__ void flush_prep_kernel(const uint32_t* __restrict__ chunk_len, uint32_t n, uint32_t* __restrict__ slot) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x)
    slot[p] = (8u + compress_bound(chunk_len[p]) + 15u) & ~15u;
}

// Thread per run: PutPartValidSize over the run's parts, in order.
__global__ void flush_policy_kernel(const uint32_t* __restrict__ key_len, const uint32_t* __restrict__ chunk_len,
                                    const uint64_t* __restrict__ offset_chunk,
                                    const uint64_t* __restrict__ size_value, const uint32_t* __restrict__ seg_first,
                                    const uint32_t* __restrict__ run_first, const kdb_flush_state* __restrict__ cin,
                                    const uint32_t* __restrict__ frame_len, const int32_t* __restrict__ fstatus,
                                    uint32_t nruns, kdb_flush_part* __restrict__ parts,
                                    uint32_t* __restrict__ pack_len, uint32_t* __restrict__ seg_flag,
                                    uint32_t* __restrict__ big, kdb_flush_state* __restrict__ cout) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += gridDim.x * blockDim.x) {
    kdb_flush_state S = cin[r];
    for (uint32_t s = run_first[r]; s < run_first[r + 1]; s++) {
      const uint32_t p0 = seg_first[s], p1 = seg_first[s + 1];
      uint64_t crc_bytes = 0;
      bool any_failed = false;
      for (uint32_t p = p0; p < p1; p++) {
        const uint64_t csz = chunk_len[p], off = offset_chunk[p], V = size_value[p];
        const uint64_t pad = padding_size(V);
        const bool first = off == 0, last = csz + off == V;
        const bool do_comp = csz != 0;                                     // :154-157
        uint64_t o = off;
        if (first) { S.enabled = 1u; S.ts_offset = 0; }                    // :159-162
        if (!S.enabled) { o = S.ts_offset; S.ts_offset = o + csz; }         // :164-171
        kdb_flush_part P{};
        P.mode = KDB_FLUSH_RAW;
        P.size = (uint32_t)csz;
        if (do_comp && S.enabled) {
          if (first) S.comp_total = 0;                                     // :177-179
          o = S.comp_total;                                                // :182
          if (fstatus[p] != 0) {                                           // :189: IOError, nothing more
            P.mode = KDB_FLUSH_FAILED;
            P.status = -1;
            P.occ = o;
            parts[p] = P;
            pack_len[p] = 0;
            any_failed = true;
            continue;
          }
          const uint64_t F = frame_len[p];
          S.comp_total += F;
          const uint64_t size_remaining = V - off;                         // :197-199 (unsigned, as there)
          const uint64_t space_left = V + pad - o;
          if (size_remaining - csz + 8u > space_left - F) {                // :199-209
            S.comp_total -= F;
            P.size = (uint32_t)(csz + 8u);
            S.enabled = 0u;
            S.ts_offset = S.comp_total + P.size;
            P.mode = KDB_FLUSH_DISABLED;
          } else {
            P.mode = KDB_FLUSH_FRAME;
            P.size = (uint32_t)F;
          }
        }
        if (do_comp && last)                                               // :237-248
          P.svc = S.enabled ? S.comp_total : (first ? S.ts_offset : o + csz);
        if (o + P.size > V + (do_comp ? pad : 0u)) P.status = -1;          // :261-266 (after the CRC)
        P.occ = o;
        parts[p] = P;
        pack_len[p] = P.mode == KDB_FLUSH_FRAME && P.status == 0 ? P.size : 0u;
        crc_bytes += P.size;
      }
      // a segment the one-thread CRC takes: one part, starting the value, small, not failed
      const bool small = p1 - p0 == 1u && offset_chunk[p0] == 0 && !any_failed &&
                         (uint64_t)key_len[s] + crc_bytes <= kSmallSeg;
      // flag: bit 0 small; bits 1..: 1 + the run's index when the segment is the run's last
      seg_flag[s] = (small ? 1u : 0u) | (s + 1 == run_first[r + 1] ? (r + 1u) << 1 : 0u);
      if (!small) big[1u + atomicAdd(big, 1u)] = s;
    }
    S.crc = 0;   // the CRC kernels write it
    cout[r] = S;
  }
}

// Byte j of part p's chunk_final.
struct PartMsg {
  const uint8_t* src;   // the frame slot (FRAME) or the chunk
  uint32_t skip;        // leading zero bytes (DISABLED: 8)
  __device__ uint32_t feed(uint64_t a, uint64_t b, uint32_t c, const uint32_t* s_t) const {
    uint64_t m = a;
    for (; m < b && m < skip; m++) c = crc::step(c, 0u, s_t);
    for (; m < b; m++) c = crc::step(c, src[m - skip], s_t);
    return c;
  }
};
struct KeyMsg {
  const uint8_t* k;
  __device__ uint32_t feed(uint64_t a, uint64_t b, uint32_t c, const uint32_t* s_t) const {
    for (uint64_t m = a; m < b; m++) c = crc::step(c, k[m], s_t);
    return c;
  }
};

__device__ __forceinline__ PartMsg part_msg(const kdb_flush_part& P, const uint8_t* chunks, uint64_t chunk_off,
                                            const uint8_t* slots, uint64_t slot_off) {
  if (P.mode == KDB_FLUSH_FRAME) return PartMsg{slots + slot_off, 0u};
  return PartMsg{chunks + chunk_off, P.mode == KDB_FLUSH_DISABLED ? 8u : 0u};
}

__global__ __launch_bounds__(256) void flush_crc_small_kernel(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, const uint32_t* __restrict__ key_len,
    const uint8_t* __restrict__ chunks, const uint64_t* __restrict__ chunk_off,
    const uint32_t* __restrict__ chunk_len, const uint64_t* __restrict__ offset_chunk,
    const uint64_t* __restrict__ size_value, const uint32_t* __restrict__ seg_first,
    const uint32_t* __restrict__ seg_flag, const uint8_t* __restrict__ slots, const uint64_t* __restrict__ slot_off,
    const uint64_t* __restrict__ frame_at, uint32_t nseg, kdb_flush_part* __restrict__ parts,
    kdb_flush_state* __restrict__ cout) {
  __shared__ uint32_t s_t[256];
  crc::stage_table(s_t);
  __syncthreads();
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
    const uint32_t f = seg_flag[s];
    if (!(f & 1u)) continue;
    const uint32_t p = seg_first[s];
    const kdb_flush_part P = parts[p];
    uint32_t c = 0xFFFFFFFFu;                      // crc restarted at 0 (:253), then the key (:254)
    const uint8_t* k = keys + key_off[s];
    for (uint32_t i = 0, kl = key_len[s]; i < kl; i++) c = crc::step(c, k[i], s_t);
    c = part_msg(P, chunks, chunk_off[p], slots, slot_off[p]).feed(0, P.size, c, s_t);   // :256
    const uint32_t crc = c ^ 0xFFFFFFFFu;
    parts[p].crc = (uint64_t)chunk_len[p] + offset_chunk[p] == size_value[p] ? crc : 0u;   // :257
    parts[p].frame_at = frame_at[p];
    if (f >> 1) cout[(f >> 1) - 1u].crc = crc;
  }
}

// Wave per listed segment: the running CRC over the key (a segment that starts
// a value) or the carried CRC, then each part's chunk_final.
__global__ __launch_bounds__(256) void flush_crc_kernel(
    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, const uint32_t* __restrict__ key_len,
    const uint8_t* __restrict__ chunks, const uint64_t* __restrict__ chunk_off,
    const uint32_t* __restrict__ chunk_len, const uint64_t* __restrict__ offset_chunk,
    const uint64_t* __restrict__ size_value, const uint32_t* __restrict__ seg_first,
    const uint32_t* __restrict__ seg_flag, const uint32_t* __restrict__ run_first,
    const kdb_flush_state* __restrict__ cin, const uint8_t* __restrict__ slots,
    const uint64_t* __restrict__ slot_off, const uint64_t* __restrict__ frame_at, const uint32_t* __restrict__ big,
    uint32_t nruns, kdb_flush_part* __restrict__ parts, kdb_flush_state* __restrict__ cout) {
  __shared__ uint32_t s_t[256];
  crc::stage_table(s_t);
  __syncthreads();
  const uint32_t nbig = big[0];
  const uint32_t lane = lane_id();
  const uint32_t nw = gridDim.x * (blockDim.x / 64u);
  for (uint32_t i = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u; i < nbig; i += nw) {
    const uint32_t s = uni(big[1u + i]);
    const uint32_t p0 = uni(seg_first[s]), p1 = uni(seg_first[s + 1]);
    uint32_t c;
    if (offset_chunk[p0] == 0) {                   // :252-255
      c = crc::extend_wave(0u, key_len[s], KeyMsg{keys + key_off[s]}, s_t);
    } else {                                       // continues the run's carried CRC
      uint32_t lo = 0, hi = nruns;                 // the run holding s: last r with run_first[r] <= s
      while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) / 2u;
        if (run_first[mid] <= s) lo = mid; else hi = mid;
      }
      c = cin[lo].crc;
    }
    for (uint32_t p = p0; p < p1; p++) {
      const kdb_flush_part P = parts[p];
      if (P.mode != KDB_FLUSH_FAILED)
        c = crc::extend_wave(c, P.size, part_msg(P, chunks, chunk_off[p], slots, slot_off[p]), s_t);
      if (lane == 0) {
        parts[p].crc = P.mode != KDB_FLUSH_FAILED && (uint64_t)chunk_len[p] + offset_chunk[p] == size_value[p] ? c : 0u;
        parts[p].frame_at = frame_at[p];
      }
    }
    const uint32_t f = seg_flag[s];
    if (lane == 0 && (f >> 1)) cout[(f >> 1) - 1u].crc = c;
  }
}

__global__ void zero_u64_kernel(uint64_t* p) { *p = 0; }

}  // namespace

uint64_t flush_scratch_bytes(uint32_t nparts, uint32_t nseg, uint64_t raw_bytes) {
  const uint64_t slots = raw_bytes + raw_bytes / 255u + (uint64_t)nparts * 40u + 64u;
  const uint64_t per_part = (uint64_t)nparts * (4 + 8 + 4 + 4 + 4 + 8);
  const uint64_t per_seg = (uint64_t)nseg * (4 + 4) + 8;
  return slots + per_part + per_seg + 10u * 256u;
}

hipError_t launch_flush(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len,
                        const uint8_t* chunks, const uint64_t* chunk_off, const uint32_t* chunk_len,
                        const uint64_t* offset_chunk, const uint64_t* size_value, const uint32_t* seg_first,
                        const uint32_t* run_first, const kdb_flush_state* carry_in, uint32_t nparts, uint32_t nseg,
                        uint32_t nruns, uint32_t max_chunk, uint8_t* scratch, uint64_t raw_bytes,
                        kdb_flush_part* parts, kdb_flush_state* carry_out, uint8_t* frames,
                        uint64_t* frames_total) {
  uint8_t* s = scratch;
  auto take = [&](uint64_t bytes) {
    uint8_t* r = s;
    s += (bytes + 255u) & ~255ull;
    return r;
  };
  uint8_t* slots = take(raw_bytes + raw_bytes / 255u + (uint64_t)nparts * 40u + 64u);
  uint32_t* slot_len = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  uint64_t* slot_off = reinterpret_cast<uint64_t*>(take((uint64_t)nparts * 8u));
  uint32_t* frame_len = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  int32_t* fstatus = reinterpret_cast<int32_t*>(take((uint64_t)nparts * 4u));
  uint32_t* pack_len = reinterpret_cast<uint32_t*>(take((uint64_t)nparts * 4u));
  uint64_t* frame_at = reinterpret_cast<uint64_t*>(take((uint64_t)nparts * 8u));
  uint32_t* seg_flag = reinterpret_cast<uint32_t*>(take((uint64_t)nseg * 4u));
  uint32_t* big = reinterpret_cast<uint32_t*>(take(4u + (uint64_t)nseg * 4u));   // count, then segment ids
  uint64_t* slots_total = reinterpret_cast<uint64_t*>(take(8));
  if (nparts == 0) {
    hipLaunchKernelGGL(zero_u64_kernel, dim3(1), dim3(1), 0, st, frames_total);
    return hipGetLastError();
  }
  const uint32_t tb = 256;
  auto grid = [&](uint32_t n) { return (n + tb - 1) / tb < 4096u ? (n + tb - 1) / tb : 4096u; };
  hipLaunchKernelGGL(flush_prep_kernel, dim3(grid(nparts)), dim3(tb), 0, st, chunk_len, nparts, slot_len);
  hipError_t e = launch_exclusive_scan(st, slot_len, nparts, slot_off, slots_total);
  if (e != hipSuccess) return e;
  e = launch_compress(true, st, chunks, chunk_off, chunk_len, nparts, 0u, max_chunk, slots, slot_off, nullptr,
                      frame_len, fstatus);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(big, 0, 4, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(flush_policy_kernel, dim3(grid(nruns)), dim3(tb), 0, st, key_len, chunk_len, offset_chunk,
                     size_value, seg_first, run_first, carry_in, frame_len, fstatus, nruns, parts, pack_len, seg_flag,
                     big, carry_out);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (kdb_lz4_pack_frames(st, slots, slot_off, pack_len, nparts, frames, frame_at, frames_total) != KDB_LZ4_OK)
    return hipErrorLaunchFailure;
  hipLaunchKernelGGL(flush_crc_small_kernel, dim3(grid(nseg)), dim3(tb), 0, st, keys, key_off, key_len, chunks,
                     chunk_off, chunk_len, offset_chunk, size_value, seg_first, seg_flag, slots, slot_off, frame_at,
                     nseg, parts, carry_out);
  const uint32_t waves = nseg < 65536u ? nseg : 65536u;
  hipLaunchKernelGGL(flush_crc_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, keys, key_off, key_len, chunks,
                     chunk_off, chunk_len, offset_chunk, size_value, seg_first, seg_flag, run_first, carry_in, slots,
                     slot_off, frame_at, big, nruns, parts, carry_out);
  return hipGetLastError();
}

}  // namespace kdb_lz4

// ------------------------------------------------------------------ C ABI
using namespace kdb_lz4;

extern "C" uint64_t kdb_flush_scratch_bytes(uint32_t nparts, uint32_t nseg, uint64_t raw_bytes) {
  return flush_scratch_bytes(nparts, nseg, raw_bytes);
}

extern "C" int kdb_flush_parts_batch(void* stream, const uint8_t* keys, const uint64_t* key_off,
                                     const uint32_t* key_len, const uint8_t* chunks, const uint64_t* chunk_off,
                                     const uint32_t* chunk_len, const uint64_t* offset_chunk,
                                     const uint64_t* size_value, const uint32_t* seg_first,
                                     const uint32_t* run_first, const kdb_flush_state* carry_in, uint32_t nparts,
                                     uint32_t nseg, uint32_t nruns, uint32_t max_chunk, uint8_t* scratch,
                                     uint64_t scratch_bytes, uint64_t raw_bytes, kdb_flush_part* parts,
                                     kdb_flush_state* carry_out, uint8_t* frames, uint64_t* frames_total) {
  if (!frames_total || (nparts && (!keys || !key_off || !key_len || !chunks || !chunk_off || !chunk_len ||
                                   !offset_chunk || !size_value || !seg_first || !run_first || !carry_in ||
                                   !scratch || !parts || !carry_out || !frames)) ||
      max_chunk > kMaxInput || (nparts && (nseg == 0 || nruns == 0)) || nseg > nparts || nruns > nseg)
    return KDB_LZ4_EINVAL;
  if (scratch_bytes < flush_scratch_bytes(nparts, nseg, raw_bytes)) return KDB_LZ4_EINVAL;
  const hipError_t e = launch_flush((hipStream_t)stream, keys, key_off, key_len, chunks, chunk_off, chunk_len,
                                    offset_chunk, size_value, seg_first, run_first, carry_in, nparts, nseg, nruns,
                                    max_chunk, scratch, raw_bytes, parts, carry_out, frames, frames_total);
  if (e == hipSuccess) return KDB_LZ4_OK;
  if (e == hipErrorNotSupported) return KDB_LZ4_EUNSUPPORTED;
  return (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? KDB_LZ4_ENODEV : KDB_LZ4_EHIP;
}
