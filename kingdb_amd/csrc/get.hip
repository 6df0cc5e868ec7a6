// kingdb_amd/csrc/get.hip -- the read path around the codec on the GPU
// (read side): CompressorLZ4::UncompressByteArray
// (/root/reference/algorithm/compressor.cc:140-249) over Uncompress
// (compressor.cc:75-137) for a batch of stored values -- what Database::GetRaw
// (interface/database.cc:65-68) and MultipartReader (interface/multipart.h:65-154)
// do one value / one frame at a time.
//
//   get_walk_kernel     thread per value: walks the 8-byte frame headers
//                       (count pass, then fill pass after a scan): every frame
//                       Uncompress would decode, the disabled-compression
//                       header (8 zero bytes, compressor.h:141-149) and the raw
//                       tail after it, or the whole value when size_value_compressed
//                       is 0
//   frame decode        the LZ4 frame kernels over ALL frames of ALL values at
//                       once (lz4_decompress.hip, frame mode)
//   get_finish_kernel   wave per value: the first failing frame ends the value
//                       (IOError), frames that decoded short are slid into place,
//                       the raw tail is copied (one 1 MiB step, compressor.cc:236),
//                       and with verification the CRC32C of what the reference
//                       streams -- seeded with checksum_initial = crc32c(key)
//                       (storage/storage_engine.h:497-500) -- is compared with
//                       the entry's checksum, only where the reference compares
//                       it (a value that ends in frames, compressor.cc:159-169)
//
// verify = 1 reproduces the reference bug-for-bug: each frame is streamed into
// the CRC twice (Uncompress :126 and UncompressByteArray :202), so a value
// stored as frames reports "Invalid checksum." (SURVEY §0-7); verify = 2 streams
// each frame once (the corrected check).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/kdb_lz4.h"
#include "crc_device.h"
#include "lz4_device.h"

namespace kdb_lz4 {

hipError_t launch_decompress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* in_len, uint32_t n, uint32_t max_in, uint32_t max_out,
                             uint8_t* dst, const uint64_t* dst_off, const uint32_t* out_cap,
                             const uint32_t* target, uint32_t* out_len, int32_t* ret);
hipError_t launch_exclusive_scan(hipStream_t st, const uint32_t* len, uint32_t n, uint64_t* off, uint64_t* total);

namespace {

constexpr uint64_t kRawStep = 1048576u;     // compressor.cc:233

__device__ __forceinline__ uint32_t rd32g(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// End of a value's walk
// kEndCap: the value's frames did not fit the launch's frame capacity (its
// status is KDB_LZ4_VALUE_UNSUPPORTED, not an IOError: the bytes may be fine)
constexpr uint32_t kEndDone = 0, kEndTail = 1, kEndError = 2, kEndCap = 3;

struct ValueWalk {
  uint64_t tail_in, tail_out, tail_len;   // raw bytes copied after the frames
  uint32_t nframes;                       // frames found (decoded by the frame kernels)
  uint32_t end;                           // kEndDone / kEndTail / kEndError / kEndCap
};

// One walk; kFill writes the frame descriptors.
template <bool kFill>
__device__ ValueWalk walk(const uint8_t* s, uint64_t avail, uint64_t svc, uint64_t size, uint64_t base_in,
                          uint64_t out_base, uint64_t* f_off, uint32_t* f_avail, uint64_t* f_out, uint32_t* f_raw,
                          uint64_t frame_cap) {
  ValueWalk w{0, 0, 0, 0, kEndDone};
  uint64_t in = 0, o = 0;
  const bool compressed = svc != 0;
  bool disabled = false;
  if (compressed) {
    for (;;) {
      if (in == svc) { w.end = kEndDone; break; }                             // :159-169
      if (in > svc || in + 8u > avail) { w.end = kEndError; break; }
      const uint32_t st = rd32g(s + in), raw = rd32g(s + in + 4);
      if (st == 0 && raw == 0) { disabled = true; in += 8u; break; }         // :171-178
      if (o + raw > size) { w.end = kEndError; break; }
      uint64_t fsz;
      if (st > 0) {
        const uint32_t csz = st - 8u;
        // a negative block size fails in the frame kernel (IOError, as in the reference)
        fsz = (int32_t)csz < 0 ? 8u : (uint64_t)csz + 8u;
        if (fsz > avail - in) { w.end = kEndError; break; }
      } else {
        fsz = (uint64_t)raw + 8u;
        if (fsz > avail - in) { w.end = kEndError; break; }
      }
      if (kFill) {
        if (w.nframes >= frame_cap) { w.end = kEndCap; break; }
        f_off[w.nframes] = base_in + in;
        f_avail[w.nframes] = (uint32_t)min(avail - in, (uint64_t)0xFFFFFFFFu);
        f_out[w.nframes] = out_base + o;
        f_raw[w.nframes] = raw;
      }
      w.nframes++;
      o += raw;
      in += fsz;
    }
  }
  if (!compressed || disabled) {                                              // :224-247
    const uint64_t left = compressed ? svc : size;
    w.end = kEndTail;
    if (in > left) {
      w.end = kEndError;
    } else {
      const uint64_t cur = min(left - in, kRawStep);
      if (in + cur > avail || o + cur > size) w.end = kEndError;
      w.tail_in = in;
      w.tail_out = o;
      w.tail_len = cur;
    }
  }
  return w;
}

__global__ void get_count_kernel(const uint8_t* __restrict__ stored, const uint64_t* __restrict__ stored_off,
                                 const uint64_t* __restrict__ avail, const uint64_t* __restrict__ svc,
                                 const uint64_t* __restrict__ size, uint32_t n, uint32_t* __restrict__ nframes) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const ValueWalk w = walk<false>(stored + stored_off[v], avail[v], svc[v], size[v], 0, 0, nullptr, nullptr,
                                    nullptr, nullptr, 0);
    nframes[v] = w.nframes;
  }
}

__global__ void get_fill_kernel(const uint8_t* __restrict__ stored, const uint64_t* __restrict__ stored_off,
                                const uint64_t* __restrict__ avail, const uint64_t* __restrict__ svc,
                                const uint64_t* __restrict__ size, const uint64_t* __restrict__ out_off, uint32_t n,
                                const uint64_t* __restrict__ frame_first, uint64_t frame_cap,
                                uint64_t* __restrict__ f_off, uint32_t* __restrict__ f_avail,
                                uint64_t* __restrict__ f_out, uint32_t* __restrict__ f_raw,
                                ValueWalk* __restrict__ walks) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const uint64_t f0 = frame_first[v];
    const uint64_t cap = f0 < frame_cap ? frame_cap - f0 : 0u;
    walks[v] = walk<true>(stored + stored_off[v], avail[v], svc[v], size[v], stored_off[v], out_off[v], f_off + f0,
                          f_avail + f0, f_out + f0, f_raw + f0, cap);
  }
}

// The CRC's message: every frame of the value, each `reps` times in a row.
struct FrameMsg {
  const uint8_t* s;        // the value's stored bytes
  const uint64_t* f_off;   // absolute frame offsets (minus base = offset in the value)
  uint64_t base;
  uint32_t nf, reps;
  uint64_t svc;
  __device__ uint32_t feed(uint64_t a, uint64_t b, uint32_t c, const uint32_t* s_t) const {
    if (reps == 1) {
      for (uint64_t m = a; m < b; m++) c = crc::step(c, s[m], s_t);
      return c;
    }
    // frames are contiguous over [0, svc): frame k is [fo_k, fo_{k+1}), seen twice
    uint32_t k = 0;
    uint64_t mbase = 0;      // message position where frame k's first copy starts
    auto flen = [&](uint32_t i) { return (i + 1 < nf ? f_off[i + 1] - base : svc) - (f_off[i] - base); };
    while (k < nf && a >= mbase + 2u * flen(k)) { mbase += 2u * flen(k); k++; }
    for (uint64_t m = a; m < b; m++) {
      while (k < nf && m >= mbase + 2u * flen(k)) { mbase += 2u * flen(k); k++; }
      const uint64_t L = flen(k);
      const uint64_t r = m - mbase;
      c = crc::step(c, s[(f_off[k] - base) + (r < L ? r : r - L)], s_t);
    }
    return c;
  }
};

constexpr int kFinishBlock = 256;

__global__ __launch_bounds__(kFinishBlock) void get_finish_kernel(
    const uint8_t* __restrict__ stored, const uint64_t* __restrict__ stored_off, const uint64_t* __restrict__ svc,
    uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, uint32_t n,
    const uint64_t* __restrict__ frame_first, uint64_t frame_cap, const uint64_t* __restrict__ f_off,
    const uint64_t* __restrict__ f_out, const uint32_t* __restrict__ f_raw, const uint32_t* __restrict__ f_len,
    const int32_t* __restrict__ f_status, const ValueWalk* __restrict__ walks, int verify,
    const uint32_t* __restrict__ checksum, const uint32_t* __restrict__ checksum_initial,
    uint64_t* __restrict__ out_len, int32_t* __restrict__ status) {
  __shared__ uint32_t s_t[256];
  crc::stage_table(s_t);
  __syncthreads();
  const uint32_t lane = lane_id();
  const uint32_t nw = gridDim.x * (kFinishBlock / 64);
  // 64 values per wave at a time, a lane each (round 6): a value whose status
  // and length follow from its walk and its one frame's status -- no slide, no
  // raw tail, no checksum -- is finished by its lane; the wave then takes the
  // others one by one (below).  One value per wave had every wave wait two
  // dependent metadata round trips per value: 354 us per 1 Mi values.
  for (uint32_t c0 = (blockIdx.x * (kFinishBlock / 64) + threadIdx.x / 64u) * 64u; c0 < n; c0 += nw * 64u) {
    bool other = false;
    {
      const uint32_t v = c0 + lane;
      if (v < n) {
        const ValueWalk w = walks[v];
        const uint64_t f0 = frame_first[v];
        int32_t st = 0;
        uint64_t defined = 0;
        bool done = true;
        if (w.end == kEndCap || f0 + w.nframes > frame_cap) {
          st = KDB_LZ4_VALUE_UNSUPPORTED;
        } else if (w.nframes > 1u) {
          done = false;
        } else {
          bool failed = false;
          if (w.nframes == 1u) {
            if (f_status[f0] != 0) {
              failed = true;
            } else if (f_out[f0] != out_off[v]) {
              done = false;                 // a slide: the wave's path
            } else {
              defined = f_len[f0];
            }
          }
          if (failed || w.end == kEndError) st = -1;
          else if (w.end == kEndTail) done = w.tail_len == 0;
          else if (verify) done = false;     // kEndDone with the checksum: the wave's CRC
        }
        if (done) {
          status[v] = st;
          out_len[v] = defined;
        }
        other = !done;
      }
    }
    uint64_t todo = ballot(other);
#pragma unroll 1
    while (todo) {
      const uint32_t v = c0 + (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1ull;
      const ValueWalk w = walks[v];
      const uint64_t f0 = frame_first[v];
      const uint8_t* s = stored + stored_off[v];
      uint8_t* o = out + out_off[v];
      int32_t st = 0;
      uint64_t defined = 0;
      if (w.end == kEndCap || f0 + w.nframes > frame_cap) {
        st = KDB_LZ4_VALUE_UNSUPPORTED;   // more frames than the launch's frame capacity
      } else {
        // frames in order: the first failure ends the value; a frame that decoded
        // fewer bytes than its header announced moves the later ones down
        bool failed = false;
        for (uint32_t k = 0; k < w.nframes; k++) {
          const uint64_t f = f0 + k;
          if (f_status[f] != 0) { failed = true; break; }
          const uint64_t at = f_out[f] - out_off[v];
          const uint32_t got = f_len[f];
          if (at != defined) {           // slide down (front to back: never overlaps wrongly)
            for (uint64_t j = 0; j < got; j += 64u) {
              const uint64_t i = j + lane;
              const uint8_t b = i < got ? o[at + i] : (uint8_t)0;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              if (i < got) o[defined + i] = b;
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
          }
          defined += got;
        }
        if (failed) {
          st = -1;
        } else if (w.end == kEndError) {
          st = -1;
        } else if (w.end == kEndTail) {
          const uint64_t to = defined;          // == walk's tail_out unless a frame decoded short
          for (uint64_t i = lane; i < w.tail_len; i += 64u) o[to + i] = s[w.tail_in + i];
          defined += w.tail_len;
        } else if (verify) {                    // kEndDone: the reference compares the CRC
          const FrameMsg msg{s, f_off + f0, stored_off[v], w.nframes, verify == 1 ? 2u : 1u, svc[v]};
          const uint64_t mlen = (verify == 1 ? 2u : 1u) * svc[v];
          const uint32_t c = crc::extend_wave(checksum_initial[v], mlen, msg, s_t);
          if (c != checksum[v]) st = -2;
        }
      }
      if (lane == 0) {
        status[v] = st;
        out_len[v] = defined;
      }
    }
  }
}

}  // namespace

uint64_t get_scratch_bytes(uint32_t n, uint64_t frame_cap) {
  return (uint64_t)n * (4 + 8 + sizeof(ValueWalk)) + frame_cap * (8 + 4 + 8 + 4 + 4 + 4) + 16u * 256u;
}

hipError_t launch_get_values(hipStream_t st, const uint8_t* stored, const uint64_t* stored_off,
                             const uint64_t* avail, const uint64_t* svc, const uint64_t* size, uint32_t n,
                             uint8_t* out, const uint64_t* out_off, int verify, const uint32_t* checksum,
                             const uint32_t* checksum_initial, uint64_t frame_cap, uint32_t max_frame_in,
                             uint32_t max_frame_out, uint8_t* scratch, uint64_t* out_len, int32_t* status) {
  uint8_t* p = scratch;
  auto take = [&](uint64_t bytes) {
    uint8_t* r = p;
    p += (bytes + 255u) & ~255ull;
    return r;
  };
  uint32_t* nframes = reinterpret_cast<uint32_t*>(take((uint64_t)n * 4));
  uint64_t* frame_first = reinterpret_cast<uint64_t*>(take((uint64_t)n * 8));
  ValueWalk* walks = reinterpret_cast<ValueWalk*>(take((uint64_t)n * sizeof(ValueWalk)));
  uint64_t* f_off = reinterpret_cast<uint64_t*>(take(frame_cap * 8));
  uint32_t* f_avail = reinterpret_cast<uint32_t*>(take(frame_cap * 4));
  uint64_t* f_out = reinterpret_cast<uint64_t*>(take(frame_cap * 8));
  uint32_t* f_raw = reinterpret_cast<uint32_t*>(take(frame_cap * 4));
  uint32_t* f_len = reinterpret_cast<uint32_t*>(take(frame_cap * 4));
  int32_t* f_status = reinterpret_cast<int32_t*>(take(frame_cap * 4));
  uint64_t* total = reinterpret_cast<uint64_t*>(take(8));
  if (n == 0) return hipSuccess;
  const uint32_t tb = 256, tg = (n + tb - 1) / tb < 4096u ? (n + tb - 1) / tb : 4096u;
  hipLaunchKernelGGL(get_count_kernel, dim3(tg), dim3(tb), 0, st, stored, stored_off, avail, svc, size, n, nframes);
  {
    const hipError_t e = launch_exclusive_scan(st, nframes, n, frame_first, total);
    if (e != hipSuccess) return e;
  }
  // The frame count is only known on the device, so the decode launch covers
  // the whole capacity; slots the walk leaves empty stay inert: offset 0 (the
  // first stored bytes, always readable), 0 bytes available and 0 output bytes
  // -- the frame kernel returns IOError for them without writing (ignored).
  hipError_t e = hipMemsetAsync(f_off, 0, frame_cap * 8, st);
  if (e == hipSuccess) e = hipMemsetAsync(f_avail, 0, frame_cap * 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(f_raw, 0, frame_cap * 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(get_fill_kernel, dim3(tg), dim3(tb), 0, st, stored, stored_off, avail, svc, size, out_off, n,
                     frame_first, frame_cap, f_off, f_avail, f_out, f_raw, walks);
  e = launch_decompress(true, st, stored, f_off, f_avail, (uint32_t)frame_cap, max_frame_in, max_frame_out, out,
                        f_out, f_raw, nullptr, f_len, f_status);
  if (e != hipSuccess) return e;
  const uint32_t fg = (n + 255) / 256 < 4096u ? (n + 255) / 256 : 4096u;   // 64 values per wave per pass
  hipLaunchKernelGGL(get_finish_kernel, dim3(fg), dim3(kFinishBlock), 0, st, stored, stored_off, svc, out, out_off, n,
                     frame_first, frame_cap, f_off, f_out, f_raw, f_len, f_status, walks, verify, checksum,
                     checksum_initial, out_len, status);
  return hipGetLastError();
}

}  // namespace kdb_lz4

using namespace kdb_lz4;

extern "C" uint64_t kdb_get_scratch_bytes(uint32_t n, uint64_t frame_cap) {
  return get_scratch_bytes(n, frame_cap);
}

extern "C" int kdb_get_values_batch(void* stream, const uint8_t* stored, const uint64_t* stored_off,
                                    const uint64_t* avail, const uint64_t* svc, const uint64_t* size, uint32_t n,
                                    uint8_t* out, const uint64_t* out_off, int verify, const uint32_t* checksum,
                                    const uint32_t* checksum_initial, uint64_t frame_cap, uint32_t max_frame_in,
                                    uint32_t max_frame_out, uint8_t* scratch, uint64_t scratch_bytes,
                                    uint64_t* out_len, int32_t* status) {
  if (verify < 0 || verify > 2 || frame_cap > 0xFFFFFFFFull || scratch_bytes < get_scratch_bytes(n, frame_cap) ||
      (n && (!stored || !stored_off || !avail || !svc || !size || !out || !out_off || !scratch || !out_len ||
             !status || (verify && (!checksum || !checksum_initial)))))
    return KDB_LZ4_EINVAL;
  const hipError_t e = launch_get_values((hipStream_t)stream, stored, stored_off, avail, svc, size, n, out, out_off,
                                         verify, checksum, checksum_initial, frame_cap, max_frame_in, max_frame_out,
                                         scratch, out_len, status);
  if (e == hipSuccess) return KDB_LZ4_OK;
  return (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? KDB_LZ4_ENODEV : KDB_LZ4_EHIP;
}
