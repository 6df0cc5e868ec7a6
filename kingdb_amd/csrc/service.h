// kingdb_amd/csrc/service.h -- the resident decode service of the per-call
// path (kdb_lz4_decompress_safe_partial, i.e. CompressorLZ4::Uncompress and
// UncompressByteArray one frame at a time: /root/reference/algorithm/lz4.cc:
// 1050-1053, compressor.cc:75-137).
//
// A launch + a stream sync per call cost ~16 us, almost
// all of it the launch path, not the decode.  The service is one wave that
// stays resident on the device while calls keep coming: a calling thread
// writes its block into a slot of a pinned, coherent, device-mapped mailbox
// and rings the slot's doorbell; the wave, polling the 64 doorbells with one
// 256-byte read, decodes the block with the same decode_block as the batch
// kernels (lz4_decompress.hip; lz4_compress.hip has the compress twin) and
// writes the bytes and then the slot's done word (request and return code in
// one store) back into host memory; the thread spins on the done word.  No
// launch and no runtime call per request.
//
// Lifetime: the host launches the wave (on a stream of its own, so two
// instances never run at once) when it finds it gone (`alive` == 0).  The wave
// exits after KDB_LZ4_SERVICE_IDLE_US (2 ms) without a request, after 20 ms in
// all, or when the host sets `stop`; before leaving it clears `alive`, looks at the doorbells once more
// and stays if a request slipped in (the host rings, then reads `alive`; the
// wave clears `alive`, then reads the doorbells: one of them sees the other).
// A caller whose request is not served within a bound relaunches it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kdb_lz4 {

constexpr uint32_t kSvcSlots = 64;           // one per lane of the service wave
constexpr uint32_t kSvcMaxOut = 8192;        // the per-call zero-copy class (decode output)
constexpr uint32_t kSvcMaxIn = kSvcMaxOut + kSvcMaxOut / 255u + 24u;
constexpr uint32_t kSvcInBytes = (kSvcMaxIn + 64u + 15u) & ~15u;
constexpr uint32_t kSvcOutBytes = kSvcMaxOut + 64u;

// A request's arguments, in a row of their own (read with the block, right
// after the doorbell): LZ4_decompress_safe_partial's (csize, osize, target)
// or LZ4_compress_limitedOutput's (input bytes, output capacity).
struct SvcArgs {
  uint32_t csize, osize, target, pad;
};

struct SvcSlot {
  uint8_t in[kSvcInBytes];         // the block / value (16-byte aligned)
  uint8_t out[kSvcOutBytes];       // the result bytes
};

// Per request, three PCIe round trips on the wave's side: the doorbells (one
// 256-byte read per poll), then the slot's arguments and the first KiB of its
// input together (the rest, if any, one more), then the result bytes and one
// 64-bit release store of (request << 32 | return value) into its done word.
struct SvcBox {
  uint32_t req[kSvcSlots];         // host: a slot's request number (written last)
  uint64_t done[kSvcSlots];        // device: (request served << 32) | return value (written last)
  SvcArgs args[kSvcSlots];         // host: the arguments of the slot's request
  uint32_t alive;                  // host sets 1 before a launch; the wave clears it as it exits
  uint32_t stop;                   // host: exit now (process teardown)
  uint32_t launches, served;       // counters (diagnostics)
  uint32_t pad[60];
  SvcSlot slot[kSvcSlots];
};

// The wave's side of a request: the slot's arguments and its input (up to
// max_in bytes) staged into LDS at `lds` (16-byte aligned; input byte i at
// lds[i]).  The arguments and the first KiB go out together, one round trip;
// the rest, if any, all in flight at once, one more.  Called right after the
// doorbell's system-scope acquire load, which orders these reads after the
// host's writes.
__device__ __forceinline__ SvcArgs svc_fetch(SvcBox* box, uint32_t sidx, uint8_t* lds, uint32_t max_in) {
  const uint32_t lane = __lane_id();
  SvcArgs* ap = &box->args[sidx];
  const uint32_t cs = __hip_atomic_load(&ap->csize, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint32_t os = __hip_atomic_load(&ap->osize, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint32_t tg = __hip_atomic_load(&ap->target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint4* in4 = reinterpret_cast<const uint4*>(box->slot[sidx].in);
  const uint4 c0 = in4[lane];
  SvcArgs a;
  a.csize = (uint32_t)__builtin_amdgcn_readfirstlane((int)cs);
  a.osize = (uint32_t)__builtin_amdgcn_readfirstlane((int)os);
  a.target = (uint32_t)__builtin_amdgcn_readfirstlane((int)tg);
  a.pad = 0;
  const uint32_t n = a.csize < max_in ? a.csize : max_in;
  const uint32_t chunks = (n + 15u) >> 4;
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  if (lane < chunks) l4[lane] = c0;
  constexpr uint32_t kMore = (kSvcInBytes / 16u + 63u) / 64u - 1u;
  if (chunks > 64u) {
    uint4 r[kMore];
#pragma unroll
    for (uint32_t k = 0; k < kMore; k++)
      if (lane + 64u * (k + 1u) < chunks) r[k] = in4[lane + 64u * (k + 1u)];
#pragma unroll
    for (uint32_t k = 0; k < kMore; k++)
      if (lane + 64u * (k + 1u) < chunks) l4[lane + 64u * (k + 1u)] = r[k];
  }
  return a;
}

}  // namespace kdb_lz4
