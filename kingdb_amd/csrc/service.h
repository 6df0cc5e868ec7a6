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
// kernels (lz4_decompress.hip) and writes the bytes, the return code and the
// slot's done word back into host memory; the thread spins on the done word.
// No launch and no runtime call per request.
//
// Lifetime: the host launches the wave (on a stream of its own, so two
// instances never run at once) when it finds it gone (`alive` == 0).  The wave
// exits after kIdle of no requests, after kLife in all, or when the host sets
// `stop`; before leaving it clears `alive`, looks at the doorbells once more
// and stays if a request slipped in (the host rings, then reads `alive`; the
// wave clears `alive`, then reads the doorbells: one of them sees the other).
// A caller whose request is not served within a bound relaunches it.
#pragma once
#include <stdint.h>

namespace kdb_lz4 {

constexpr uint32_t kSvcSlots = 64;           // one per lane of the service wave
constexpr uint32_t kSvcMaxOut = 8192;        // the per-call zero-copy class (decode output)
constexpr uint32_t kSvcMaxIn = kSvcMaxOut + kSvcMaxOut / 255u + 24u;
constexpr uint32_t kSvcInBytes = (kSvcMaxIn + 64u + 15u) & ~15u;
constexpr uint32_t kSvcOutBytes = kSvcMaxOut + 64u;

struct SvcSlot {
  uint32_t csize, osize, target;   // LZ4_decompress_safe_partial's arguments
  int32_t ret;                     // its return value
  uint32_t pad[12];
  uint8_t in[kSvcInBytes];         // the block (16-byte aligned)
  uint8_t out[kSvcOutBytes];       // the decoded bytes
};

struct SvcBox {
  uint32_t req[kSvcSlots];         // host: a slot's request number (written last)
  uint32_t done[kSvcSlots];        // device: the request number served (written last)
  uint32_t alive;                  // host sets 1 before a launch; the wave clears it as it exits
  uint32_t stop;                   // host: exit now (process teardown)
  uint32_t launches, served;       // counters (diagnostics)
  uint32_t pad[60];
  SvcSlot slot[kSvcSlots];
};

}  // namespace kdb_lz4
