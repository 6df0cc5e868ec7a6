// kingdb_amd/csrc/service.h -- the resident services of the per-call path:
// per-call decodes (kdb_lz4_decompress_safe_partial, i.e.
// CompressorLZ4::Uncompress and UncompressByteArray one frame at a time:
// /root/reference/algorithm/lz4.cc:1050-1053, compressor.cc:75-137) and
// per-call compressions (kdb_lz4_compress_limitedOutput, lz4.cc:664-682).
//
// A launch + a stream sync per call cost ~16 us, almost
// all of it the launch path, not the codec.  A service is one wave that stays
// resident on the device while calls keep coming: a calling thread writes its
// request into a slot of a pinned, coherent, device-mapped mailbox and rings
// the slot's doorbell; the wave, polling the 64 doorbells, runs the request
// with the same device code as the batch kernels (lz4_decompress.hip's
// decode_block, lz4_compress.hip's compress_block) and writes the bytes and
// then the slot's done word (request and return code in one store) back into
// host memory; the thread spins on the done word.  No launch and no runtime
// call per request.
//
// Per request the wave reads host memory over PCIe, so what a request waits
// for is PCIe round trips (round 5):
//  * each poll (relaxed system-scope loads, which bypass the caches) also reads the first kSvcPostSlots slots' POSTS: a 128-byte
//    record per slot holding the request's arguments and, for inputs up to
//    kSvcPostInline bytes (a 100-byte value, or its ~60-byte block), the input
//    itself.  The host writes the post, then its two tags (one per 64-byte
//    line: tag1 at the end of line 1, then tag0 at the start of line 0), then
//    the doorbell.  A 64-byte line is read as one unit, so a line whose tag
//    is the request's number holds that request's bytes; with both tags equal
//    to the doorbell the wave takes the request straight from the poll -- no
//    second round trip for its arguments and input.  Otherwise (larger
//    inputs, slots past kSvcPostSlots, a post read before it was complete)
//    the wave fetches them after an acquire fence, as before.
//
// Two mailboxes (round 5): an INBOX the host writes (doorbells, arguments,
// posts, inputs, stop, active, the A/B knobs) and an OUTBOX the wave writes
// (done words, replies, results, alive, counters).  The outbox is pinned host
// memory: the host spins on it locally.  The inbox is fine-grained device
// memory the host writes through the large BAR when the device has one
// (write-combining: the host fences before each doorbell), so the wave's polls
// and its input reads stay in its own HBM instead of crossing PCIe: a ping
// with 112 / 2 400 / 8 192 input bytes took 2.41 / 3.03 / 4.82 us against
// 3.71 / 6.23 / 12.31 us with the inbox in host memory, and no torn input in
// 30 000 rounds (tools/probe/bar_probe.hip).  Without a large BAR both are the
// same host-memory box.  Both have the SvcBox layout; each side touches only
// its own fields of each.
//
// Lifetime: the host launches an instance (on a stream of its own, so two
// instances never run at once) when it finds `alive` == 0, and stores the
// instance's generation in `alive` first.  The wave exits after
// KDB_LZ4_SERVICE_IDLE_US (2 ms) without a request, after 20 ms in all, or
// when the host sets `stop`; before leaving it clears `alive` -- only if it
// still holds its own generation, so an old instance never clears the flag
// of the one queued behind it -- then looks at the doorbells once more and
// stays if a request slipped in (the host rings, then reads `alive`; the wave
// clears `alive`, then reads the doorbells: one of them sees the other).
// A caller whose request is not served within a bound relaunches it.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lz4_device.h"

namespace kdb_lz4 {

constexpr uint32_t kSvcSlots = 64;           // one per lane of the service wave
constexpr uint32_t kSvcMaxOut = 8192;        // the per-call zero-copy class (decode output)
constexpr uint32_t kSvcMaxIn = kSvcMaxOut + kSvcMaxOut / 255u + 24u;
constexpr uint32_t kSvcInBytes = (kSvcMaxIn + 64u + 15u) & ~15u;
constexpr uint32_t kSvcOutBytes = kSvcMaxOut + 64u;
constexpr uint32_t kSvcPostSlots = 16;       // slots whose posts every poll reads (2 KiB)

constexpr uint32_t kSvcInline = 108;         // result bytes a reply carries
constexpr uint32_t kSvcPostInline = 104;     // input bytes a post carries

// A request's arguments: LZ4_decompress_safe_partial's (csize, osize, target)
// or LZ4_compress_limitedOutput's (input bytes, output capacity).
struct SvcArgs {
  uint32_t csize, osize, target, pad;
};

// A slot's post (slots < kSvcPostSlots): line 0 = tag0, the arguments and
// input bytes [0, 48); line 1 = input bytes [48, 104), a checksum of dwords
// 1-29 (the arguments and the input: svc_weight) and tag1.  The tags say
// which request the lines belong to; the checksum guards against a line the
// wave read in pieces across the host's write (measured: a post taken on
// tags alone decoded wrong bytes once in some 10^4 calls).
struct SvcPost {
  uint32_t tag0;
  uint32_t csize, osize, target;
  uint8_t data[kSvcPostInline];
  uint32_t sum;
  uint32_t tag1;
};
static_assert(sizeof(SvcPost) == 128, "two 64-byte lines");

// A slot's reply (decode service, slots < kSvcPostSlots, results up to
// kSvcInline bytes): line 0 = tag0, the return value, a checksum of the 108
// data bytes, then data[0, 48); line 1 = data[48, 108) and tag1.  Written by
// one store instruction (8 lanes x 16 bytes), with no release: the host takes
// the result from it when both tags are the request's number and the
// checksum matches (svc_weight, kdb_lz4_capi.hip), which spares the
// wait for the result's write to be acknowledged before the done word; the
// done word (relaxed) only says kSvcReplied, and a host that reads a reply
// whose bytes are not all there yet reads it again.
struct SvcReply {
  uint32_t tag0;
  int32_t rc;
  uint32_t sum, pad;
  uint8_t data[kSvcInline];
  uint32_t tag1;
};
static_assert(sizeof(SvcReply) == 128, "two 64-byte lines");
// Whether slot sidx's result of return value rc goes back in a reply (the
// serve callback then leaves slot.out unwritten); its done word then holds
// kSvcReplied | rc, a value no return code takes (results are < 2^30; error
// codes are negative).
constexpr uint32_t kSvcReplied = 0x40000000u;
__host__ __device__ inline bool svc_replies(uint32_t sidx, int rc) {
  return sidx < kSvcPostSlots && rc >= 0 && rc <= (int)kSvcInline;
}
// the checksums: the sum of dword i x (2 i + 1) x 0x9E3779B1 (mod 2^32) over
// a record's dwords: any one dword that differs changes it (odd factors)
__host__ __device__ inline uint32_t svc_weight(uint32_t i) { return (2u * i + 1u) * 0x9E3779B1u; }
__host__ inline uint32_t svc_sum_host(const uint32_t* w, uint32_t first, uint32_t n) {
  uint32_t s = 0;
  for (uint32_t i = first; i < first + n; i++) s += w[i] * svc_weight(i);
  return s;
}

struct SvcSlot {
  uint8_t in[kSvcInBytes];         // the block / value (16-byte aligned), when not in the post
  uint8_t out[kSvcOutBytes];       // the result bytes
};

struct SvcBox {
  uint32_t req[kSvcSlots];         // host (inbox): a slot's request number (written last); outbox: the host's copy
  uint64_t done[kSvcSlots];        // device: (request served << 32) | return value (written last)
  SvcArgs args[kSvcSlots];         // host: the arguments of slots >= kSvcPostSlots
  uint32_t alive;                  // host: the generation it launched last (0: none); the wave clears its own
  uint32_t stop;                   // host: exit now (process teardown)
  uint32_t launches, served;       // counters (diagnostics)
  uint32_t active;                 // host: 1 + the highest slot leased (how many posts a poll reads)
  uint32_t gen;                    // host: the last generation launched
  uint32_t polls, inline_served;   // device: counters (diagnostics)
  uint32_t replied;                // device: requests answered by a reply (diagnostics)
  uint32_t no_post, no_reply;      // host: the wave ignores the posts / never replies (A/B knobs)
  uint32_t no_pipe;                // host: one poll in flight instead of two (A/B knob)
  uint32_t pad[52];
  SvcPost post[kSvcPostSlots];     // 128-byte aligned (offset 2048)
  SvcReply reply[kSvcPostSlots];
  SvcSlot slot[kSvcSlots];
};
static_assert(offsetof(SvcBox, post) % 128 == 0 && offsetof(SvcBox, slot) % 16 == 0, "mailbox layout");

__device__ __forceinline__ uint32_t svc_relaxed(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Everything this wave wrote before, out to memory: the release fence's L2
// write-back (buffer_wbl2), then a wait for it written out here.  The
// compiler's own wait after the write-back is dropped by its waitcnt pass
// when no load or store is outstanding (it does not count the write-back),
// and a store that followed then reached the host ahead of the bytes written
// before it (tests/test_service_isa.py checks every write-back is waited for).
__device__ __forceinline__ void svc_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) (expcnt, lgkmcnt: no wait)
}
// A store the host reads, after every earlier write of this wave.
__device__ __forceinline__ void svc_store(uint32_t* p, uint32_t v) {
  svc_release();
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef uint32_t svc_u32x4 __attribute__((ext_vector_type(4)));

// One poll: the 64 doorbells (lane l: slot l's), the host's `active`, and the
// posts of the first 8 / 16 slots (lane l: bytes [16 l, 16 l + 16) of the
// posts of slots 0-7, resp. 8-15).  Every load is relaxed at system scope
// (sc0 sc1: past the caches).
struct SvcPoll {
  uint32_t r, act, stop;
  svc_u32x4 p0, p1;
};
__device__ __forceinline__ SvcPoll svc_poll(const SvcBox* box, uint32_t act) {
  const uint32_t lane = lane_id();
  SvcPoll q;
  q.r = svc_relaxed(&box->req[lane]);
  q.act = svc_relaxed(&box->active);
  q.stop = svc_relaxed(&box->stop);
  // the same five loads every poll (so the wait for the older poll is a
  // static count); posts past the leased slots lie past the buffer's range
  // and read as 0 without touching memory.  Cache policy 17 = sc0 | sc1
  // (system scope) on gfx950.
  const __amdgpu_buffer_rsrc_t posts = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<SvcPost*>(box->post), 0, (int)(128u * (act < kSvcPostSlots ? act : kSvcPostSlots)), 0x00020000);
  q.p0 = __builtin_amdgcn_raw_buffer_load_b128(posts, (int)(16u * lane), 0, 17);
  q.p1 = __builtin_amdgcn_raw_buffer_load_b128(posts, (int)(16u * lane + 1024u), 0, 17);
  return q;
}

// The wave's side of a request whose post was not usable: its arguments and
// input (up to max_in bytes) staged into LDS at `lds` (16-byte aligned; input
// byte i at lds[i]).  The post (or the arguments row) and the first KiB of
// the slot's input go out together, one round trip; the rest, if any, all in
// flight at once, one more.  Called after an acquire fence that follows the
// doorbell's load, which orders these reads after the host's writes.
__device__ __forceinline__ SvcArgs svc_fetch(const SvcBox* box, uint32_t sidx, uint8_t* lds, uint32_t max_in) {
  const uint32_t lane = lane_id();
  const bool posted = sidx < kSvcPostSlots;
  const uint32_t* ap = posted ? &box->post[sidx].csize : &box->args[sidx].csize;
  const uint32_t cs = svc_relaxed(ap), os = svc_relaxed(ap + 1), tg = svc_relaxed(ap + 2);
  const uint4* in4 = reinterpret_cast<const uint4*>(box->slot[sidx].in);
  const uint4* pin4 = reinterpret_cast<const uint4*>(posted ? box->post[sidx].data : box->slot[sidx].in);
  const uint4 c0 = in4[lane];
  const uint4 pc = lane < 7u ? pin4[lane] : make_uint4(0, 0, 0, 0);   // a post's input: 112 bytes from data
  SvcArgs a;
  a.csize = (uint32_t)__builtin_amdgcn_readfirstlane((int)cs);
  a.osize = (uint32_t)__builtin_amdgcn_readfirstlane((int)os);
  a.target = (uint32_t)__builtin_amdgcn_readfirstlane((int)tg);
  a.pad = 0;
  const uint32_t n = a.csize < max_in ? a.csize : max_in;
  const uint32_t chunks = (n + 15u) >> 4;
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  if (posted && a.csize <= kSvcPostInline) {     // the input is in the post
    if (lane < chunks) l4[lane] = pc;
    return a;
  }
  if (lane < chunks) l4[lane] = c0;
  constexpr uint32_t kMore = (kSvcInBytes / 16u + 63u) / 64u - 1u;
  if (chunks > 64u) {
    // every load unconditional (indices clamped to the last chunk, inside the
    // slot): with per-lane conditions around them the compiler kept the array
    // in scratch memory, a round trip per chunk (ScratchSize 160 per lane)
    uint4 r[kMore];
#pragma unroll
    for (uint32_t k = 0; k < kMore; k++) r[k] = in4[min(lane + 64u * (k + 1u), chunks - 1u)];
#pragma unroll
    for (uint32_t k = 0; k < kMore; k++)
      if (lane + 64u * (k + 1u) < chunks) l4[lane + 64u * (k + 1u)] = r[k];
  }
  return a;
}

// A request's input (csize bytes, known from its post) staged from the slot
// into LDS: every chunk in flight at once, one round trip.  After an acquire
// fence, as svc_fetch.
__device__ __forceinline__ void svc_fetch_input(const SvcBox* box, uint32_t sidx, uint8_t* lds, uint32_t csize,
                                                uint32_t max_in) {
  const uint32_t lane = lane_id();
  const uint32_t n = csize < max_in ? csize : max_in;
  const uint32_t chunks = (n + 15u) >> 4;
  const uint4* in4 = reinterpret_cast<const uint4*>(box->slot[sidx].in);
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  constexpr uint32_t kAll = (kSvcInBytes / 16u + 63u) / 64u;
  if (chunks == 0u) return;
  uint4 r[kAll];   // (unconditional loads, clamped: see svc_fetch)
#pragma unroll
  for (uint32_t k = 0; k < kAll; k++) r[k] = in4[min(lane + 64u * k, chunks - 1u)];
#pragma unroll
  for (uint32_t k = 0; k < kAll; k++)
    if (lane + 64u * k < chunks) l4[lane + 64u * k] = r[k];
}

// The request of slot sidx (doorbell `want`) taken from poll q when its post
// is complete: the arguments, and the input staged at lds[0, csize).  Returns
// 0 when the post is not usable (then svc_fetch), 1 when the request is
// complete, 2 when only the arguments are (its input is in the slot: then
// svc_fetch_input).
// The checksum's weight of dword 4 (lane & 7) + c of the post whose first lane
// is lane & ~7 (0 for the dwords it does not cover: 0 = tag0, 30 = the sum,
// 31 = tag1): per lane, computed once per wave.
__device__ __forceinline__ svc_u32x4 svc_post_weights(uint32_t lane) {
  svc_u32x4 w;
  const uint32_t d = 4u * (lane & 7u);
  w.x = d >= 1u ? svc_weight(d) : 0u;
  w.y = svc_weight(d + 1u);
  w.z = d + 2u <= 29u ? svc_weight(d + 2u) : 0u;
  w.w = d + 3u <= 29u ? svc_weight(d + 3u) : 0u;
  return w;
}
// The sum over each aligned group of 8 lanes, in every lane of the group (DPP:
// pairs, quads, then the two quads of each half row).
__device__ __forceinline__ uint32_t svc_sum8(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);   // row_half_mirror
  return v;
}

__device__ __forceinline__ int svc_from_post(const SvcPoll& q, uint32_t sidx, uint32_t want, uint8_t* lds,
                                              SvcArgs* a, const svc_u32x4& pw) {
  if (sidx >= kSvcPostSlots) return 0;
  const uint32_t lane = lane_id();
  const uint32_t b = 8u * (sidx & 7u);           // the post's first lane
  const bool hi = sidx >= 8u;
  const uint32_t x = hi ? q.p1.x : q.p0.x, y = hi ? q.p1.y : q.p0.y, z = hi ? q.p1.z : q.p0.z,
                 w = hi ? q.p1.w : q.p0.w;
  const uint32_t tag0 = readlane(x, b), tag1 = readlane(w, b + 7u);
  if (tag0 != want || tag1 != want) return 0;
  // the checksum over dwords 1-29 (dword d = 4 (lane - b) + component): each
  // lane's share, summed over the post's 8 lanes (the other groups sum other
  // posts, unused here)
  const uint32_t sum = svc_sum8(x * pw.x + y * pw.y + z * pw.z + w * pw.w);
  if (readlane(sum, b) != readlane(z, b + 7u)) return 0;
  a->csize = readlane(y, b);
  a->osize = readlane(z, b);
  a->target = readlane(w, b);
  a->pad = 0;
  if (a->csize > kSvcPostInline) return 2;        // the input is in the slot: fetch it
  // lanes b+1 .. b+7 hold post bytes [16, 128): input bytes [0, 112)
  if (lane > b && lane < b + 8u) reinterpret_cast<uint4*>(lds)[lane - b - 1u] = make_uint4(x, y, z, w);
  return 1;
}

// (svc_replies) Writes slot sidx's reply (request `want`, return value rc, result bytes at
// LDS `res`, 16-byte aligned, readable for 112 bytes).
__device__ __forceinline__ void svc_write_reply(SvcBox* box, uint32_t sidx, uint32_t want, int rc,
                                                const uint8_t* res) {
  const uint32_t lane = lane_id();
  // lane j (0..7) holds reply bytes [16 j, 16 j + 16); data dword i sits at
  // reply byte 16 + 4 i
  svc_u32x4 d = {0u, 0u, 0u, 0u};
  if (lane >= 1u && lane < 8u) {
    const uint4 x = reinterpret_cast<const uint4*>(res)[lane - 1u];
    d = svc_u32x4{x.x, x.y, x.z, x.w};
  }
  // the checksum: lane j's share (data dwords 4 (j - 1) .. + 3; lane 7's last
  // dword is tag1), summed over lanes 0-7 (svc_sum8; lane 0's data is 0)
  const uint32_t i0 = 4u * (lane - 1u);
  const uint32_t part = d.x * svc_weight(i0) + d.y * svc_weight(i0 + 1u) + d.z * svc_weight(i0 + 2u) +
                        (lane < 7u ? d.w * svc_weight(i0 + 3u) : 0u);
  const uint32_t sum = readlane(svc_sum8(part), 0);
  if (lane == 0u) d = svc_u32x4{want, (uint32_t)rc, sum, 0u};
  if (lane == 7u) d.w = want;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(&box->reply[sidx], 0, 128, 0x00020000);
  // sc0 sc1: straight to system memory
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, lane < 8u ? (int)(16u * lane) : (int)0x80000000, 0, 17);
}

// The service loop shared by both kinds: polls, takes each
// pending slot's request (from its post, or fetched), runs serve(sidx, args,
// &res) -- the input at lds[0, csize), returning the return word after
// writing the result bytes to obox->slot[sidx].out (and setting res to the
// result's LDS copy, if it has one) -- then writes the reply (short results
// in LDS) and publishes (request << 32 | rc) in the slot's done word.  Every wave reaches an exit: idle_ticks without a
// request, life_ticks in all, or the host's stop.
template <class Serve>
__device__ __forceinline__ void svc_loop(const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks, uint64_t life_ticks,
                                         uint8_t* lds, uint32_t max_in, Serve serve) {
  const uint32_t lane = lane_id();
  // lane i: the last request of slot i served
  uint32_t seen = (uint32_t)(__hip_atomic_load(&obox->done[lane], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >> 32);
  const uint64_t t0 = wall_clock64();
#if KDB_SVC_DEBUG   // (diagnostic: instances of this box running at once)
  if (lane == 0) {
    const uint32_t was = __hip_atomic_fetch_add(&obox->pad[0], 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    if (was != 0u) __hip_atomic_fetch_add(&obox->pad[1], 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
  }
#endif
  uint64_t t_last = t0;
  uint32_t served = 0, polls = 0, inl = 0, rep = 0;
#if KDB_SVC_DEBUG   // (diagnostic: wall-clock ticks spent fetching, serving, answering)
  uint64_t dbg_fetch = 0, dbg_serve = 0, dbg_answer = 0;
#endif
  uint32_t act = kSvcPostSlots;
  const bool post_on = svc_relaxed(&ibox->no_post) == 0u, reply_on = svc_relaxed(&ibox->no_reply) == 0u;
  const svc_u32x4 pw = svc_post_weights(lane);
  auto serve_pending = [&](uint64_t pend, const SvcPoll& q) {
#pragma unroll 1
    while (pend) {
      const uint32_t sidx = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1u;
      const uint32_t want = readlane(q.r, sidx);
#if KDB_SVC_DEBUG
      const uint64_t ta = wall_clock64();
#endif
      SvcArgs a;
      const int how = post_on ? svc_from_post(q, sidx, want, lds, &a, pw) : 0;
      if (how == 1) {
        inl++;
      } else {
        // the doorbell's writes before the fetch's plain loads (a relaxed
        // load of the doorbell + this fence synchronise with its release)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (how == 2) svc_fetch_input(ibox, sidx, lds, a.csize, max_in);   // the arguments came with the poll
        else a = svc_fetch(ibox, sidx, lds, max_in);
      }
      const uint8_t* res = nullptr;
#if KDB_SVC_DEBUG
      const uint64_t tb = wall_clock64();
#endif
      const int rc = serve(sidx, a, &res);
#if KDB_SVC_DEBUG
      const uint64_t tc = wall_clock64();
      dbg_fetch += tb - ta;
      dbg_serve += tc - tb;
#endif
      if (res && reply_on && svc_replies(sidx, rc)) {
        // the reply carries the result; the done word only says so (kSvcReplied
        // | rc), relaxed: no wait for any earlier write to be acknowledged
        svc_write_reply(obox, sidx, want, rc, res);
        if (lane == 0)
          __hip_atomic_store(&obox->done[sidx], ((uint64_t)want << 32) | (kSvcReplied | (uint32_t)rc),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        rep++;
      } else {
        // after the bytes (plain stores, which may sit dirty in L2): the
        // request and its return value, one store
        svc_release();
        if (lane == 0)
          __hip_atomic_store(&obox->done[sidx], ((uint64_t)want << 32) | (uint32_t)rc, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (lane == sidx) seen = want;
#if KDB_SVC_DEBUG
      dbg_answer += wall_clock64() - tc;
#endif
      served++;
    }
  };
  // true when the wave leaves
  auto look = [&](const SvcPoll& q) -> bool {
    // the posts consumed on every path: otherwise the compiler sinks their
    // loads into the branch that serves, issued only once the doorbell is
    // back -- a second round trip on every request (0.39 us measured); here
    // they are waited for with the doorbells they travelled with
    asm volatile("" ::"v"(q.p0), "v"(q.p1));
    polls++;
    act = uni(q.act);
    const uint64_t pend = ballot(q.r != seen);
    if (pend) {
      serve_pending(pend, q);
      t_last = wall_clock64();
      return false;
    }
    const uint64_t now = wall_clock64();
    const bool stop = uni(q.stop) != 0u, old = now - t0 > life_ticks;
    if (!(stop || old || now - t_last > idle_ticks)) {
      __builtin_amdgcn_s_sleep(1);
      return false;
    }
    // leave: clear alive (when it is still this instance's), then look at
    // the doorbells once more.  A caller that rang before it read alive sees
    // alive set, so it is served here (idle: and the wave goes on; at its end
    // of life or at stop: these last ones, then it leaves); one that rang
    // later sees it clear and launches the next instance, which queues behind
    // this one.
    if (lane == 0 && svc_relaxed(&obox->alive) == gen) svc_store(&obox->alive, 0u);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const SvcPoll q2 = svc_poll(ibox, act);
    const uint64_t pend2 = ballot(q2.r != seen);
    if (pend2 == 0) return true;
    serve_pending(pend2, q2);
    if (stop || old) return true;
    if (lane == 0 && svc_relaxed(&obox->alive) == 0u) svc_store(&obox->alive, gen);
    t_last = wall_clock64();
    return false;
  };
  if (svc_relaxed(&ibox->no_pipe) != 0u) {
    // one poll in flight at a time
#pragma unroll 1
    for (;;) {
      const SvcPoll q = svc_poll(ibox, act);
      if (look(q)) break;
    }
  } else {
    // Two polls in flight, half a read latency apart: each is looked at
    // while the next one travels, so a doorbell is seen about half a latency
    // sooner.  Every poll's state (stop included) travels with it, so a look
    // waits for nothing younger.  (A request answered by its done word waits,
    // at its release, for the poll in flight too.)  Unrolled by two so that
    // no poll's registers are copied while its loads are still filling them.
    SvcPoll qa = svc_poll(ibox, act);
    __builtin_amdgcn_s_sleep(16);   // ~1 000 cycles: the stagger
#pragma unroll 1
    for (;;) {
      const SvcPoll qb = svc_poll(ibox, act);
      if (look(qa)) break;
      qa = svc_poll(ibox, act);
      if (look(qb)) break;
    }
  }
#if KDB_SVC_DEBUG
  if (lane == 0) {
    __hip_atomic_fetch_sub(&obox->pad[0], 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(&obox->pad[2], (uint32_t)dbg_fetch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(&obox->pad[3], (uint32_t)dbg_serve, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(&obox->pad[4], (uint32_t)dbg_answer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(&obox->pad[5], (uint32_t)(wall_clock64() - t0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
#endif
  svc_release();
  if (lane == 0) {   // (statistics: relaxed)
    __hip_atomic_store(&obox->served, svc_relaxed(&obox->served) + served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&obox->polls, svc_relaxed(&obox->polls) + polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&obox->inline_served, svc_relaxed(&obox->inline_served) + inl, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&obox->replied, svc_relaxed(&obox->replied) + rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace kdb_lz4
