// kingdb_amd/csrc/lz4_device.h -- device-side building blocks shared by the
// gfx950 LZ4 compress / decompress kernels.
//
// Execution model (CDNA4, wave64): one wavefront owns one value.  Control flow
// of the LZ4 parse is wave-uniform (every scalar below is the same in all 64
// lanes and is pinned to SGPRs with readfirstlane); the lanes cooperate on the
// byte work -- staging, literal/match copies, match-length scans (ballot +
// ctz), catch-up scans and the speculative 64-position hash search.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kdb_lz4 {

// LZ4 r1.3.0 constants (/root/reference/algorithm/lz4.cc:222-246, lz4.h:102).
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kLastLiterals = 5;
constexpr uint32_t kMfLimit = 12;
constexpr uint32_t kMinLength = 13;
constexpr uint32_t k64KLimit = 65536u + 11u;   // byU16 iff S < this (lz4.cc:673)
constexpr uint32_t kMaxDistance = 65535u;
constexpr uint32_t kRunMask = 15u;
constexpr uint32_t kMlMask = 15u;
constexpr uint32_t kMaxInput = 0x7E000000u;
constexpr uint32_t kHash16Entries = 8192u;    // 13-bit byU16 hash (lz4.cc:376)
constexpr uint32_t kTableBytes = kHash16Entries * 2u;

// Status word for values a launch cannot process (distinct from every LZ4
// return code, which is >= -(csize+1)).
constexpr int32_t kUnsupported = INT32_MIN;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t uni(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ int unii(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint32_t readlane(uint32_t x, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}

// v_writelane_b32: `old` with lane l replaced by the uniform v (clang has no
// builtin for it; the LLVM intrinsic is declared directly)
extern "C" __device__ int kdb_llvm_writelane(int v, int l, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t l, uint32_t old) {
  return (uint32_t)kdb_llvm_writelane((int)v, (int)l, (int)old);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Lanes-below / lanes-up-to masks (lane in 0..63; 2ull<<63 wraps to 0 -> ~0).
__device__ __forceinline__ uint64_t mask_lt(uint32_t l) { return (1ull << l) - 1ull; }
__device__ __forceinline__ uint64_t mask_le(uint32_t l) { return (2ull << l) - 1ull; }

// Index of the first zero lane in a ballot, 64 if none.
__device__ __forceinline__ uint32_t first_zero(uint64_t m) {
  uint64_t z = ~m;
  return z ? (uint32_t)__builtin_ctzll(z) : 64u;
}
// The same as one s_ff0_i32_b64 (the compiler's ctz(~m) with the "none" case
// is s_not + s_ff1 + s_min): the index of the first zero bit, -1 if none.
__device__ __forceinline__ int first_zero_or_neg(uint64_t m) {
  int r;
  asm("s_ff0_i32_b64 %0, %1" : "=s"(r) : "s"(m));
  return r;
}
// One s_flbit_i32_b64: the number of zero bits above the highest set bit of
// m (lanes 63, 62, ... before the first set one), -1 if m is 0.
__device__ __forceinline__ int leading_zeros_or_neg(uint64_t m) {
  int r;
  asm("s_flbit_i32_b64 %0, %1" : "=s"(r) : "s"(m));
  return r;
}

// Dynamic work distribution of the persistent kernels.  Lane 0 claims `batch`
// consecutive value indices with one device-scope atomic.  A single counter
// saturates near 88 claims/us (microarch "dequeue") -- a launch of 128 Ki
// 100-byte values was bound by exactly that -- so the index space is split
// into kQueues ranges with a counter each: a workgroup starts on range
// blockIdx % kQueues and moves to the next range when its own is exhausted (a
// plain load first, so finished ranges cost no atomics).  next() hands out
// values one ahead of their use.
//
// 32 ranges, counters 256 bytes apart.  Eight counters 64 bytes apart still
// bound the tiny classes: their claims all served together near 60-70 per us
// (1 Mi x 100 B decompress 1.10 ms, compress 1.02 ms); 32 counters 256 B apart
// 0.46 / 0.81 ms, the headline decompress 2.81 -> 2.65 ms and the mixed batch's
// 2.75 -> 2.38 ms (profiles/r04_d/r04_vw_ab_queues.txt: 8 at 4 KiB, 64 at
// 1 KiB or 4 KiB measured the same as 32 at 256 B).
constexpr uint32_t kQueues = 32, kQueueStride = 64;   // counters: 32 x u32, 256 B apart (work_counter slots)
struct WorkQueue {
  uint32_t* ctr;
  uint32_t n, batch, cur, end, nr, q, left, guide;
  // nr ranges: 1, or kQueues for launches whose claim rate would saturate one
  // counter (work_queues() on the host picks)
  // c == nullptr: a direct launch (grid == n, see launch_counter), workgroup b
  // takes value b and nothing else -- no counter, so no memset before it.
  // guide > 0: guided claims -- a claim takes at most 1/guide of what is left
  // per wave of its range, so claims shrink as a range runs out and the waves'
  // last claims end close together (the launch's tail is one small claim).
  // For values with work enough per claim (the host sets it from the batch's
  // largest value): 1 Mi x 4 KiB compress 9.01 -> 8.85 ms; 100-byte values
  // and the decoders lose more to the extra claims than the tail gives back
  // (profiles/r04_d/r04_y_ab_guided.txt).
  // vb / vgrid: this wave's index among the launch's waves and their number
  // (the workgroup's and the grid's, for one-wave workgroups)
  __device__ static WorkQueue make(uint32_t* c, uint32_t n, uint32_t batch, uint32_t nr, uint32_t guide = 0,
                                   uint32_t vb = blockIdx.x, uint32_t vgrid = gridDim.x) {
    if (!c) return WorkQueue{c, n, batch, vb, min(vb + 1u, n), 1u, 0u, 0u, 0u};
    nr = nr > 1u ? kQueues : 1u;
    // a guided claim divides what is left by guide x (waves per range)
    return WorkQueue{c, n, batch, 0u, 0u, nr, vb % nr, nr, guide * max(vgrid / nr, 1u)};
  }
  __device__ __forceinline__ void claim() {
    while (left) {
      const uint32_t lo = (uint32_t)((uint64_t)n * q / nr), hi = (uint32_t)((uint64_t)n * (q + 1u) / nr);
      uint32_t v = 0, b = batch;
      if (lane_id() == 0) {
        uint32_t* c = ctr + kQueueStride * q;
        const uint32_t seen = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (seen < hi - lo) {
          if (guide) {
            const uint32_t per = (hi - lo - seen) / guide;
            b = per < 1u ? 1u : per < batch ? per : batch;
          }
          v = atomicAdd(c, b);
        } else {
          v = hi - lo;
        }
      }
      v = uni(v);
      b = uni(b);
      if (v < hi - lo) {
        cur = lo + v;
        end = min(cur + b, hi);
        return;
      }
      q = q + 1u == nr ? 0u : q + 1u;
      left--;
    }
    cur = end = n;
  }
  __device__ __forceinline__ uint32_t next() {   // n when every range is exhausted
    if (cur >= end) {
      claim();
      if (cur >= end) return n;
    }
    return cur++;
  }
};

// Per-value metadata read through the scalar cache (s_load, counted by
// lgkmcnt): a vector load would be counted by vmcnt behind the next value's
// prefetch loads and the previous value's byte stores, and waiting for it
// (vmcnt(0): the counts are not static) exposed the whole prefetch latency
// at every value.
template <class T>
__device__ __forceinline__ T sload(const T* p, uint32_t i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// LZ4_compressBound (lz4.h:103).
__host__ __device__ __forceinline__ uint32_t compress_bound(uint32_t n) {
  return n > kMaxInput ? 0u : n + n / 255u + 16u;
}

// Unaligned little-endian u32 at byte offset b of a 16B-aligned LDS buffer
// that is readable for 4 bytes past b+3 (two aligned dwords + v_alignbyte).
// (A single unaligned ds_read_b32 returns the same bytes on gfx950 --
// tools/probe/lds_unaligned.hip -- but measured far slower: compress 11.3 ->
// 13.8 ms, decompress 3.6 -> 5.6 ms at 1 Mi x 4 KiB.)
__device__ __forceinline__ uint32_t lds_rd32(const uint8_t* lds, uint32_t b) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds);
  uint32_t q = b >> 2;
  return __builtin_amdgcn_alignbyte(w[q + 1], w[q], b & 3u);   // (without the & 3: compress slower, r04_h)
}

// Copies n bytes at global g (any alignment) into the 16B-aligned LDS buffer
// `lds` with whole aligned 16-byte loads; byte i of the value lands at
// lds[head + i] with head = g & 15 (returned).  An aligned 16-byte chunk never
// crosses a page, so the over-read around [g, g+n) cannot fault.  The pointer
// is rebased with pointer arithmetic (not via an integer) so the compiler keeps
// the global address space: global_load_dwordx4, not flat.
__device__ __forceinline__ uint32_t stage_to_lds(const uint8_t* g, uint32_t n, uint8_t* lds) {
  const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
  const uint4* base = reinterpret_cast<const uint4*>(g - head);
  const uint32_t chunks = (head + n + 15u) >> 4;
  uint4* l = reinterpret_cast<uint4*>(lds);
  for (uint32_t c = lane_id(); c < chunks; c += 64u) l[c] = base[c];
  return head;
}

// Stores bytes lds_base[off .. off+n) (lds_base 16B-aligned LDS) to global g
// (any alignment): byte stores up to g's 16-byte boundary, then 16-byte stores
// (ds_read_b128 when the LDS side is aligned too), then the tail.
__device__ __forceinline__ void flush_lds_to_global(uint8_t* g, const uint8_t* lds_base, uint32_t off,
                                                    uint32_t n) {
  const uint32_t lane = lane_id();
  const uint32_t mis = (uint32_t)((16u - (reinterpret_cast<uintptr_t>(g) & 15u)) & 15u);
  const uint32_t pre = mis < n ? mis : n;
  if (lane < pre) g[lane] = lds_base[off + lane];
  const uint32_t body = (n - pre) >> 4;
  uint4* g4 = reinterpret_cast<uint4*>(g + pre);
  const uint32_t sb = off + pre;
  if ((sb & 15u) == 0) {
    const uint4* l4 = reinterpret_cast<const uint4*>(lds_base + sb);
    for (uint32_t i = lane; i < body; i += 64u) g4[i] = l4[i];
  } else {
    for (uint32_t i = lane; i < body; i += 64u) {
      const uint32_t b = sb + 16u * i;
      g4[i] = make_uint4(lds_rd32(lds_base, b), lds_rd32(lds_base, b + 4u), lds_rd32(lds_base, b + 8u),
                         lds_rd32(lds_base, b + 12u));
    }
  }
  const uint32_t done = pre + 16u * body;
  if (lane < n - done) g[done + lane] = lds_base[off + done + lane];
}

// Diagnostic knobs for A/B experiments (class splits, ring sizes, grid caps,
// stream fork): read from the environment only in a build with
// -DKDB_LZ4_TUNING (tools/build_variants.sh <name>:-DKDB_LZ4_TUNING); the
// shipped library always uses the defaults.
long kdb_tune(const char* name, long dflt);

hipError_t work_counter(hipStream_t st, uint32_t** ctr);
// after the launches reading a counter slot are queued on st: fences the slot
// against reuse (launch_util.hip)
hipError_t work_counter_release(hipStream_t st, uint32_t* ctr);
uint32_t persistent_grid(const void* kern, size_t lds, uint32_t n, uint32_t waves = 1);
// service waves (service.h) resident on `dev` right now (kdb_lz4_capi.hip)
uint32_t services_resident(int dev);
// The launch's work counter: a direct launch (n no larger than the resident
// grid, so one value per workgroup) needs none (*ctr = nullptr, no memset:
// the scalar entry points' latency); otherwise a zeroed counter slot.
hipError_t launch_counter(hipStream_t st, uint32_t n, uint32_t grid, uint32_t** ctr);
uint32_t claim_batch(uint32_t n, uint32_t grid);
// the WorkQueue guide for a launch whose values are up to max_len bytes
uint32_t claim_guide(uint32_t max_len);
// the same for the LDS decoder's launches (max_out: their largest output)
uint32_t decode_guide(uint32_t max_out);
// WorkQueue ranges for a launch whose values are at most max_len bytes
uint32_t work_queues(uint32_t max_len);
// size-class launches on a second stream: *aux waits for st's work so far;
// fork_end makes st wait for aux (KDB_LZ4_NOFORK=1: aux == st)
hipError_t fork_begin(hipStream_t st, hipStream_t* aux);
hipError_t fork_end(hipStream_t st, hipStream_t aux);
// wave priority of the big-value (in-place / ring) class launches, whose
// values are a mixed batch's critical path (KDB_LZ4_BIGPRIO, default 0)
uint32_t env_prio();
// The kernels the calling thread's last launch_compress / launch_decompress
// queued, by their rocprof names (kdb_lz4_last_kernels): the bench labels its
// roofline with them instead of guessing from the size classes.
// The compressor's lane-order guard (selftest.hip): runs the device self-test
// once per device; hipErrorNotSupported when the device fails it.
hipError_t lane_order_check();
int lane_order_state(int dev, uint32_t* bad);
// lane_order_check behind a per-thread cache of the last device that passed
inline hipError_t lane_order_ok() {
  static thread_local int ok_dev = -1;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess || dev == ok_dev) return e;
  e = lane_order_check();
  if (e == hipSuccess) ok_dev = dev;
  return e;
}
void launch_notes_reset();
void launch_note(const char* kernel);
const char* launch_notes();

}  // namespace kdb_lz4
