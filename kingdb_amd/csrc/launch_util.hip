// kingdb_amd/csrc/launch_util.hip -- launch plumbing shared by the kernels:
// persistent-grid sizing and the per-launch work counters they dequeue from.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "lz4_device.h"

namespace kdb_lz4 {

namespace {
// Per-device pool of 8 KiB counter slots (a WorkQueue's kQueues counters,
// kQueueStride apart).  A launch takes the next slot round-robin and zeroes
// it on its own stream.  Each slot carries an event recorded on the stream of
// its last user (work_counter_release, after the launches that read it): a
// slot handed out again -- 1024 launches later -- first waits for that event,
// so a slot is never zeroed under a kernel still dequeuing from it, whatever
// the number of streams and host threads.
constexpr uint32_t kSlotBytes = kQueues * kQueueStride * 4u, kSlots = 1024;
static_assert(kSlotBytes == 8192u, "32 counters 256 B apart");
struct Pool {
  uint8_t* base = nullptr;
  std::atomic<uint32_t> next{0};
  hipEvent_t ev[kSlots] = {};
  bool live[kSlots] = {};
  std::mutex mu;               // guards ev/live
};
std::mutex g_mu;
std::unordered_map<int, Pool*> g_pools;

Pool* pool_of(uint8_t* ctr, uint32_t* slot) {
  std::lock_guard<std::mutex> l(g_mu);
  for (auto& kv : g_pools) {
    Pool* p = kv.second;
    if (p && ctr >= p->base && ctr < p->base + (size_t)kSlots * kSlotBytes) {
      *slot = (uint32_t)((ctr - p->base) / kSlotBytes);
      return p;
    }
  }
  return nullptr;
}
}  // namespace

hipError_t work_counter(hipStream_t st, uint32_t** ctr) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  Pool* p;
  {
    std::lock_guard<std::mutex> l(g_mu);
    Pool*& slot = g_pools[dev];
    if (!slot) {
      slot = new Pool();
      e = hipMalloc(&slot->base, (size_t)kSlots * kSlotBytes);
      if (e != hipSuccess) {
        delete slot;
        slot = nullptr;
        return e;
      }
    }
    p = slot;
  }
  const uint32_t i = p->next.fetch_add(1) % kSlots;
  {
    std::lock_guard<std::mutex> l(p->mu);
    if (p->live[i]) {                  // the slot's previous users must be done with it
      e = hipEventSynchronize(p->ev[i]);
      if (e != hipSuccess) return e;
      p->live[i] = false;
    }
  }
  uint8_t* c = p->base + (size_t)i * kSlotBytes;
  e = hipMemsetAsync(c, 0, kSlotBytes, st);
  *ctr = reinterpret_cast<uint32_t*>(c);
  return e;
}

// The launches that read `ctr` are all queued on `st` (or joined into it):
// record the slot's fence there.
hipError_t work_counter_release(hipStream_t st, uint32_t* ctr) {
  if (!ctr) return hipSuccess;
  uint32_t i = 0;
  Pool* p = pool_of(reinterpret_cast<uint8_t*>(ctr), &i);
  if (!p) return hipErrorInvalidValue;
  std::lock_guard<std::mutex> l(p->mu);
  hipError_t e = hipSuccess;
  if (!p->ev[i] && (e = hipEventCreateWithFlags(&p->ev[i], hipEventDisableTiming)) != hipSuccess) return e;
  if ((e = hipEventRecord(p->ev[i], st)) != hipSuccess) return e;
  p->live[i] = true;
  return hipSuccess;
}

long kdb_tune(const char* name, long dflt) {
#ifdef KDB_LZ4_TUNING
  const char* e = getenv(name);
  return e && *e ? strtol(e, nullptr, 0) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

hipError_t launch_counter(hipStream_t st, uint32_t n, uint32_t grid, uint32_t** ctr) {
  *ctr = nullptr;
  if (grid >= n) return hipSuccess;
  return work_counter(st, ctr);
}

uint32_t services_resident(int dev);   // kdb_lz4_capi.hip (service.h)

// Workgroups of 64 threads resident at once for `kern` with `lds` bytes of
// dynamic LDS, capped at n (the kernels dequeue values dynamically, so a
// workgroup that is admitted late simply takes fewer values).
// `waves` > 1: workgroups of that many waves (one value each at a time), at
// most ceil(n / waves) of them.
uint32_t persistent_grid(const void* kern, size_t lds, uint32_t n, uint32_t waves) {
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * (int)waves, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  static const int cap = (int)kdb_tune("KDB_LZ4_PER_CU", 0);   // cap workgroups per CU
  if (cap > 0 && per_cu > cap) per_cu = cap;
  static const bool dbg = kdb_tune("KDB_LZ4_DEBUG", 0) != 0;
  if (dbg) fprintf(stderr, "persistent_grid: lds=%zu per_cu=%d cus=%d\n", lds, per_cu, cus);
  uint64_t slots = (uint64_t)per_cu * (uint64_t)cus;
  // a resident service wave (service.h) holds a wave slot and LDS on some CU
  // for as long as calls keep coming: a grid that counted on that CU's full
  // capacity would leave a workgroup waiting behind it, and the launch's tail
  // with it, so each one resident on this device takes a margin off the grid
  // (a workgroup of several waves waits for a whole CU's worth: one per wave)
  const uint32_t svc = services_resident(dev);
  const uint64_t margin = waves > 1 ? svc : 8u * svc;
  if (svc) slots = slots > margin + 1u ? slots - margin : 1u;
  const uint32_t groups = waves > 1 ? (uint32_t)(((uint64_t)n + waves - 1u) / waves) : n;
  return (uint32_t)(groups < slots ? groups : slots);
}

// Fork/join of a second stream, so that size-class launches overlap: the
// long-latency big-value class runs beside the small classes, and its tail
// (the last few big values) no longer idles the rest of the GPU.  One
// non-blocking stream and two events per host thread, device and CALLER
// stream: batches a caller issues on different streams keep their own aux
// streams, so one batch's big class never queues behind another's.  The set
// is bounded per thread (kForks, least recently used out): a caller that
// makes a stream per request does not grow it without end; an evicted aux
// stream is drained before it is destroyed.
namespace {
struct Fork {
  int dev = -1;
  hipStream_t st = nullptr;
  hipStream_t aux = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  uint64_t used = 0;
};
constexpr int kForks = 8;
thread_local Fork t_fork[kForks];
thread_local uint64_t t_fork_clock = 0;

void fork_destroy(Fork& f) {
  if (f.aux) {
    (void)hipStreamSynchronize(f.aux);
    (void)hipStreamDestroy(f.aux);
  }
  if (f.fork) (void)hipEventDestroy(f.fork);
  if (f.join) (void)hipEventDestroy(f.join);
  f = Fork();
}

// the entry of (dev, st); with create, a fresh one in the least recently used slot
Fork* fork_of(int dev, hipStream_t st, bool create, hipError_t* e) {
  *e = hipSuccess;
  Fork* lru = &t_fork[0];
  for (Fork& f : t_fork) {
    if (f.aux && f.dev == dev && f.st == st) {
      f.used = ++t_fork_clock;
      return &f;
    }
    if (f.used < lru->used) lru = &f;
  }
  if (!create) return nullptr;
  fork_destroy(*lru);
  Fork f;
  f.dev = dev;
  f.st = st;
  if ((*e = hipStreamCreateWithFlags(&f.aux, hipStreamNonBlocking)) != hipSuccess ||
      (*e = hipEventCreateWithFlags(&f.fork, hipEventDisableTiming)) != hipSuccess ||
      (*e = hipEventCreateWithFlags(&f.join, hipEventDisableTiming)) != hipSuccess) {
    fork_destroy(f);
    return nullptr;
  }
  f.used = ++t_fork_clock;
  *lru = f;
  return lru;
}
}  // namespace

hipError_t fork_begin(hipStream_t st, hipStream_t* aux) {
  static const bool off = kdb_tune("KDB_LZ4_NOFORK", 0) != 0;   // classes in sequence on one stream
  *aux = st;
  if (off) return hipSuccess;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  Fork* f = fork_of(dev, st, true, &e);
  if (!f) return e;
  if ((e = hipEventRecord(f->fork, st)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(f->aux, f->fork, 0)) != hipSuccess) return e;
  *aux = f->aux;
  return hipSuccess;
}

// st waits for everything queued on aux (no-op when aux == st)
hipError_t fork_end(hipStream_t st, hipStream_t aux) {
  if (aux == st) return hipSuccess;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  Fork* f = fork_of(dev, st, false, &e);
  if (!f || f->aux != aux) return hipErrorInvalidHandle;
  if ((e = hipEventRecord(f->join, aux)) != hipSuccess) return e;
  return hipStreamWaitEvent(st, f->join, 0);
}

// Ranges per launch.  Tiny values saturate one counter (128 Ki 100-byte
// values: ~70 claims/us), and even at 4 KiB, where the rate is far below
// that, a contended counter's latency shows: decompress 5.79 ms with one
// range vs 5.30 ms with eight (1 Mi x 4 KiB), 2.65 ms with kQueues (32, see
// lz4_device.h) in round 4.  So: kQueues, unless overridden.
uint32_t work_queues(uint32_t max_len) {
  (void)max_len;
  static const int env = (int)kdb_tune("KDB_LZ4_QUEUES", 0);   // force 1 range (or kQueues)
  if (env > 0) return (uint32_t)env;
  return kQueues;
}

uint32_t claim_guide(uint32_t max_len) {
  static const long env = kdb_tune("KDB_LZ4_GUIDE", -1);   // force a guide (0 = off)
  if (env >= 0) return (uint32_t)env;
  return max_len >= 2048u ? 4u : 0u;
}

// The LDS decoder's launches: guide 1 (a claim at most all that is left per
// wave of its range) for values >= 2 KiB: 1 Mi x 4 KiB decompress 2.64 ->
// 2.59 ms (guide 2 the same; profiles/r04_d/r04_q_ab_decode_guide.txt); the
// 100-byte class keeps fixed claims (a guide cost it more claims than tail).
uint32_t decode_guide(uint32_t max_out) {
  static const long env = kdb_tune("KDB_LZ4_DGUIDE", -1);   // force a guide (0 = off)
  if (env >= 0) return (uint32_t)env;
  return max_out >= 2048u ? 1u : 0u;
}

// Values per counter claim: ~1/8 of a workgroup's share, at most 16, so the
// claim rate stays far below one counter's ceiling and the tail stays short.
uint32_t claim_batch(uint32_t n, uint32_t grid) {
  uint64_t b = grid ? (uint64_t)n / ((uint64_t)grid * 8u) : 1u;
  if (b < 1) b = 1;
  if (b > 16) b = 16;
  return (uint32_t)b;
}

uint32_t env_prio() { return kdb_tune("KDB_LZ4_BIGPRIO", 0) != 0 ? 1u : 0u; }

namespace {
thread_local char t_notes[512];
thread_local size_t t_notes_len = 0;
}  // namespace

void launch_notes_reset() {
  t_notes_len = 0;
  t_notes[0] = 0;
}

void launch_note(const char* kernel) {
  const size_t k = strlen(kernel);
  if (t_notes_len + k + 2 > sizeof(t_notes)) return;
  if (t_notes_len) t_notes[t_notes_len++] = ';';
  memcpy(t_notes + t_notes_len, kernel, k + 1);
  t_notes_len += k;
}

const char* launch_notes() { return t_notes; }

}  // namespace kdb_lz4
