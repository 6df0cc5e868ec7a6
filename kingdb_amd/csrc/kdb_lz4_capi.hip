// kingdb_amd/csrc/kdb_lz4_capi.hip -- the C ABI declared in include/kdb_lz4.h.
//
// Batch entry points launch the gfx950 kernels on the caller's stream.  The
// scalar LZ4 mirrors (one value per call, host buffers) go through the same
// kernels as a batch of one, using a per-thread, per-device staging context
// (pinned host + device buffers + a private stream) that grows on demand.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../../include/kdb_lz4.h"
#include "lz4_device.h"
#include "service.h"

namespace kdb_lz4 {
hipError_t launch_compress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                           const uint32_t* src_len, uint32_t n, uint32_t min_len, uint32_t max_len, uint8_t* dst,
                           const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t* frame_len,
                           int32_t* ret);
hipError_t launch_decompress(bool frame, hipStream_t st, const uint8_t* src, const uint64_t* src_off,
                             const uint32_t* in_len, uint32_t n, uint32_t max_in, uint32_t max_out,
                             uint8_t* dst, const uint64_t* dst_off, const uint32_t* out_cap,
                             const uint32_t* target, uint32_t* out_len, int32_t* ret);
hipError_t launch_gen_g1(uint8_t* dst, uint64_t first_piece, uint64_t npieces, uint32_t seed,
                         hipStream_t st);
hipError_t launch_decode_service(hipStream_t st, const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks,
                                 uint64_t life_ticks);
hipError_t launch_compress_service(hipStream_t st, const SvcBox* ibox, SvcBox* obox, uint32_t gen, uint64_t idle_ticks,
                                   uint64_t life_ticks);
}  // namespace kdb_lz4

using namespace kdb_lz4;

namespace {

inline int hip_status(hipError_t e) {
  if (e == hipSuccess) return KDB_LZ4_OK;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorInsufficientDriver)
    return KDB_LZ4_ENODEV;
  if (e == hipErrorNotSupported) return KDB_LZ4_EUNSUPPORTED;   // the lane-order self-test failed
  return KDB_LZ4_EHIP;
}

// Largest value the byU16 kernels take (lz4.cc:673: S < 65547).

// Per-thread, per-device context of the scalar entry points.
//
// A scalar call is latency, not bandwidth: one value, one kernel, the caller
// waiting.  Values whose class kernel touches each input byte once and writes
// each output byte once (compress <= 8 KiB, decode of <= 8 KiB output: the
// LDS-staged kernels) run ZERO-COPY: metadata, input and output live in one
// pinned, coherent, device-mapped host buffer that the kernel reads and writes
// over PCIe -- one launch and one stream sync per call, no DMA.  Larger values
// (the in-place kernels read the input many times; the ring decoder reads
// back its own output) are staged through device memory: one H2D copy, the
// launch, one D2H copy of metadata + output, one sync.
struct ScalarCtx {
  hipStream_t stream = nullptr;
  uint8_t* host = nullptr;    // pinned, coherent, mapped: [meta 64 B][in][out]
  uint8_t* hdev = nullptr;    // its device address
  size_t hcap = 0;
  uint8_t* dev = nullptr;     // device staging for large values: [meta 64 B][out][in]
  size_t dcap = 0;
  ~ScalarCtx() {
    if (dev) (void)hipFree(dev);
    if (host) (void)hipHostFree(host);
    if (stream) (void)hipStreamDestroy(stream);
  }
  // A failed call returns only once nothing it queued can still write the
  // staging the next call reuses; if the stream cannot even be drained, the
  // buffers are dropped (leaked, not freed) and the next call allocates anew.
  int failed(int ret) {
    if (stream && hipStreamSynchronize(stream) != hipSuccess) {
      host = hdev = dev = nullptr;
      hcap = dcap = 0;
      stream = nullptr;
    }
    return ret;
  }
  static size_t grow(size_t have, size_t bytes) {
    size_t want = have ? have : 1u << 16;
    while (want < bytes) want *= 2;
    return want;
  }
  int reserve(size_t host_bytes, size_t dev_bytes) {
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return KDB_LZ4_EHIP;
    if (host_bytes > hcap) {
      if (host) (void)hipHostFree(host);
      host = hdev = nullptr;
      hcap = 0;
      const size_t want = grow(0, host_bytes);
      if (hipHostMalloc(&host, want, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return KDB_LZ4_EHIP;
      if (hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), host, 0) != hipSuccess) return KDB_LZ4_EHIP;
      hcap = want;
    }
    if (dev_bytes > dcap) {
      if (dev) (void)hipFree(dev);
      dev = nullptr;
      dcap = 0;
      const size_t want = grow(0, dev_bytes);
      if (hipMalloc(&dev, want) != hipSuccess) return KDB_LZ4_EHIP;
      dcap = want;
    }
    return KDB_LZ4_OK;
  }
};

ScalarCtx& scalar_ctx(int* err) {
  thread_local std::unordered_map<int, ScalarCtx> ctxs;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  *err = hip_status(e);
  return ctxs[dev];
}

// Layout of the scalar staging buffers: a 64-byte metadata block (offsets,
// lengths, caps, results) followed by the input and output regions.
struct Meta {
  uint64_t src_off, dst_off;
  uint32_t len, cap, target, out_len;
  int32_t ret, pad;
};
static_assert(sizeof(Meta) <= 64, "meta block");
constexpr size_t kMetaBytes = 64;
// Largest value (compress) / output (decode) the zero-copy route takes: the
// LDS-staged class kernels (lz4_compress.hip kMidLdsMax, the decoder's
// default LDS split).
constexpr uint32_t kZeroCopyMax = 8192u;

inline size_t align16(size_t x) { return (x + 15u) & ~(size_t)15u; }

inline Meta read_meta(const uint8_t* p) {
  Meta m;
  memcpy(&m, const_cast<const uint8_t*>(p), sizeof(m));
  return m;
}

// ---- the resident services (service.h): per device and process, up to
// KDB_LZ4_SERVICE_WAVES (default 8, at most 16) waves for per-call decodes and as many for
// per-call compressions, each with a mailbox and a stream of its own; a
// calling thread is assigned one of them (round robin) with its slot, so
// concurrent callers are served side by side.  KDB_LZ4_SERVICE=0 turns it
// off (every call launches, as before); KDB_LZ4_SERVICE_IDLE_US (default
// 2000) is how long a wave waits for the next request before it exits.
bool service_on() {
  static const bool on = [] {
    const char* e = getenv("KDB_LZ4_SERVICE");
    return !(e && *e == '0');
  }();
  return on;
}

enum SvcKind { kSvcDecode = 0, kSvcCompress = 1 };
constexpr int kSvcWavesMax = 16;
int svc_waves() {
  static const int n = [] {
    const char* e = getenv("KDB_LZ4_SERVICE_WAVES");
    const int v = e && *e ? atoi(e) : 8;
    return v < 1 ? 1 : (v > kSvcWavesMax ? kSvcWavesMax : v);
  }();
  return n;
}
// services()[svc_index(device, kind, wave)]
inline size_t svc_index(int dev, int kind, int wave) {
  return ((size_t)dev * 2u + (size_t)kind) * (size_t)kSvcWavesMax + (size_t)wave;
}
// The inbox may be a write-combining BAR mapping: its stores leave the core's
// buffers, in no particular order, at a store fence (a no-op cost on host memory).
inline void svc_wc_fence() { __builtin_ia32_sfence(); }
struct Service {
  std::mutex mu;
  int kind = kSvcDecode;
  int wave = 0;
  hipStream_t stream = nullptr;
  SvcBox* box = nullptr;     // the outbox, host view (pinned, coherent, mapped); also the host's copies
                             // of req and active
  SvcBox* dbox = nullptr;    // its device address
  SvcBox* in = nullptr;      // the inbox, host view: device memory through the BAR, or `box` (service.h)
  SvcBox* din = nullptr;     // its device address
  bool in_device = false;
  bool no_reply = false;     // KDB_LZ4_SVC_REPLY=0 (also in the inbox, for the wave)
  uint64_t idle_ticks = 0, life_ticks = 0;
  std::vector<int> free_slots;
  bool ok = false;
  int device = 0;
  bool launch() {            // (mu held) a new instance, behind any old one on the stream
    // its generation (never 0) marks `alive` as its own: an older instance
    // that exits later leaves it alone (service.h)
    uint32_t gen = box->gen + 1u;
    if (gen == 0u) gen = 1u;
    box->gen = gen;
    __atomic_store_n(&box->alive, gen, __ATOMIC_SEQ_CST);
    const hipError_t e = kind == kSvcDecode ? launch_decode_service(stream, din, dbox, gen, idle_ticks, life_ticks)
                                            : launch_compress_service(stream, din, dbox, gen, idle_ticks, life_ticks);
    if (e != hipSuccess) {
      __atomic_store_n(&box->alive, 0u, __ATOMIC_SEQ_CST);
      return false;
    }
    box->launches++;
    return true;
  }
  void ensure_running() {
    if (__atomic_load_n(&box->alive, __ATOMIC_SEQ_CST) != 0u) return;
    std::lock_guard<std::mutex> l(mu);
    if (__atomic_load_n(&box->alive, __ATOMIC_SEQ_CST) == 0u) (void)launch();
  }
};

std::mutex g_svc_mu;
std::vector<Service*>& services() {
  static std::vector<Service*>* v = new std::vector<Service*>();   // never destroyed: waves may still read them
  return *v;
}
// process teardown: every service wave is told to leave, and is given a
// moment to (it also leaves by itself once idle)
void stop_services() {
  std::lock_guard<std::mutex> l(g_svc_mu);
  for (Service* s : services()) {
    if (!s || !s->ok) continue;
    __atomic_store_n(&s->in->stop, 1u, __ATOMIC_SEQ_CST);
    svc_wc_fence();
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(&s->box->alive, __ATOMIC_SEQ_CST) != 0u &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(50)) {
    }
#if KDB_SVC_DEBUG   // (diagnostic build: where a served request's wave time went, in 10 ns ticks)
    const SvcBox* b = s->box;
    if (b->served)
      fprintf(stderr,
              "SVCDBG kind %d wave %d: served %u (from the poll %u, replied %u) polls %u launches %u; per request: "
              "fetch %.0f serve %.0f answer %.0f ticks; wave time per poll %.1f ticks\n",
              s->kind, s->wave, b->served, b->inline_served, b->replied, b->polls, b->launches, (double)b->pad[2] / b->served,
              (double)b->pad[3] / b->served, (double)b->pad[4] / b->served, (double)b->pad[5] / (b->polls + 1));
#endif
  }
}

// Whether [p, p + n) lies inside one mapping of this process (/proc/self/maps):
// a device allocation the CPU can reach through the large BAR is mapped at its
// device address; one it cannot is not mapped at all.
bool host_mapped(const void* p, size_t n) {
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  unsigned long lo = 0, hi = 0;
  bool in = false;
  char line[512];
  while (!in && fgets(line, sizeof(line), f))
    if (sscanf(line, "%lx-%lx", &lo, &hi) == 2 && lo <= a && a + n <= hi) in = true;
  fclose(f);
  return in;
}
// The inbox in fine-grained device memory the host writes through the BAR
// (service.h), when the device has a large BAR (KDB_LZ4_SVC_INBOX=host keeps
// it in host memory); nullptr when it cannot be had.
SvcBox* device_inbox(int dev, hipStream_t st) {
  const char* e = getenv("KDB_LZ4_SVC_INBOX");
  if (e && strcmp(e, "host") == 0) return nullptr;
  int large_bar = 0;
  if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) != hipSuccess || !large_bar) return nullptr;
  void* d = nullptr;
  if (hipExtMallocWithFlags(&d, sizeof(SvcBox), hipDeviceMallocFinegrained) != hipSuccess) return nullptr;
  SvcBox* b = static_cast<SvcBox*>(d);
  bool ok = hipMemsetAsync(d, 0, sizeof(SvcBox), st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess &&
            host_mapped(d, sizeof(SvcBox));
  if (ok) {   // a canary through the mapping and back
    __atomic_store_n(&b->pad[0], 0x5A17C0DEu, __ATOMIC_SEQ_CST);
    svc_wc_fence();
    ok = __atomic_load_n(&b->pad[0], __ATOMIC_SEQ_CST) == 0x5A17C0DEu;
    __atomic_store_n(&b->pad[0], 0u, __ATOMIC_SEQ_CST);
    svc_wc_fence();
  }
  if (!ok) {
    (void)hipFree(d);
    return nullptr;
  }
  return b;
}

Service* service_of(int dev, int kind, int wave) {
  std::lock_guard<std::mutex> l(g_svc_mu);
  std::vector<Service*>& v = services();
  const size_t at = svc_index(dev, kind, wave);
  if (v.size() <= at) v.resize(at + 1, nullptr);
  if (v[at]) return v[at]->ok ? v[at] : nullptr;
  Service* s = new Service();
  v[at] = s;
  s->device = dev;
  s->kind = kind;
  s->wave = wave;
  void* h = nullptr;
  int rate_khz = 0;
  if (hipHostMalloc(&h, sizeof(SvcBox), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  memset(h, 0, sizeof(SvcBox));
  s->box = static_cast<SvcBox*>(h);
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&s->dbox), h, 0) != hipSuccess ||
      hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
    return nullptr;
  const char* e = getenv("KDB_LZ4_SERVICE_IDLE_US");
  const uint64_t idle_us = e && *e ? strtoull(e, nullptr, 10) : 2000u;
  s->idle_ticks = idle_us * (uint64_t)rate_khz / 1000u;
  s->life_ticks = 20ull * (uint64_t)rate_khz;    // 20 ms, then a fresh instance (bounds how long a
                                                  // batch launch can wait behind the wave for a slot)
  s->in = s->box;
  s->din = s->dbox;
  if (SvcBox* ib = device_inbox(dev, s->stream)) {
    s->in = s->din = ib;
    s->in_device = true;
  }
  for (int i = (int)kSvcSlots - 1; i >= 0; i--) s->free_slots.push_back(i);
  // A/B knobs of the protocol (service.h): KDB_LZ4_SVC_POST=0 has the wave
  // fetch every request, KDB_LZ4_SVC_REPLY=0 answer every one by its done word
  const char* po = getenv("KDB_LZ4_SVC_POST");
  const char* re = getenv("KDB_LZ4_SVC_REPLY");
  s->no_reply = re && *re == '0';
  s->in->no_post = po && *po == '0';
  s->in->no_reply = s->no_reply;
  const char* pp = getenv("KDB_LZ4_SVC_PIPE");   // KDB_LZ4_SVC_PIPE=0: one poll in flight
  s->in->no_pipe = pp && *pp == '0';
  svc_wc_fence();
  static bool registered = false;
  if (!registered) {
    registered = true;
    atexit(stop_services);
  }
  s->ok = true;
  return s;
}

}  // namespace

namespace kdb_lz4 {
uint32_t services_resident(int dev) {
  if (!service_on()) return 0;
  std::lock_guard<std::mutex> l(g_svc_mu);
  const std::vector<Service*>& v = services();
  uint32_t n = 0;
  for (int kind = 0; kind < 2; kind++)
    for (int w = 0; w < kSvcWavesMax; w++) {
      const size_t at = svc_index(dev, kind, w);
      const Service* s = at < v.size() ? v[at] : nullptr;
      if (s && s->ok && __atomic_load_n(&s->box->alive, __ATOMIC_ACQUIRE)) n++;
    }
  return n;
}
}  // namespace kdb_lz4

namespace {

// A calling thread's wave and slot for a device and kind, the slot returned
// when the thread exits; slot -1 when every wave's 64 are taken (the call
// launches instead).
struct Lease {
  Service* s;
  int slot;
};
struct SlotLease {
  std::unordered_map<int, Lease> slot;   // 2 * device + kind -> lease
  ~SlotLease() {
    for (auto& kv : slot) {
      Service* s = kv.second.s;
      if (!s || kv.second.slot < 0) continue;
      std::lock_guard<std::mutex> l(s->mu);
      s->free_slots.push_back(kv.second.slot);
    }
  }
};
thread_local SlotLease t_lease;
std::atomic<unsigned> g_next_wave{0};
Lease lease_of(int dev, int kind) {
  SlotLease& lease = t_lease;
  const int key = 2 * dev + kind;
  auto it = lease.slot.find(key);
  if (it != lease.slot.end()) return it->second;
  const int waves = svc_waves();
  const int first = (int)(g_next_wave.fetch_add(1, std::memory_order_relaxed) % (unsigned)waves);
  Lease got{nullptr, -1};
  for (int i = 0; i < waves && got.slot < 0; i++) {
    Service* s = service_of(dev, kind, (first + i) % waves);
    if (!s) continue;
    std::lock_guard<std::mutex> l(s->mu);
    if (!s->free_slots.empty()) {
      got = Lease{s, s->free_slots.back()};
      s->free_slots.pop_back();
      // how many posts the wave's polls read (service.h): the leased slots'
      const uint32_t hi = (uint32_t)got.slot + 1u;
      if (hi > __atomic_load_n(&s->box->active, __ATOMIC_RELAXED)) {   // (the host's copy)
        const uint32_t a = std::min(hi, kSvcPostSlots);
        __atomic_store_n(&s->box->active, a, __ATOMIC_RELAXED);
        __atomic_store_n(&s->in->active, a, __ATOMIC_RELEASE);
        svc_wc_fence();
      }
    }
  }
  lease.slot[key] = got;
  return got;
}

// One call through a service: the slot's arguments (csize = input bytes,
// osize = output capacity, target) and input; false when it could not be
// used (no service, no free slot, no answer within a second -- the caller
// then launches as before).  *ret = the kernel's return word, the output
// copied to dest when it is > 0.
#if KDB_SVC_DEBUG
thread_local const uint8_t* t_dbg_out = nullptr;
thread_local uint64_t t_dbg_done = 0;
thread_local SvcBox* t_dbg_box = nullptr;
thread_local std::vector<char> t_dbg_last;
#endif
bool service_call(int kind, const char* source, uint32_t in_len, char* dest, uint32_t cap, int target, int* ret) {
  if (!service_on()) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const Lease ls = lease_of(dev, kind);
  if (ls.slot < 0) return false;
  Service* s = ls.s;
  const int k = ls.slot;
  SvcSlot& sl_in = s->in->slot[k];
  SvcSlot& sl = s->box->slot[k];
  // the request number: from the host's copy (the inbox may be device memory,
  // whose reads cross PCIe)
  uint32_t want = __atomic_load_n(&s->box->req[k], __ATOMIC_RELAXED) + 1u;
  if (want == 0u) {
    // 2^32 calls on this slot: 0 is never a request number (a zero-filled reply
    // record or done word would pass for its answer), and a reply record
    // written one wrap ago may carry any tag, so its tags are cleared (the
    // slot's previous request is answered: the wave writes nothing here now)
    want = 1u;
    if ((uint32_t)k < kSvcPostSlots) {
      __atomic_store_n(&s->box->reply[k].tag0, 0u, __ATOMIC_RELAXED);
      __atomic_store_n(&s->box->reply[k].tag1, 0u, __ATOMIC_RELAXED);
    }
  }
  if ((uint32_t)k < kSvcPostSlots) {
    // the post: arguments and (up to kSvcPostInline bytes) the input, the
    // checksum and both tags, built here and written whole (service.h)
    SvcPost p;
    p.tag0 = p.tag1 = want;
    p.csize = in_len;
    p.osize = cap;
    p.target = (uint32_t)target;
    const bool inl = in_len <= kSvcPostInline;
    if (inl) {
      if (in_len) memcpy(p.data, source, in_len);
      memset(p.data + in_len, 0, kSvcPostInline - in_len);
    } else {
      memset(p.data, 0, kSvcPostInline);
      memcpy(sl_in.in, source, in_len);
    }
    uint32_t w[32];
    memcpy(w, &p, sizeof(w));
    p.sum = svc_sum_host(w, 1, 29);
    memcpy(&s->in->post[k], &p, sizeof(p));
  } else {
    const SvcArgs a{in_len, cap, (uint32_t)target, 0u};
    memcpy(&s->in->args[k], &a, sizeof(a));
    if (in_len) memcpy(sl_in.in, source, in_len);
  }
  svc_wc_fence();                                                 // the request's bytes, then
  __atomic_store_n(&s->in->req[k], want, __ATOMIC_RELEASE);       // the doorbell
  __atomic_store_n(&s->box->req[k], want, __ATOMIC_RELAXED);      // (the host's copy; the same word without a BAR)
  svc_wc_fence();                                                 // on its way now
  __atomic_thread_fence(__ATOMIC_SEQ_CST);                        // ... and before alive is read
  s->ensure_running();
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t done = 0;
  // a short result (decode or compress) comes back in the slot's reply (service.h), ahead of
  // the done word: taken when both tags are this request's and the checksum
  // of its 108 data bytes matches
  SvcReply* rp =
      (uint32_t)k < kSvcPostSlots && !s->no_reply ? &s->box->reply[k] : nullptr;
  for (uint32_t spins = 1;; spins++) {
    if (rp && __atomic_load_n(&rp->tag0, __ATOMIC_ACQUIRE) == want) {
      SvcReply r;
      memcpy(&r, rp, sizeof(r));
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      uint32_t w[27];
      memcpy(w, r.data, sizeof(w));
      const uint32_t sum = svc_sum_host(w, 0, 27);
      if (r.tag0 == want && r.tag1 == want && r.sum == sum && r.rc >= 0 && r.rc <= (int32_t)kSvcInline &&
          r.rc <= (int32_t)cap) {
        *ret = r.rc;
        if (r.rc > 0) memcpy(dest, r.data, (size_t)r.rc);
        return true;
      }
    }
    done = __atomic_load_n(&s->box->done[k], __ATOMIC_ACQUIRE);
    // answered in the reply record (its bytes may still be on their way): keep
    // reading the reply
    if ((uint32_t)(done >> 32) == want && !(rp && ((uint32_t)done & 0xC0000000u) == kSvcReplied)) break;
    __builtin_ia32_pause();
    if ((spins & 1023u) == 0) {
      const auto waited = std::chrono::steady_clock::now() - t0;
      if (waited > std::chrono::microseconds(200)) s->ensure_running();   // it had just left: once more
      // past half a millisecond (a busy device, a service being relaunched)
      // the thread stops burning its core: it sleeps between checks
      if (waited > std::chrono::microseconds(500)) std::this_thread::sleep_for(std::chrono::microseconds(20));
      if (waited > std::chrono::seconds(1)) {
        // no answer (the device busy past a second?): this thread gives the
        // slot up for good (the wave may still write it) and launches
        t_lease.slot[2 * s->device + s->kind] = Lease{nullptr, -1};
        return false;
      }
    }
  }
  *ret = (int32_t)(uint32_t)done;
  if (*ret > 0) memcpy(dest, sl.out, (size_t)*ret);
#if KDB_SVC_DEBUG
  t_dbg_out = sl.out;
  t_dbg_done = done;
  t_dbg_box = s->box;
#endif
  return true;
}

}  // namespace

extern "C" {

int kdb_lz4_version(void) { return 10000; }

int kdb_lz4_service_stats(int device, uint32_t* launches, uint32_t* served, uint32_t* alive) {
  if (!launches || !served || !alive || device < 0) return KDB_LZ4_EINVAL;
  *launches = *served = *alive = 0;
  std::lock_guard<std::mutex> l(g_svc_mu);
  const std::vector<Service*>& v = services();
  for (int kind = 0; kind < 2; kind++)
    for (int w = 0; w < kSvcWavesMax; w++) {
      const size_t at = svc_index(device, kind, w);
      const Service* s = at < v.size() ? v[at] : nullptr;
      if (!s || !s->ok) continue;
      *launches += __atomic_load_n(&s->box->launches, __ATOMIC_ACQUIRE);
      *served += __atomic_load_n(&s->box->served, __ATOMIC_ACQUIRE);
      *alive += __atomic_load_n(&s->box->alive, __ATOMIC_ACQUIRE) != 0u ? 1u : 0u;   // (a generation)
    }
  return KDB_LZ4_OK;
}

int kdb_lz4_service_counters(int device, uint32_t* polls, uint32_t* from_post, uint32_t* replied) {
  if (!polls || !from_post || !replied || device < 0) return KDB_LZ4_EINVAL;
  *polls = *from_post = *replied = 0;
  std::lock_guard<std::mutex> l(g_svc_mu);
  const std::vector<Service*>& v = services();
  for (int kind = 0; kind < 2; kind++)
    for (int w = 0; w < kSvcWavesMax; w++) {
      const size_t at = svc_index(device, kind, w);
      const Service* s = at < v.size() ? v[at] : nullptr;
      if (!s || !s->ok) continue;
      *polls += __atomic_load_n(&s->box->polls, __ATOMIC_ACQUIRE);
      *from_post += __atomic_load_n(&s->box->inline_served, __ATOMIC_ACQUIRE);
      *replied += __atomic_load_n(&s->box->replied, __ATOMIC_ACQUIRE);
    }
  return KDB_LZ4_OK;
}

int kdb_lz4_device_count(int* count) {
  if (!count) return KDB_LZ4_EINVAL;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = e == hipSuccess ? n : 0;
  return e == hipSuccess ? KDB_LZ4_OK : KDB_LZ4_ENODEV;
}
// Binding a device runs its lane-order self-test (selftest.hip) at once, so a
// device the compressor cannot be exact on is reported here, not mid-batch.
int kdb_lz4_set_device(int device) {
  const int rc = hip_status(hipSetDevice(device));
  if (rc != KDB_LZ4_OK) return rc;
  const hipError_t e = lane_order_check();
  return e == hipErrorNotSupported ? KDB_LZ4_OK : hip_status(e);   // the failure shows at compress time
}
int kdb_lz4_selftest(int device, int* state, uint32_t* bad_lanes) {
  if (!state) return KDB_LZ4_EINVAL;
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return hip_status(e);
  if (device != cur && (e = hipSetDevice(device)) != hipSuccess) return hip_status(e);
  e = lane_order_check();
  const int rc = e == hipSuccess || e == hipErrorNotSupported ? KDB_LZ4_OK : hip_status(e);
  *state = lane_order_state(device, bad_lanes);
  if (device != cur) (void)hipSetDevice(cur);
  return rc;
}
int kdb_lz4_warmup(void) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_status(e);
  {
    static std::mutex mu;
    static std::unordered_map<int, bool> done;
    std::lock_guard<std::mutex> l(mu);
    if (done[dev]) return KDB_LZ4_OK;
    if ((e = lane_order_check()) != hipSuccess && e != hipErrorNotSupported) return hip_status(e);
    // one value per compress class (<= 4 KiB, the LDS-staged, in place, byU32)
    // as frames, and their decode: every kernel family's first launch
    const uint32_t lens[4] = {100u, 6000u, 20000u, 70000u};
    uint64_t src_off[4], dst_off[4], total_in = 0, total_out = 0;
    for (int i = 0; i < 4; i++) {
      src_off[i] = total_in;
      dst_off[i] = total_out;
      total_in += align16(lens[i] + 16);
      total_out += align16(8u + compress_bound(lens[i]) + 16);
    }
    uint8_t *d = nullptr, *meta = nullptr;
    hipStream_t st = nullptr;
    const size_t mbytes = 4 * (8 + 4 + 8 + 4 + 4 + 4 + 4);
    if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) == hipSuccess &&
        (e = hipMalloc(&d, total_in + total_out + total_in)) == hipSuccess &&
        (e = hipMalloc(&meta, mbytes + 256)) == hipSuccess && (e = hipMemsetAsync(d, 0x61, total_in, st)) == hipSuccess) {
      uint8_t h[mbytes + 256] = {};
      uint64_t* so = reinterpret_cast<uint64_t*>(h);
      uint32_t* sl = reinterpret_cast<uint32_t*>(h + 32);
      uint64_t* doff = reinterpret_cast<uint64_t*>(h + 48);
      uint32_t* cap = reinterpret_cast<uint32_t*>(h + 80);
      uint64_t* ooff = reinterpret_cast<uint64_t*>(h + 96);
      for (int i = 0; i < 4; i++) {
        so[i] = src_off[i];
        sl[i] = lens[i];
        doff[i] = total_in + dst_off[i];
        cap[i] = lens[i];
        ooff[i] = total_in + total_out + src_off[i];
      }
      uint32_t* flen = reinterpret_cast<uint32_t*>(meta + 128);
      int32_t* stat = reinterpret_cast<int32_t*>(meta + 144);
      uint32_t* olen = reinterpret_cast<uint32_t*>(meta + 160);
      if ((e = hipMemcpyAsync(meta, h, 128, hipMemcpyHostToDevice, st)) == hipSuccess)
        e = launch_compress(true, st, d, reinterpret_cast<uint64_t*>(meta), reinterpret_cast<uint32_t*>(meta + 32), 4,
                            0u, 70000u, d, reinterpret_cast<uint64_t*>(meta + 48), nullptr, flen, stat);
      // the frames' slots are read back as inputs of the same length class
      if (e == hipSuccess)
        e = launch_decompress(true, st, d, reinterpret_cast<uint64_t*>(meta + 48), flen, 4,
                              8u + compress_bound(70000u), 70000u, d, reinterpret_cast<uint64_t*>(meta + 96),
                              reinterpret_cast<uint32_t*>(meta + 80), nullptr, olen, stat);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    if (meta) (void)hipFree(meta);
    if (d) (void)hipFree(d);
    if (st) (void)hipStreamDestroy(st);
    if (e != hipSuccess) return hip_status(e);
    done[dev] = true;
  }
  return KDB_LZ4_OK;
}

int kdb_lz4_last_kernels(char* buf, uint64_t cap) {
  if (!buf || cap == 0) return KDB_LZ4_EINVAL;
  const char* s = launch_notes();
  const size_t n = strlen(s);
  const size_t k = n < cap - 1 ? n : (size_t)cap - 1;
  memcpy(buf, s, k);
  buf[k] = 0;
  return KDB_LZ4_OK;
}
#ifndef KDB_BUILD_ID
#define KDB_BUILD_ID "unstamped"
#endif
int kdb_lz4_build_id(char* buf, uint64_t cap) {
  if (!buf || cap == 0) return KDB_LZ4_EINVAL;
  const size_t n = strlen(KDB_BUILD_ID);
  const size_t k = n < cap - 1 ? n : (size_t)cap - 1;
  memcpy(buf, KDB_BUILD_ID, k);
  buf[k] = 0;
  return KDB_LZ4_OK;
}
int kdb_lz4_get_device(int* device) { return device ? hip_status(hipGetDevice(device)) : KDB_LZ4_EINVAL; }
int kdb_lz4_malloc(void** ptr, uint64_t bytes) {
  return ptr ? hip_status(hipMalloc(ptr, bytes ? bytes : 1)) : KDB_LZ4_EINVAL;
}
int kdb_lz4_free(void* ptr) { return hip_status(hipFree(ptr)); }
int kdb_lz4_host_alloc(void** ptr, uint64_t bytes) {
  return ptr ? hip_status(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault)) : KDB_LZ4_EINVAL;
}
int kdb_lz4_host_free(void* ptr) { return hip_status(hipHostFree(ptr)); }
int kdb_lz4_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream) {
  return hip_status(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
}
int kdb_lz4_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream) {
  return hip_status(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
}
int kdb_lz4_memcpy_d2d(void* dst, const void* src, uint64_t bytes, void* stream) {
  return hip_status(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
}
int kdb_lz4_memset(void* ptr, int value, uint64_t bytes, void* stream) {
  return hip_status(hipMemsetAsync(ptr, value, bytes, (hipStream_t)stream));
}
int kdb_lz4_stream_create(void** stream) {
  return stream ? hip_status(hipStreamCreateWithFlags((hipStream_t*)stream, hipStreamNonBlocking))
                : KDB_LZ4_EINVAL;
}
int kdb_lz4_stream_destroy(void* stream) { return hip_status(hipStreamDestroy((hipStream_t)stream)); }
int kdb_lz4_stream_sync(void* stream) { return hip_status(hipStreamSynchronize((hipStream_t)stream)); }
// Waits for the calling thread's device.  A resident service wave (service.h)
// counts as work in flight for hipDeviceSynchronize and would hold it for up
// to its idle time (2 ms) or lifetime (20 ms): the device's services are told
// to leave first (each serves what is already rung), and callers that ring
// meanwhile wait on the service's lock, then relaunch it after the sync.
int kdb_lz4_device_sync(void) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_status(e);
  std::vector<Service*> held;
  {
    std::lock_guard<std::mutex> l(g_svc_mu);
    for (int kind = 0; kind < 2; kind++)
      for (int w = 0; w < kSvcWavesMax; w++) {
        const size_t at = svc_index(dev, kind, w);
        Service* s = at < services().size() ? services()[at] : nullptr;
        if (s && s->ok) held.push_back(s);
      }
  }
  for (Service* s : held) {
    s->mu.lock();
    __atomic_store_n(&s->in->stop, 1u, __ATOMIC_SEQ_CST);
    svc_wc_fence();
  }
  e = hipDeviceSynchronize();
  for (Service* s : held) {
    __atomic_store_n(&s->in->stop, 0u, __ATOMIC_SEQ_CST);
    svc_wc_fence();
    s->mu.unlock();
  }
  return hip_status(e);
}
int kdb_lz4_service_seed_requests(uint32_t req, uint32_t reply_tag) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_status(e);
  std::vector<Service*> held;
  {
    std::lock_guard<std::mutex> l(g_svc_mu);
    for (int kind = 0; kind < 2; kind++)
      for (int w = 0; w < kSvcWavesMax; w++) {
        const size_t at = svc_index(dev, kind, w);
        Service* s = at < services().size() ? services()[at] : nullptr;
        if (s && s->ok) held.push_back(s);
      }
  }
  for (Service* s : held) {
    std::lock_guard<std::mutex> l(s->mu);
    __atomic_store_n(&s->in->stop, 1u, __ATOMIC_SEQ_CST);
    svc_wc_fence();
    e = hipStreamSynchronize(s->stream);   // the wave has left
    __atomic_store_n(&s->in->stop, 0u, __ATOMIC_SEQ_CST);
    if (e != hipSuccess) return hip_status(e);
    for (uint32_t k = 0; k < kSvcSlots; k++) {
      __atomic_store_n(&s->in->req[k], req, __ATOMIC_RELAXED);
      __atomic_store_n(&s->box->req[k], req, __ATOMIC_RELAXED);
      __atomic_store_n(&s->box->done[k], (uint64_t)req << 32, __ATOMIC_RELAXED);
      if (k < kSvcPostSlots) {
        SvcReply& r = s->box->reply[k];
        memset(&r, 0, sizeof(r));   // zero data: checksum 0
        r.tag0 = r.tag1 = reply_tag;
      }
    }
    svc_wc_fence();
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  return KDB_LZ4_OK;
}
int kdb_lz4_event_create(void** event) {
  return event ? hip_status(hipEventCreate((hipEvent_t*)event)) : KDB_LZ4_EINVAL;
}
int kdb_lz4_event_destroy(void* event) { return hip_status(hipEventDestroy((hipEvent_t)event)); }
int kdb_lz4_event_record(void* event, void* stream) {
  return hip_status(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
}
int kdb_lz4_event_sync(void* event) { return hip_status(hipEventSynchronize((hipEvent_t)event)); }
int kdb_lz4_stream_wait_event(void* stream, void* event) {
  return event ? hip_status(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0)) : KDB_LZ4_EINVAL;
}
int kdb_lz4_event_elapsed_ms(void* start, void* stop, float* ms) {
  return ms ? hip_status(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop)) : KDB_LZ4_EINVAL;
}

// ------------------------------------------------------------------ scalar
int kdb_lz4_compressBound(int isize) { return (int)compress_bound((uint32_t)isize); }

int kdb_lz4_compress_limitedOutput(const char* source, char* dest, int inputSize, int maxOutputSize) {
  if ((uint32_t)inputSize > kMaxInput) return 0;                 // lz4.cc:465
  if (maxOutputSize < 0) maxOutputSize = 0;
  int err = 0;
  ScalarCtx& c = scalar_ctx(&err);
  if (err) return 0;
  const uint32_t S = (uint32_t)inputSize;
  // The kernel never writes past the cap, and the cap never needs to exceed
  // the bound for the return value to be exact.
  const uint32_t bound = compress_bound(S);
  const uint32_t cap = (uint32_t)maxOutputSize < bound ? (uint32_t)maxOutputSize : bound;
  Meta m{};
  m.len = S;
  m.cap = (uint32_t)maxOutputSize;
  if (S <= 4096u && cap <= kSvcOutBytes && lane_order_ok() == hipSuccess) {   // the resident compress service
    int sret = 0;
    if (service_call(kSvcCompress, source, S, dest, cap, 0, &sret))
      return sret > 0 && sret != KDB_LZ4_VALUE_UNSUPPORTED ? sret : 0;
  }
  if (S <= kZeroCopyMax) {                       // zero-copy: [meta][in][out] in mapped host memory
    const size_t in_at = kMetaBytes, out_at = kMetaBytes + align16((size_t)S + 16);
    if (c.reserve(out_at + align16(cap + 16), 0) != KDB_LZ4_OK) return 0;
    m.src_off = in_at;
    m.dst_off = out_at;
    memcpy(c.host, &m, sizeof(m));
    if (S) memcpy(c.host + in_at, source, S);
    Meta* dm = reinterpret_cast<Meta*>(c.hdev);
    if (launch_compress(false, c.stream, c.hdev, &dm->src_off, &dm->len, 1, S, S, c.hdev, &dm->dst_off, &dm->cap,
                        nullptr, &dm->ret) != hipSuccess ||
        hipStreamSynchronize(c.stream) != hipSuccess)
      return c.failed(0);
    m = read_meta(c.host);
    if (m.ret > 0) memcpy(dest, c.host + out_at, (size_t)m.ret);
    return m.ret > 0 ? m.ret : 0;
  }
  // device staging: [meta][out][in]; one D2H of meta + the whole output slot
  const size_t out_at = kMetaBytes, in_at = kMetaBytes + align16((size_t)cap + 16);
  const size_t bytes = in_at + align16((size_t)S + 16);
  if (c.reserve(bytes, bytes) != KDB_LZ4_OK) return 0;
  m.src_off = in_at;
  m.dst_off = out_at;
  memcpy(c.host, &m, sizeof(m));
  memcpy(c.host + in_at, source, S);
  Meta* dm = reinterpret_cast<Meta*>(c.dev);
  if (hipMemcpyAsync(c.dev, c.host, kMetaBytes, hipMemcpyHostToDevice, c.stream) != hipSuccess ||
      hipMemcpyAsync(c.dev + in_at, c.host + in_at, S, hipMemcpyHostToDevice, c.stream) != hipSuccess ||
      launch_compress(false, c.stream, c.dev, &dm->src_off, &dm->len, 1, S, S, c.dev, &dm->dst_off, &dm->cap,
                      nullptr, &dm->ret) != hipSuccess ||
      hipMemcpyAsync(c.host, c.dev, in_at, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
      hipStreamSynchronize(c.stream) != hipSuccess)
    return c.failed(0);
  m = read_meta(c.host);
  if (m.ret > 0) memcpy(dest, c.host + out_at, (size_t)m.ret);
  return m.ret > 0 ? m.ret : 0;
}

int kdb_lz4_decompress_safe_partial(const char* source, char* dest, int compressedSize,
                                    int targetOutputSize, int maxDecompressedSize) {
  if (compressedSize < 0 || maxDecompressedSize < 0) return -1;
  int err = 0;
  ScalarCtx& c = scalar_ctx(&err);
  if (err) return -1;
  const uint32_t C = (uint32_t)compressedSize, O = (uint32_t)maxDecompressedSize;
  Meta m{};
  m.len = C;
  m.cap = O;
  m.target = (uint32_t)targetOutputSize;
  // the LDS-resident decoder's share (lz4_decompress.hip: output <= its split,
  // block <= that output's bound + a frame header)
  const bool zc = O <= kZeroCopyMax && C <= kZeroCopyMax + kZeroCopyMax / 255u + 24u;
#if KDB_SVC_DEBUG   // (diagnostic build: every service answer checked against a launch)
  static thread_local bool t_no_svc = false;
  if (zc && C <= kSvcMaxIn && O <= kSvcMaxOut && !t_no_svc) {
    int sret = 0;
    std::vector<char> mine((size_t)O + 1);
    if (service_call(kSvcDecode, source, C, mine.data(), O, targetOutputSize, &sret)) {
      const int r1 = sret == KDB_LZ4_VALUE_UNSUPPORTED ? -1 : sret;
      t_no_svc = true;
      const int r2 = kdb_lz4_decompress_safe_partial(source, dest, compressedSize, targetOutputSize, maxDecompressedSize);
      t_no_svc = false;
      size_t at = 0;
      if (r1 == r2 && r2 > 0) while (at < (size_t)r2 && mine[at] == dest[at]) at++;
      if (r1 != r2 || (r2 > 0 && at != (size_t)r2)) {
        const Lease ls = lease_of(0, kSvcDecode);
        const std::vector<char>& last = t_dbg_last;
        size_t nbad = 0, stale = 0, later = 0;
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        for (size_t j = 0; r2 > 0 && j < (size_t)r2; j++) {
          nbad += mine[j] != dest[j];
          stale += mine[j] != dest[j] && j < last.size() && mine[j] == last[j];
          later += t_dbg_out && (char)t_dbg_out[j] != dest[j];
        }
        fprintf(stderr,
                "SVCDBG slot %d: C %u O %u target %d: service %d launch %d, first diff %zu, %zu bytes differ, %zu "
                "of them the slot's previous output; after 2 ms the slot differs in %zu; done %llx alive %u served %u "
                "launches %u overlaps %u running %u\n",
                ls.slot, C, O, targetOutputSize, r1, r2, at, nbad, stale, later, (unsigned long long)t_dbg_done,
                t_dbg_box ? t_dbg_box->alive : 0u, t_dbg_box ? t_dbg_box->served : 0u,
                t_dbg_box ? t_dbg_box->launches : 0u, t_dbg_box ? t_dbg_box->pad[1] : 0u,
                t_dbg_box ? t_dbg_box->pad[0] : 0u);
      }
      if (r2 > 0) t_dbg_last.assign(dest, dest + r2);
      return r2;
    }
  }
#else
  if (zc && C <= kSvcMaxIn && O <= kSvcMaxOut) {   // the resident decode service (service.h)
    int sret = 0;
    if (service_call(kSvcDecode, source, C, dest, O, targetOutputSize, &sret))
      return sret == KDB_LZ4_VALUE_UNSUPPORTED ? -1 : sret;
  }
#endif
  if (zc) {                                      // zero-copy: [meta][in][out] in mapped host memory
    const size_t in_at = kMetaBytes, out_at = kMetaBytes + align16((size_t)C + 16);
    if (c.reserve(out_at + align16((size_t)O + 16), 0) != KDB_LZ4_OK) return -1;
    m.src_off = in_at;
    m.dst_off = out_at;
    memcpy(c.host, &m, sizeof(m));
    if (C) memcpy(c.host + in_at, source, C);
    Meta* dm = reinterpret_cast<Meta*>(c.hdev);
    if (launch_decompress(false, c.stream, c.hdev, &dm->src_off, &dm->len, 1, C, O, c.hdev, &dm->dst_off, &dm->cap,
                          &dm->target, &dm->out_len, &dm->ret) != hipSuccess ||
        hipStreamSynchronize(c.stream) != hipSuccess)
      return c.failed(-1);
    m = read_meta(c.host);
    if (m.ret == KDB_LZ4_VALUE_UNSUPPORTED) return -1;
    if (m.ret > 0) memcpy(dest, c.host + out_at, (size_t)m.ret);
    return m.ret;
  }
  const size_t out_at = kMetaBytes, in_at = kMetaBytes + align16((size_t)O + 16);
  const size_t bytes = in_at + align16((size_t)C + 16);
  if (c.reserve(bytes, bytes) != KDB_LZ4_OK) return -1;
  m.src_off = in_at;
  m.dst_off = out_at;
  memcpy(c.host, &m, sizeof(m));
  memcpy(c.host + in_at, source, C);
  Meta* dm = reinterpret_cast<Meta*>(c.dev);
  if (hipMemcpyAsync(c.dev, c.host, kMetaBytes, hipMemcpyHostToDevice, c.stream) != hipSuccess ||
      hipMemcpyAsync(c.dev + in_at, c.host + in_at, C, hipMemcpyHostToDevice, c.stream) != hipSuccess ||
      launch_decompress(false, c.stream, c.dev, &dm->src_off, &dm->len, 1, C, O, c.dev, &dm->dst_off, &dm->cap,
                        &dm->target, &dm->out_len, &dm->ret) != hipSuccess ||
      hipMemcpyAsync(c.host, c.dev, in_at, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
      hipStreamSynchronize(c.stream) != hipSuccess)
    return c.failed(-1);
  m = read_meta(c.host);
  if (m.ret == KDB_LZ4_VALUE_UNSUPPORTED) return -1;
  if (m.ret > 0) memcpy(dest, c.host + out_at, (size_t)m.ret);
  return m.ret;
}

// ------------------------------------------------------------------- batch
uint64_t kdb_lz4_frame_bound(uint32_t size) { return 8u + (uint64_t)compress_bound(size); }

int kdb_lz4_compress_blocks_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint32_t n, uint32_t max_len, uint8_t* dst,
                                  const uint64_t* dst_off, const uint32_t* dst_cap, int32_t* ret) {
  if (n == 0) return KDB_LZ4_OK;
  if (!src || !src_off || !src_len || !dst || !dst_off || !dst_cap || !ret) return KDB_LZ4_EINVAL;
  return hip_status(launch_compress(false, (hipStream_t)stream, src, src_off, src_len, n, 0u, max_len, dst,
                                    dst_off, dst_cap, nullptr, ret));
}

int kdb_lz4_decompress_blocks_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                    const uint32_t* in_len, uint32_t n, uint32_t max_in, uint32_t max_out,
                                    uint8_t* dst, const uint64_t* dst_off, const uint32_t* dst_cap,
                                    const uint32_t* target, int32_t* ret) {
  if (n == 0) return KDB_LZ4_OK;
  if (!src || !src_off || !in_len || !dst || !dst_off || !dst_cap || !ret) return KDB_LZ4_EINVAL;
  return hip_status(launch_decompress(false, (hipStream_t)stream, src, src_off, in_len, n, max_in, max_out,
                                      dst, dst_off, dst_cap, target, nullptr, ret));
}

int kdb_lz4_compress_frames_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint32_t n, uint32_t max_len, uint8_t* dst,
                                  const uint64_t* dst_off, uint32_t* frame_len, int32_t* status) {
  if (n == 0) return KDB_LZ4_OK;
  if (!src || !src_off || !src_len || !dst || !dst_off || !frame_len || !status) return KDB_LZ4_EINVAL;
  return hip_status(launch_compress(true, (hipStream_t)stream, src, src_off, src_len, n, 0u, max_len, dst,
                                    dst_off, nullptr, frame_len, status));
}

int kdb_lz4_decompress_frames_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                    const uint32_t* avail, uint32_t n, uint32_t max_in, uint32_t max_out,
                                    uint8_t* dst, const uint64_t* dst_off, const uint32_t* dst_cap,
                                    uint32_t* out_len, int32_t* status) {
  if (n == 0) return KDB_LZ4_OK;
  if (!src || !src_off || !avail || !dst || !dst_off || !dst_cap || !out_len || !status)
    return KDB_LZ4_EINVAL;
  return hip_status(launch_decompress(true, (hipStream_t)stream, src, src_off, avail, n, max_in, max_out,
                                      dst, dst_off, dst_cap, nullptr, out_len, status));
}

int kdb_lz4_gen_g1(uint8_t* dst, uint64_t first_piece, uint64_t npieces, uint32_t seed, void* stream) {
  if (!dst) return KDB_LZ4_EINVAL;
  return hip_status(launch_gen_g1(dst, first_piece, npieces, seed, (hipStream_t)stream));
}

// Link-time aliases with the reference's exact C names (algorithm/lz4.h:36-38,
// extern "C"), so an object built against lz4.h links against this library.
int LZ4_compressBound(int isize) { return kdb_lz4_compressBound(isize); }
int LZ4_compress_limitedOutput(const char* s, char* d, int n, int m) {
  return kdb_lz4_compress_limitedOutput(s, d, n, m);
}
int LZ4_decompress_safe_partial(const char* s, char* d, int c, int t, int m) {
  return kdb_lz4_decompress_safe_partial(s, d, c, t, m);
}

}  // extern "C"
