// kingdb_amd/csrc/flush_hook.cc -- the write-buffer flush hook
// (kingdb_include/cache/lz4_flush.h).  Compiled by the
// KingDB build that applies the hook (oracle/kingdb_hook.py, INTEGRATION.md
// level 4), like compressor.cc.
//
// One pipeline per write buffer:
//   client threads   LZ4FlushDefer: the PutPartValidSize call goes into the
//                    intake (key, chunk, offsets, thread id) under a ticket
//   worker thread    takes the intake in ticket order, in batches (at most
//                    kBatchBytes / kBatchParts, or whatever came within
//                    kBatchAge, or everything when a flush asks), and runs each
//                    batch through kdb_flush_parts_batch (include/kdb_flush.h):
//                    frames, the disable rule, offsets, size_value_compressed
//                    and the running CRC32C on the GPU, each client thread's
//                    state (the reference's ThreadStorage slots,
//                    /root/reference/interface/database.cc:159-257) carried
//                    from batch to batch; the results wait per ticket
//   flush thread     LZ4FlushOrders: waits for the tickets of the buffer being
//                    flushed (usually long done: the worker runs while the
//                    buffer fills), then completes each order in place
// The reference's put contract (database.cc:128-276): a put it acknowledges is
// stored, and a put it refuses gets its IOError at that very call.
//   * A GPU batch that fails is retried once on a fresh stream and fresh
//     staging; if that fails too, the batch is completed on the host in the
//     reference's own disabled-compression form (:199-209: 8 zero bytes + the
//     raw chunk for the part that switches, the raw chunk for the value's later
//     parts; offsets, size_value_compressed and the CRC32C as the reference
//     computes them on that branch) -- no LZ4 runs on the host, and no
//     acknowledged put is lost.  Each thread's carried state follows it, so the
//     next batch (GPU again) continues from it.
//   * The only IOErrors PutPartValidSize can return (:189, :261-266) need a part
//     outside the regular shape -- a value's parts in order, contiguous from
//     offset 0, non-empty (see Pipeline::regular) -- so such a part waits for
//     its own result inside LZ4FlushDefer and returns the reference's status
//     there, before its order reaches the buffer; regular parts cannot fail and
//     return at once.
#include "cache/lz4_flush.h"

#include "algorithm/compressor.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "../../include/kdb_flush.h"
#include "../../include/kdb_lz4.h"
#include "util/logger.h"

#ifdef KDB_LZ4_HANG_DUMP
// Debug builds only (-DKDB_LZ4_HANG_DUMP, CPU model): SIGUSR1 makes every
// thread print its stack (SIGUSR2 to each task), for a run that stopped.
#include <dirent.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>
static void kdb_dump_one(int) {
  void* b[64];
  const int n = backtrace(b, 64);
  char hdr[64];
  const int l = snprintf(hdr, sizeof hdr, "---- thread %ld\n", (long)syscall(SYS_gettid));
  (void)!write(2, hdr, l);
  backtrace_symbols_fd(b, n, 2);
}
static void kdb_dump_all(int) {
  DIR* d = opendir("/proc/self/task");
  if (!d) return;
  while (struct dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    syscall(SYS_tgkill, getpid(), atol(e->d_name), SIGUSR2);
    usleep(20000);
  }
  closedir(d);
}
#endif

namespace kdb {

namespace {

constexpr uint64_t kBatchBytes = 8ull << 20;   // raw bytes that start a batch at once
constexpr size_t kBatchParts = 65536;           // parts that start a batch at once
constexpr auto kBatchAge = std::chrono::microseconds(1000);   // oldest waiting part

inline uint64_t a256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// Pinned host + device staging of one pipeline, kept across batches, and
// handed to the next pipeline when a database closes (StagingPool): pinned
// allocations cost milliseconds, a Close should not pay to free them.
struct Staging {
  void* host = nullptr;
  void* dev = nullptr;
  void* stream = nullptr;
  uint64_t hcap = 0, dcap = 0;
  ~Staging() { release(); }
  void release() {
    if (host) kdb_lz4_host_free(host);
    if (dev) kdb_lz4_free(dev);
    if (stream) kdb_lz4_stream_destroy(stream);
    host = dev = stream = nullptr;
    hcap = dcap = 0;
  }
  // after a failure: drain what the stream still has queued, or forget the
  // buffers (leaked, not freed: a kernel may still write them)
  void drop() {
    if (stream && kdb_lz4_stream_sync(stream) == KDB_LZ4_OK) {
      release();
      return;
    }
    host = dev = stream = nullptr;
    hcap = dcap = 0;
  }
  static uint64_t grow(uint64_t cap, uint64_t want) {
    uint64_t c = cap ? cap : (16ull << 20);
    while (c < want) c *= 2;
    return c;
  }
  bool reserve(uint64_t hbytes, uint64_t dbytes) {
    if (!stream && kdb_lz4_stream_create(&stream) != KDB_LZ4_OK) return false;
    if (hbytes > hcap) {
      if (host) kdb_lz4_host_free(host);
      host = nullptr;
      const uint64_t c = grow(hcap, hbytes);
      hcap = 0;
      if (kdb_lz4_host_alloc(&host, c) != KDB_LZ4_OK) return false;
      hcap = c;
    }
    if (dbytes > dcap) {
      if (dev) kdb_lz4_free(dev);
      dev = nullptr;
      const uint64_t c = grow(dcap, dbytes);
      dcap = 0;
      if (kdb_lz4_malloc(&dev, c) != KDB_LZ4_OK) return false;
      dcap = c;
    }
    return true;
  }
};

class StagingPool {
 public:
  static StagingPool& get() {
    static StagingPool* p = new StagingPool();   // never destroyed: HIP may be gone at exit
    return *p;
  }
  void put(int device, Staging& s) {
    if (!s.stream) return;
    std::lock_guard<std::mutex> l(mu_);
    if (free_.size() >= 4) return;                 // (then s frees its own)
    free_.push_back(Entry{device, s.host, s.dev, s.stream, s.hcap, s.dcap});
    s.host = s.dev = s.stream = nullptr;
    s.hcap = s.dcap = 0;
  }
  void take(int device, Staging& s) {
    std::lock_guard<std::mutex> l(mu_);
    for (size_t i = 0; i < free_.size(); i++)
      if (free_[i].device == device) {
        const Entry e = free_[i];
        free_.erase(free_.begin() + (long)i);
        s.host = e.host;
        s.dev = e.dev;
        s.stream = e.stream;
        s.hcap = e.hcap;
        s.dcap = e.dcap;
        return;
      }
  }

 private:
  struct Entry {
    int device;
    void *host, *dev, *stream;
    uint64_t hcap, dcap;
  };
  std::mutex mu_;
  std::vector<Entry> free_;
};

// One queued PutPartValidSize call.  Its key and (small) chunk bytes were
// copied by the client thread into that thread's intake arena (below), so the
// queue holds plain pointers: no shared_ptr of the caller's ByteArrays is
// copied here and released on the worker (a cross-core cache-line transfer
// per put), and the caller's own value buffer is freed on the caller's thread,
// as in the reference.  A chunk over kInlineMax bytes is referenced instead
// (hold), not copied.
struct Intake {
  std::thread::id tid;
  const char* kp;
  const char* cp;
  uint64_t kn, cn;
  uint64_t offset_chunk, size_value;
  ByteArray hold;
  uint64_t ticket;
};
constexpr uint64_t kInlineMax = 4096;          // chunks copied into the intake arena
constexpr uint64_t kArenaBytes = 1ull << 20;    // one intake arena block

// A client thread's current intake arena block.  Order chunks are slices of
// it (CompressorLZ4::Slice), so the block lives while any of them sits in the
// write buffer; every batch that has intakes in it also holds it (Pipeline::
// intake_blocks_), so the worker can read it whatever the orders do.
struct IntakeArena {
  uint64_t owner = 0;        // Pipeline::id_
  size_t lane = 0;           // the lane it was last registered with
  uint64_t gen = ~0ull;      // that lane's batch generation then
  ByteArray blk;
  char* base = nullptr;
  uint64_t used = 0, cap = 0;
};
thread_local IntakeArena t_arena;
// A client thread's per-pipeline state (Pipeline::thread_pipe): the shape of
// its current value (Pipeline::regular) and its lane (Pipeline::lane_of).
struct ThreadPipe {
  struct Track {
    bool open = false;       // the thread's last part left its value unfinished
    uint64_t end = 0, size_value = 0;
  } track;
  struct LaneOf {
    size_t lane;
    uint64_t bytes;
  } lane{0, 0};
  bool lane_set = false;
};
std::atomic<uint64_t> g_pipeline_ids{1};
// ids of the pipelines alive now: a client thread's per-pipeline records
// (Pipeline::thread_pipe) of closed databases are dropped against it
std::mutex g_live_mu;
std::unordered_set<uint64_t> g_live_ids;
// KDB_LZ4_FLUSH_STATS: when WriteBuffer::WritePart accounted this thread's last
// deferred chunk (its lock and buffer-full wait come after that point)
thread_local std::chrono::steady_clock::time_point t_accounted;
thread_local bool t_accounted_set = false;
std::atomic<uint64_t> g_after_account_max_ns{0};
const bool g_stats_on = [] {
  const char* e = getenv("KDB_LZ4_FLUSH_STATS");
  return e && *e && *e != '0';
}();

struct Result {
  ByteArray chunk_final;   // KDB_FLUSH_FRAME / KDB_FLUSH_DISABLED: a slice of the batch's arena
  uint64_t occ = 0, svc = 0;
  uint32_t crc = 0;
  uint8_t mode = KDB_FLUSH_RAW;
  int8_t status = 0;       // -1: PutPartValidSize returns IOError (mode FAILED: :189, else :261-266)
  bool ready = false;      // the lane that took the part has published it
  bool consumed = false;
};

// database.cc's two IOError statuses of PutPartValidSize
Status put_status(const Result& r) {
  if (r.mode == KDB_FLUSH_FAILED) return Status::IOError("LZ4_compress_limitedOutput() failed");   // compressor.cc:33
  log::emerg("Database::PutPartValidSize()", "Error: write was attempted outside of the allocated memory.");
  return Status::IOError("Prevented write to occur outside of the allocated memory.");                // :264-265
}

// KDB_LZ4_FLUSH_INJECT=<first>:<count> -- test knob: GPU batch attempts
// first .. first+count-1 (counted from 1) fail as a failed
// kdb_flush_parts_batch would (tests/test_kingdb_dropin.py).
struct Inject {
  uint64_t first = 0, count = 0;
  Inject() {
    const char* e = getenv("KDB_LZ4_FLUSH_INJECT");
    if (!e || !*e) return;
    char* end = nullptr;
    first = strtoull(e, &end, 10);
    count = end && *end == ':' ? strtoull(end + 1, nullptr, 10) : 1;
  }
  bool fails(uint64_t attempt) const { return first && attempt >= first && attempt - first < count; }
};

using Clock = std::chrono::steady_clock;
inline double ms_since(Clock::time_point t) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
}

// KDB_LZ4_FLUSH_STATS=1: where a pipeline's time went, printed to stderr when
// it stops (tools/write_path_cmp.py --stats).
struct Stats {
  bool on = false;
  uint64_t flushes = 0, orders = 0, waits = 0;
  double wait_ms = 0, complete_ms = 0;
  // the longest single wait / complete() call, and the longest gap between
  // one complete() ending and the next starting (the rest of a flush pass)
  double max_wait_ms = 0, max_complete_ms = 0, max_between_ms = 0;
  Clock::time_point last_complete_end{};
  bool completed_once = false;
  // timeline (ms since the pipeline started): each complete() call's start,
  // duration, orders and whether the flush pass is a sync one, and where the
  // client's longest gap between puts began
  struct Pass { double at, ms; size_t orders; bool sync; };
  std::vector<Pass> passes;
  Clock::time_point born = Clock::now();
  Stats() {
    const char* e = getenv("KDB_LZ4_FLUSH_STATS");
    on = e && *e && *e != '0';
  }
};

// One device's share of a pipeline: a worker thread bound to the device, its
// intake, staging and stream, and the carried PutPartValidSize state of the
// client threads whose parts it takes.  A client thread's parts go to one
// lane at a time; it moves to the next lane only at a value's first part with
// bytes, where the reference resets every piece of that state
// (database.cc:159-162, 177-179, 252-255), so no state crosses lanes.
struct Lane {
  int device = 0;
  size_t index = 0;
  std::thread worker;
  std::condition_variable cv_work;          // (with Pipeline::mu_)
  // intake: client threads and this lane's worker, under Pipeline::mu_
  std::vector<Intake> intake;
  std::vector<ByteArray> intake_blocks;     // the arena blocks intake's bytes live in
  uint64_t gen = 0;                         // batches taken so far
  uint64_t intake_bytes = 0;
  Clock::time_point intake_since;
  bool drain = false;
  // worker only
  std::unordered_map<std::thread::id, kdb_flush_state> state;
  Staging stg;
  std::atomic<int> phase{0};                // 0 waiting for intake, 1 batch, 3 dropping results
  // stats (worker; read after it joined)
  uint64_t batches = 0, parts = 0, raw_bytes = 0;
  double gpu_ms = 0, stage_ms = 0, results_ms = 0, init_ms = 0, first_batch_ms = 0;
};
// bytes a client thread sends to one lane before it moves on (at a value's
// first part), so even one writer spreads its batches over the devices
constexpr uint64_t kLaneSpan = 2ull << 20;

class Pipeline {
 public:
  explicit Pipeline(int device) : device_(device) {
    {
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live_ids.insert(id_);
    }
    // the lanes: this thread's device (the one the caller bound with
    // kdb_lz4_set_device) only, by default -- in a deployment of one process
    // per GPU no process touches another's device; KDB_LZ4_FLUSH_DEVICES=<n>
    // opts in to n lanes, this device first, then the next visible ones
    int count = 1;
    if (kdb_lz4_device_count(&count) != KDB_LZ4_OK || count < 1) count = 1;
    const char* cap = getenv("KDB_LZ4_FLUSH_DEVICES");
    const long want = cap && *cap ? strtol(cap, nullptr, 10) : 1;
    const int n = (int)std::max(1L, std::min<long>(count, want));
    for (int k = 0; k < n; k++) {
      lanes_.emplace_back(new Lane());
      lanes_.back()->device = (device + k) % count;
      lanes_.back()->index = (size_t)k;
    }
    for (auto& L : lanes_) L->worker = std::thread(&Pipeline::run, this, L.get());
    // KDB_LZ4_FLUSH_WATCH=<s>: a diagnostic thread prints the pipeline's state
    // every <s> seconds (tickets issued and processed, intake, worker phase,
    // a flush waiting), so a run that stops making progress shows where
    const char* w = getenv("KDB_LZ4_FLUSH_WATCH");
    const long ws = w ? strtol(w, nullptr, 10) : 0;
    if (ws > 0) watch_ = std::thread(&Pipeline::watch, this, ws);
  }
  ~Pipeline() {
    {
      std::lock_guard<std::mutex> l(g_live_mu);
      g_live_ids.erase(id_);
    }
    const Clock::time_point t0 = Clock::now();
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    for (auto& L : lanes_) L->cv_work.notify_all();
    cv_done_.notify_all();
    for (auto& L : lanes_) L->worker.join();
    if (watch_.joinable()) watch_.join();
    Lane sum;
    for (auto& L : lanes_) {
      sum.batches += L->batches;
      sum.parts += L->parts;
      sum.raw_bytes += L->raw_bytes;
      sum.gpu_ms += L->gpu_ms;
      sum.stage_ms += L->stage_ms;
      sum.results_ms += L->results_ms;
      sum.init_ms = std::max(sum.init_ms, L->init_ms);
      if (L->index == 0) sum.first_batch_ms = L->first_batch_ms;
    }
    if (stats_.on)
      fprintf(stderr,
              "lz4_flush_stats batches %llu parts %llu raw_bytes %llu stage_ms %.2f gpu_ms %.2f results_ms %.2f "
              "flushes %llu orders %llu waits %llu wait_ms %.2f complete_ms %.2f stop_ms %.2f defer_ms %.2f "
              "client_stalls %llu client_stall_ms %.2f client_max_gap_ms %.2f init_ms %.2f first_batch_ms %.2f "
              "max_after_account_ms %.2f max_wait_ms %.2f max_complete_ms %.2f max_between_ms %.2f\n",
              (unsigned long long)sum.batches, (unsigned long long)sum.parts,
              (unsigned long long)sum.raw_bytes, sum.stage_ms, sum.gpu_ms, sum.results_ms,
              (unsigned long long)stats_.flushes, (unsigned long long)stats_.orders, (unsigned long long)stats_.waits,
              stats_.wait_ms, stats_.complete_ms, ms_since(t0), defer_ns_.load() / 1e6,
              (unsigned long long)stalls_.load(), stall_ns_.load() / 1e6, stall_max_ns_.load() / 1e6, sum.init_ms,
              sum.first_batch_ms, g_after_account_max_ns.load() / 1e6, stats_.max_wait_ms, stats_.max_complete_ms,
              stats_.max_between_ms);
    if (stats_.on) {
      fprintf(stderr, "lz4_flush_lanes %zu", lanes_.size());
      for (auto& L : lanes_)
        fprintf(stderr, " | lane %zu device %d batches %llu parts %llu raw_bytes %llu gpu_ms %.2f", L->index, L->device,
                (unsigned long long)L->batches, (unsigned long long)L->parts, (unsigned long long)L->raw_bytes,
                L->gpu_ms);
      fprintf(stderr, "\n");
    }
    if (stats_.on)
      fprintf(stderr, "lz4_flush_contract settled_parts %llu refused_parts %llu host_batches %llu host_parts %llu\n",
              (unsigned long long)settles_.load(), (unsigned long long)refused_.load(),
              (unsigned long long)host_batches_.load(), (unsigned long long)host_parts_.load());
    if (stats_.on) {
      fprintf(stderr, "lz4_flush_timeline client_max_gap_at_ms %.2f", stall_max_at_ns_.load() / 1e6);
      for (const Stats::Pass& q : stats_.passes)
        fprintf(stderr, " | pass at %.2f ms %.2f orders %zu sync %d", q.at, q.ms, q.orders, (int)q.sync);
      fprintf(stderr, "\n");
    }
  }

  Status defer(ByteArray& key, ByteArray& chunk, uint64_t offset_chunk, uint64_t size_value, uint32_t* ticket,
               ByteArray* staged) {
    bool kick;
    const Clock::time_point t0 = stats_.on ? Clock::now() : Clock::time_point();
    if (stats_.on) {
      // the client's time between two of its puts: gaps over 1 ms are stalls
      // outside the hook (a write buffer that blocks, the allocator, ...)
      thread_local Clock::time_point t_last;
      thread_local const Pipeline* t_owner = nullptr;
      if (t_owner == this) {
        const uint64_t gap = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t0 - t_last).count();
        if (gap > 1000000u) {
          stall_ns_.fetch_add(gap, std::memory_order_relaxed);
          stalls_.fetch_add(1, std::memory_order_relaxed);
        }
        uint64_t m = stall_max_ns_.load(std::memory_order_relaxed);
        while (gap > m && !stall_max_ns_.compare_exchange_weak(m, gap, std::memory_order_relaxed)) {}
        if (gap > m)
          stall_max_at_ns_.store(
              (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_last - stats_.born).count(),
              std::memory_order_relaxed);
      }
      t_owner = this;
      t_last = t0;
      if (t_accounted_set) {
        const uint64_t g = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t0 - t_accounted).count();
        uint64_t mx = g_after_account_max_ns.load(std::memory_order_relaxed);
        while (g > mx && !g_after_account_max_ns.compare_exchange_weak(mx, g, std::memory_order_relaxed)) {}
      }
    }
    const uint64_t kn = key.size(), cn = chunk.size();
    const bool inline_chunk = cn <= kInlineMax;
    const uint64_t need = kn + (inline_chunk ? cn : 0);
    IntakeArena& a = t_arena;
    if (a.owner != id_ || a.used + need > a.cap) {
      const uint64_t cap = std::max(kArenaBytes, need);
      char* p = new char[cap];
      a.blk = NewShallowCopyByteArray(p, cap);
      a.base = p;
      a.used = 0;
      a.cap = cap;
      a.owner = id_;
      a.gen = ~0ull;
    }
    char* kp = a.base + a.used;
    memcpy(kp, key.data(), kn);
    const char* cp;
    if (inline_chunk) {
      memcpy(kp + kn, chunk.data(), cn);
      cp = kp + kn;
      *staged = CompressorLZ4::Slice(a.blk, a.used + kn, cn);
    } else {
      cp = chunk.data();
      *staged = chunk;
    }
    a.used += need;
    const bool settle = !regular(offset_chunk, cn, size_value);
    Lane& L = *lanes_[lane_of(offset_chunk, cn)];
    uint64_t mine;
    {
      std::lock_guard<std::mutex> l(mu_);
      mine = next_ticket_;
      *ticket = (uint32_t)next_ticket_++;
      if (L.intake.empty()) L.intake_since = Clock::now();
      if (a.lane != L.index || a.gen != L.gen) {
        L.intake_blocks.push_back(a.blk);
        a.lane = L.index;
        a.gen = L.gen;
      }
      L.intake.push_back(Intake{std::this_thread::get_id(), kp, cp, kn, cn, offset_chunk, size_value,
                                inline_chunk ? ByteArray() : chunk, mine});
      L.intake_bytes += cn;
      kick = L.intake_bytes >= kBatchBytes || L.intake.size() >= kBatchParts;
    }
    if (kick) L.cv_work.notify_one();
    Status s = Status::OK();
    if (settle) s = settle_part(L, mine);
    if (stats_.on) defer_ns_.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count(),
                                       std::memory_order_relaxed);
    return s;
  }

  // Whether this client thread's part has the regular shape, in which
  // PutPartValidSize cannot fail: a value's first part (offset 0, bytes), or
  // the next part of the value this thread's last part belongs to (same
  // size_value, contiguous offset, bytes); an empty value (no bytes, size 0).
  // Why nothing else is needed (database.cc:143-266, per thread): a first part
  // with bytes resets the state (:159-162, :177-179); while compression stays
  // on, a frame F <= chunk + 8 (compressor.cc:40-48) is kept only if the
  // value's raw rest + 8 still fits behind it (:197-200), so by induction
  // o + (size_value - offset) + 8 <= size_value + padding before each part, F
  // never exceeds space_left (no unsigned wrap at :200), and neither a kept
  // frame nor the part that switches (chunk + 8) nor the raw parts after it
  // -- contiguous, so they add up to the value's rest -- pass :262; Compress
  // fails (:189) only above LZ4_MAX_INPUT_SIZE.  Any other part (a gap, an
  // overlap, parts of two values interleaved on one thread, an empty chunk in
  // a value, a part after the value's end) is settled synchronously.
  bool regular(uint64_t offset_chunk, uint64_t cn, uint64_t size_value) {
    ThreadPipe::Track& t = thread_pipe().track;
    const bool bytes = cn > 0 && cn <= 0x7E000000ull;
    bool ok;
    if (offset_chunk == 0 && bytes) {
      ok = true;
      t.end = cn;
      t.size_value = size_value;
    } else if (t.open && bytes && offset_chunk == t.end && size_value == t.size_value) {
      ok = true;
      t.end += cn;
    } else {
      ok = offset_chunk == 0 && cn == 0 && size_value == 0;
      t.end = 0;
    }
    t.open = ok && t.end < size_value;
    return ok;
  }

  // The lane this client thread's part goes to (see Lane): the thread keeps
  // its lane until it has sent it kLaneSpan bytes, and moves on only at a
  // value's first part with bytes.
  size_t lane_of(uint64_t offset_chunk, uint64_t cn) {
    ThreadPipe& tp = thread_pipe();
    ThreadPipe::LaneOf& t = tp.lane;
    if (!tp.lane_set) {
      t = ThreadPipe::LaneOf{next_lane_.fetch_add(1, std::memory_order_relaxed) % lanes_.size(), 0};
      tp.lane_set = true;
    }
    if (lanes_.size() > 1 && offset_chunk == 0 && cn > 0 && t.bytes >= kLaneSpan) {
      t.lane = next_lane_.fetch_add(1, std::memory_order_relaxed) % lanes_.size();
      t.bytes = 0;
    }
    t.bytes += cn;
    return t.lane;
  }

  // This client thread's record for THIS pipeline (one per database: the
  // reference keeps PutPartValidSize's state per Database and per thread, and
  // a thread may interleave the parts of values in two databases).  Keyed by
  // the pipeline id in a thread_local map, with the last pipeline cached, so
  // switching databases never resets the other's lane or value tracking.
  ThreadPipe& thread_pipe() {
    thread_local uint64_t last_id = 0;
    thread_local ThreadPipe* last = nullptr;
    if (last_id == id_ && last) return *last;
    thread_local std::unordered_map<uint64_t, ThreadPipe> all;
    if (all.find(id_) == all.end() && !all.empty()) {
      // a thread that outlives many databases keeps records of the open ones only
      std::lock_guard<std::mutex> l(g_live_mu);
      for (auto it = all.begin(); it != all.end();) it = g_live_ids.count(it->first) ? std::next(it) : all.erase(it);
    }
    last = &all[id_];      // node-based: the reference stays valid across inserts
    last_id = id_;
    return *last;
  }

  // An irregular part waits for its own result (its lane is asked to take
  // the intake at once) and returns PutPartValidSize's status; a refused
  // part's result is dropped here, as its order never reaches the buffer.
  Status settle_part(Lane& L, uint64_t mine) {
    settles_.fetch_add(1, std::memory_order_relaxed);
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (processed_ <= mine) {
        L.drain = true;
        L.cv_work.notify_one();
        cv_done_.wait(lk, [&] { return processed_ > mine; });
      }
    }
    Result r0;
    {
      std::lock_guard<std::mutex> l(res_mu_);
      const uint64_t at = mine - res_base_;   // not consumed (no order holds it yet), so still queued
      if (at >= res_.size() || !res_[at].ready || res_[at].status == 0) return Status::OK();
      r0.mode = res_[at].mode;
      cancelled_.insert((uint32_t)mine);
    }
    refused_.fetch_add(1, std::memory_order_relaxed);
    return put_status(r0);
  }

  void cancel(uint32_t ticket) {
    std::lock_guard<std::mutex> l(res_mu_);
    cancelled_.insert(ticket);
  }

  void complete(std::vector<Order>& orders);

  // bytes the write buffer accounts for a deferred chunk of `raw` bytes: what
  // its frame is expected to take, at the compressed/raw ratio of the last
  // batch (the reference accounts the compressed chunk, write_buffer.cc:170,
  // which sets its flush cadence and its rate limiter's input)
  uint64_t accounted(uint64_t raw) const {
    const uint64_t r = ratio_q16_.load(std::memory_order_relaxed);
    const uint64_t a = (raw * r) >> 16;
    return a ? a : 1;
  }

 private:
  void run(Lane* L);
  void watch(long seconds);
  void drop_consumed();
  void process(Lane& L, std::vector<Intake>& batch);
  int gpu_batch(Lane& L, std::vector<Intake>& batch, std::vector<Result>& out);
  void host_batch(Lane& L, std::vector<Intake>& batch, std::vector<Result>& out);

  // the 64-bit ticket of an order's 32 bits (outstanding tickets span < 2^32)
  uint64_t full_ticket(uint32_t t) const { return res_base_ + (uint32_t)(t - (uint32_t)res_base_); }

  const int device_;
  const uint64_t id_ = g_pipeline_ids.fetch_add(1);
  std::vector<std::unique_ptr<Lane>> lanes_;
  std::atomic<size_t> next_lane_{0};
  std::thread watch_;
  std::atomic<uint64_t> complete_waits_for_{0};   // a flush waiting for this ticket (0: none)
  // tickets (client threads, lanes, flush thread)
  std::mutex mu_;
  std::condition_variable cv_done_;
  uint64_t next_ticket_ = 1;
  uint64_t processed_ = 1;           // tickets below have results
  bool stop_ = false, garbage_ = false;
  // results, by ticket (lanes fill them, in any order; the flush thread consumes)
  std::mutex res_mu_;
  std::deque<Result> res_;
  uint64_t res_base_ = 1;            // ticket of res_.front()
  uint64_t ready_below_ = 1;         // tickets below are published
  std::unordered_set<uint32_t> cancelled_;
  Inject inject_;
  // KDB_LZ4_FLUSH_MAX_PARTS=<n> -- test knob: at most n parts per GPU batch, so
  // a small stream's multipart values straddle batches (tests/test_hook_contract.py)
  const size_t max_parts_ = [] {
    const char* e = getenv("KDB_LZ4_FLUSH_MAX_PARTS");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
  }();
  std::atomic<uint64_t> attempts_{0};
  Stats stats_;
  std::atomic<uint64_t> ratio_q16_{1u << 16};
  std::atomic<uint64_t> defer_ns_{0};           // client threads' time in defer() (stats only)
  std::atomic<uint64_t> settles_{0}, refused_{0};   // irregular parts settled in defer(), and refused there
  std::atomic<uint64_t> host_batches_{0}, host_parts_{0};
  std::atomic<uint64_t> gpu_batches_{0};   // batches completed on the host (GPU failed twice)
  std::atomic<uint64_t> stall_ns_{0}, stalls_{0}, stall_max_ns_{0}, stall_max_at_ns_{0};   // client gaps > 1 ms between puts   // accounted / raw bytes of the last batch, x 2^16
};

void Pipeline::run(Lane* Lp) {
  Lane& L = *Lp;
  const Clock::time_point t_init = Clock::now();
  kdb_lz4_set_device(L.device);
  (void)kdb_lz4_warmup();   // this device's first launches, once per device
  StagingPool::get().take(L.device, L.stg);
  // the first batch's staging (pinned host + device) is allocated here, while
  // the database opens, not under the first puts: until a batch completes,
  // deferred chunks are accounted at their raw size (LZ4FlushAccount), and a
  // slow first batch had let 1 M 100-byte puts fill the write buffer on that
  // prior and block on its flush (client_embedded)
  if (!L.stg.host) (void)L.stg.reserve(16ull << 20, 16ull << 20);
  L.init_ms = ms_since(t_init);
  std::vector<Intake> batch;
  std::vector<ByteArray> blocks;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      for (;;) {
        if (L.index == 0 && garbage_) {   // (lane 0 frees the consumed results)
          garbage_ = false;
          lk.unlock();
          L.phase.store(3, std::memory_order_relaxed);
          drop_consumed();
          L.phase.store(0, std::memory_order_relaxed);
          lk.lock();
          continue;
        }
        if (L.intake.empty()) {
          L.drain = false;
          if (stop_) {
            StagingPool::get().put(L.device, L.stg);
            return;
          }
          L.cv_work.wait(lk);
          continue;
        }
        if (stop_ || L.drain || L.intake_bytes >= kBatchBytes || L.intake.size() >= kBatchParts ||
            Clock::now() - L.intake_since >= kBatchAge)
          break;
        L.cv_work.wait_until(lk, L.intake_since + kBatchAge);
      }
      if (max_parts_ && L.intake.size() > max_parts_) {   // (test knob: the rest stays queued)
        batch.assign(std::make_move_iterator(L.intake.begin()),
                     std::make_move_iterator(L.intake.begin() + (long)max_parts_));
        L.intake.erase(L.intake.begin(), L.intake.begin() + (long)max_parts_);
        blocks = L.intake_blocks;                          // (the rest's arena blocks stay registered too)
        L.intake_bytes = 0;
        for (const Intake& e : L.intake) L.intake_bytes += e.cn;
        L.intake_since = Clock::now();
      } else {
        batch.swap(L.intake);
        blocks.swap(L.intake_blocks);
        L.intake_bytes = 0;
      }
      L.gen++;
    }
    L.phase.store(1, std::memory_order_relaxed);
    process(L, batch);   // publishes the results, then processed_
    L.phase.store(0, std::memory_order_relaxed);
    batch.clear();
    blocks.clear();
  }
}

void Pipeline::watch(long seconds) {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(seconds);
    if (cv_done_.wait_until(lk, until, [&] { return stop_; })) break;
    fprintf(stderr, "lz4_flush_watch pipeline %llu tickets_issued %llu processed_below %llu host_batches %llu "
            "flush_waits_for %llu batches %llu",
            (unsigned long long)id_, (unsigned long long)next_ticket_, (unsigned long long)processed_,
            (unsigned long long)host_batches_.load(), (unsigned long long)complete_waits_for_.load(),
            (unsigned long long)gpu_batches_.load());
    for (auto& L : lanes_)
      fprintf(stderr, " | lane %zu device %d intake %zu blocks %zu drain %d phase %d", L->index, L->device,
              L->intake.size(), L->intake_blocks.size(), (int)L->drain, L->phase.load());
    fprintf(stderr, "\n");
  }
}

void Pipeline::process(Lane& L, std::vector<Intake>& batch) {
  std::vector<Result> out(batch.size());
  int rc = gpu_batch(L, batch, out);
  if (rc != KDB_LZ4_OK) {   // once more, on a fresh stream and fresh staging
    log::emerg("LZ4FlushPipeline", "GPU batch of %zu parts failed (%d); retrying", batch.size(), rc);
    L.stg.drop();
    rc = gpu_batch(L, batch, out);
  }
  if (rc != KDB_LZ4_OK) {
    log::emerg("LZ4FlushPipeline", "GPU batch failed twice (%d): %zu parts stored uncompressed", rc, batch.size());
    L.stg.drop();
    for (Result& r : out) r = Result();
    host_batch(L, batch, out);
  }
  // publish by ticket (lanes finish in any order); processed_ is the lowest
  // ticket any lane still holds
  uint64_t w;
  {
    std::lock_guard<std::mutex> l(res_mu_);
    for (size_t i = 0; i < batch.size(); i++) {
      const uint64_t at = batch[i].ticket - res_base_;
      if (at >= res_.size()) res_.resize(at + 1);
      res_[at] = std::move(out[i]);
      res_[at].ready = true;
    }
    while (ready_below_ - res_base_ < res_.size() && res_[ready_below_ - res_base_].ready) ready_below_++;
    w = ready_below_;
  }
  {
    std::lock_guard<std::mutex> l(mu_);
    if (w > processed_) processed_ = w;
  }
  cv_done_.notify_all();
}

// A batch the GPU could not run (twice), completed on the host exactly as
// PutPartValidSize completes parts whose compression is switched off
// (database.cc:143-266 with the :199 test taken): the first compressed part of
// a value becomes 8 zero bytes + its chunk (:200-208), later parts stay raw
// (:164-174), offsets / size_value_compressed / the CRC32C follow those
// branches (:237-257) and the :261-266 check is made.  Every acknowledged put
// is stored (readable by the reference's UncompressByteArray, compressor.cc:
// 173-180, 213-245); each thread's carried state is the reference's after the
// same calls, so a later GPU batch continues from it.  No LZ4 on the host;
// the CRC32C is the drop-in's host Crc32cExtend (compressor.cc).
void Pipeline::host_batch(Lane& L, std::vector<Intake>& batch, std::vector<Result>& out) {
  const uint32_t m = (uint32_t)batch.size();
  uint64_t dis_bytes = 0;
  for (const Intake& e : batch) dis_bytes += e.cn + 8;
  char* a = dis_bytes ? new char[dis_bytes] : nullptr;
  ByteArray arena = a ? NewShallowCopyByteArray(a, dis_bytes) : ByteArray();
  uint64_t at = 0;
  for (uint32_t i = 0; i < m; i++) {
    const Intake& e = batch[i];
    Result& r = out[i];
    kdb_flush_state& S = L.state[e.tid];
    const uint64_t csz = e.cn, off = e.offset_chunk, V = e.size_value;
    const uint64_t pad = (V / 65536u + 1u) * 8u;                     // format.h:63-71
    const bool first = off == 0, last = csz + off == V, do_comp = csz != 0;
    uint64_t o = off, size = csz;
    r.mode = KDB_FLUSH_RAW;
    if (first) { S.enabled = 1u; S.ts_offset = 0; }                   // :159-162
    if (!S.enabled) { o = S.ts_offset; S.ts_offset = o + csz; }        // :164-171
    if (do_comp && S.enabled) {
      if (first) S.comp_total = 0;                                    // :177-179
      o = S.comp_total;                                               // :182
      if (csz > 0x7E000000ull) {                                      // :185-189 (LZ4_MAX_INPUT_SIZE)
        r.mode = KDB_FLUSH_FAILED;
        r.status = -1;
        r.occ = o;
        continue;
      }
      size = csz + 8u;                                                // :199-209, the test taken
      S.enabled = 0u;
      S.ts_offset = S.comp_total + size;
      r.mode = KDB_FLUSH_DISABLED;
      memset(a + at, 0, 8);
      memcpy(a + at + 8, e.cp, csz);
      r.chunk_final = CompressorLZ4::Slice(arena, at, size);
      at += size;
    }
    if (do_comp && last) r.svc = S.enabled ? S.comp_total : (first ? S.ts_offset : o + csz);   // :237-248
    if (first) S.crc = Crc32cExtend(0u, e.kp, e.kn);                 // :251-255
    if (r.mode == KDB_FLUSH_DISABLED) {
      static const char zeros[8] = {0};
      S.crc = Crc32cExtend(S.crc, zeros, 8);
    }
    S.crc = Crc32cExtend(S.crc, e.cp, csz);                          // :256
    r.crc = last ? S.crc : 0u;                                        // :257
    r.occ = o;
    if (o + size > V + (do_comp ? pad : 0u)) r.status = -1;           // :261-266
  }
  host_batches_.fetch_add(1, std::memory_order_relaxed);
  host_parts_.fetch_add(m, std::memory_order_relaxed);
}

// The batch through the GPU: layout (segments, runs), staging, one
// kdb_flush_parts_batch, results.  0 or a KDB_LZ4_E* code.
int Pipeline::gpu_batch(Lane& L, std::vector<Intake>& batch, std::vector<Result>& out) {
  const Clock::time_point t_start = Clock::now();
  if (inject_.fails(attempts_.fetch_add(1) + 1)) return KDB_LZ4_EHIP;
  const uint32_t m = (uint32_t)batch.size();
  // ---- layout: a segment is one thread's consecutive parts of one value; a
  // run is one thread's segments whose policy state chains (a new run starts
  // at a first part with bytes: everything resets there, database.cc:159-179)
  struct Cur {
    uint32_t run, seg;
  };
  std::unordered_map<std::thread::id, Cur> cur;
  std::vector<uint32_t> part_seg(m), seg_run, seg_head;   // seg_head: the segment's first entry
  std::vector<std::thread::id> run_tid;
  std::vector<kdb_flush_state> carry;
  std::thread::id last_tid;
  auto last_it = cur.end();
  for (uint32_t i = 0; i < m; i++) {
    const Intake& e = batch[i];
    // (consecutive parts mostly come from one thread: skip the hash lookup)
    auto it = (last_it != cur.end() && e.tid == last_tid) ? last_it : cur.find(e.tid);
    const bool fresh = e.offset_chunk == 0;
    if (it == cur.end() || (fresh && e.cn > 0)) {
      const bool seen = it != cur.end();
      const uint32_t r = (uint32_t)run_tid.size();
      run_tid.push_back(e.tid);
      kdb_flush_state s{};
      if (!seen) {
        auto st = L.state.find(e.tid);
        if (st != L.state.end()) s = st->second;
      }
      carry.push_back(s);
      const uint32_t sg = (uint32_t)seg_run.size();
      seg_run.push_back(r);
      seg_head.push_back(i);
      if (seen) it->second = Cur{r, sg};
      else it = cur.emplace(e.tid, Cur{r, sg}).first;
      part_seg[i] = sg;
    } else if (fresh) {
      const uint32_t sg = (uint32_t)seg_run.size();
      seg_run.push_back(it->second.run);
      seg_head.push_back(i);
      it->second.seg = sg;
      part_seg[i] = sg;
    } else {
      part_seg[i] = it->second.seg;
    }
    last_tid = e.tid;
    last_it = it;
  }
  const uint32_t nseg = (uint32_t)seg_run.size(), nruns = (uint32_t)run_tid.size();
  // order: segments grouped by run, parts grouped by segment (both stable)
  std::vector<uint32_t> seg_order(nseg), seg_pos(nseg), run_first(nruns + 1, 0), seg_first(nseg + 1, 0),
      perm(m);
  const bool identity = nseg == m && nruns == m;   // every part a value of its own: nothing moves
  if (identity) {
    for (uint32_t i = 0; i <= m; i++) run_first[i] = seg_first[i] = i;
    for (uint32_t i = 0; i < m; i++) perm[i] = seg_order[i] = seg_pos[i] = i;
  } else {
    for (uint32_t s = 0; s < nseg; s++) run_first[seg_run[s] + 1]++;
    for (uint32_t r = 0; r < nruns; r++) run_first[r + 1] += run_first[r];
    std::vector<uint32_t> fill(run_first.begin(), run_first.end() - 1);
    for (uint32_t s = 0; s < nseg; s++) {
      const uint32_t at = fill[seg_run[s]]++;
      seg_order[at] = s;
      seg_pos[s] = at;
    }
    for (uint32_t i = 0; i < m; i++) seg_first[seg_pos[part_seg[i]] + 1]++;
    for (uint32_t s = 0; s < nseg; s++) seg_first[s + 1] += seg_first[s];
    std::vector<uint32_t> pf(seg_first.begin(), seg_first.end() - 1);
    for (uint32_t i = 0; i < m; i++) perm[pf[seg_pos[part_seg[i]]]++] = i;
  }
  // ---- staging: host [meta | keys | chunks], device [same | scratch | outputs | frames]
  uint64_t key_bytes = 0, raw_bytes = 0, frame_cap = 0;
  uint32_t max_chunk = 0;
  for (uint32_t s = 0; s < nseg; s++) key_bytes += batch[seg_head[seg_order[s]]].kn;
  for (uint32_t i = 0; i < m; i++) {
    const uint64_t c = batch[i].cn;
    if (c > 0x7E000000ull) return KDB_LZ4_EUNSUPPORTED;
    raw_bytes += c;
    frame_cap += (8 + kdb_lz4_compressBound((int)c) + 15) & ~15ull;
    if (c > max_chunk) max_chunk = (uint32_t)c;
  }
  const uint64_t o_key_off = 0, o_key_len = o_key_off + a256(8ull * nseg), o_chunk_off = o_key_len + a256(4ull * nseg),
                 o_chunk_len = o_chunk_off + a256(8ull * m), o_offset = o_chunk_len + a256(4ull * m),
                 o_size = o_offset + a256(8ull * m), o_seg_first = o_size + a256(8ull * m),
                 o_run_first = o_seg_first + a256(4ull * (nseg + 1)),
                 o_carry = o_run_first + a256(4ull * (nruns + 1)),
                 o_keys = o_carry + a256(sizeof(kdb_flush_state) * nruns), o_chunks = o_keys + a256(key_bytes),
                 in_bytes = o_chunks + a256(raw_bytes + 64);
  const uint64_t scratch = kdb_flush_scratch_bytes(m, nseg, raw_bytes);
  const uint64_t d_scratch = in_bytes, d_out = d_scratch + a256(scratch);
  const uint64_t p_parts = 0, p_carry = a256(sizeof(kdb_flush_part) * m),
                 p_total = p_carry + a256(sizeof(kdb_flush_state) * nruns), out_bytes = p_total + 256;
  const uint64_t d_frames = d_out + out_bytes, dev_bytes = d_frames + a256(frame_cap);
  const uint64_t h_out = in_bytes, h_frames = h_out + out_bytes, host_bytes = h_frames + a256(frame_cap);
  if (!L.stg.reserve(host_bytes, dev_bytes)) return KDB_LZ4_EHIP;
  char* hb = static_cast<char*>(L.stg.host);
  char* db = static_cast<char*>(L.stg.dev);
  auto H64 = [&](uint64_t o) { return reinterpret_cast<uint64_t*>(hb + o); };
  auto H32 = [&](uint64_t o) { return reinterpret_cast<uint32_t*>(hb + o); };
  {
    uint64_t ko = 0, co = 0;
    for (uint32_t s = 0; s < nseg; s++) {
      const Intake& k = batch[seg_head[seg_order[s]]];
      H64(o_key_off)[s] = ko;
      H32(o_key_len)[s] = (uint32_t)k.kn;
      memcpy(hb + o_keys + ko, k.kp, k.kn);
      ko += k.kn;
    }
    for (uint32_t q = 0; q < m; q++) {
      const Intake& e = batch[perm[q]];
      const uint64_t c = e.cn;
      H64(o_chunk_off)[q] = co;
      H32(o_chunk_len)[q] = (uint32_t)c;
      H64(o_offset)[q] = e.offset_chunk;
      H64(o_size)[q] = e.size_value;
      memcpy(hb + o_chunks + co, e.cp, c);
      co += c;
    }
    memcpy(H32(o_seg_first), seg_first.data(), 4ull * (nseg + 1));
    memcpy(H32(o_run_first), run_first.data(), 4ull * (nruns + 1));
    memcpy(hb + o_carry, carry.data(), sizeof(kdb_flush_state) * nruns);
  }
  const double t_stage = ms_since(t_start);
  const Clock::time_point t_gpu = Clock::now();
  void* st = L.stg.stream;
  auto D8 = [&](uint64_t o) { return reinterpret_cast<uint8_t*>(db + o); };
  auto D32 = [&](uint64_t o) { return reinterpret_cast<uint32_t*>(db + o); };
  auto D64 = [&](uint64_t o) { return reinterpret_cast<uint64_t*>(db + o); };
  int rc = kdb_lz4_memcpy_h2d(db, hb, in_bytes, st);
  if (!rc)
    rc = kdb_flush_parts_batch(st, D8(o_keys), D64(o_key_off), D32(o_key_len), D8(o_chunks), D64(o_chunk_off),
                               D32(o_chunk_len), D64(o_offset), D64(o_size), D32(o_seg_first), D32(o_run_first),
                               reinterpret_cast<const kdb_flush_state*>(db + o_carry), m, nseg, nruns, max_chunk,
                               D8(d_scratch), scratch, raw_bytes,
                               reinterpret_cast<kdb_flush_part*>(db + d_out + p_parts),
                               reinterpret_cast<kdb_flush_state*>(db + d_out + p_carry), D8(d_frames),
                               D64(d_out + p_total));
  if (!rc) rc = kdb_lz4_memcpy_d2h(hb + h_out, db + d_out, out_bytes, st);
  if (!rc) rc = kdb_lz4_stream_sync(st);
  if (rc) return rc;
  const uint64_t total = *H64(h_out + p_total);
  if (total > frame_cap) return KDB_LZ4_EHIP;
  if (total) {
    rc = kdb_lz4_memcpy_d2h(hb + h_frames, db + d_frames, total, st);
    if (!rc) rc = kdb_lz4_stream_sync(st);
    if (rc) return rc;
  }
  const double t_gpu_ms = ms_since(t_gpu);
  const Clock::time_point t_res = Clock::now();
  // ---- results, in ticket order
  // one arena per batch: the packed frames, then the disabled-compression forms
  const kdb_flush_part* parts = reinterpret_cast<const kdb_flush_part*>(hb + h_out + p_parts);
  const kdb_flush_state* cout = reinterpret_cast<const kdb_flush_state*>(hb + h_out + p_carry);
  uint64_t disabled_bytes = 0;
  for (uint32_t q = 0; q < m; q++)
    if (parts[q].status == 0 && parts[q].mode == KDB_FLUSH_DISABLED) disabled_bytes += parts[q].size;
  ByteArray arena;
  if (total + disabled_bytes) {
    char* a = new char[total + disabled_bytes];
    memcpy(a, hb + h_frames, total);
    arena = NewShallowCopyByteArray(a, total + disabled_bytes);
  }
  uint64_t dis_at = total;
  for (uint32_t q = 0; q < m; q++) {
    const kdb_flush_part& P = parts[q];
    Intake& e = batch[perm[q]];
    Result& r = out[perm[q]];
    r.occ = P.occ;
    r.svc = P.svc;
    r.crc = P.crc;
    r.mode = (uint8_t)P.mode;
    r.status = P.status == 0 ? 0 : -1;
    if (r.status) continue;
    if (P.mode == KDB_FLUSH_FRAME) {
      if (P.frame_at + P.size > total) return KDB_LZ4_EHIP;
      r.chunk_final = CompressorLZ4::Slice(arena, P.frame_at, P.size);
    } else if (P.mode == KDB_FLUSH_DISABLED) {             // database.cc:201-206
      char* b = arena.data() + dis_at;
      memset(b, 0, 8);
      memcpy(b + 8, e.cp, P.size - 8);
      r.chunk_final = CompressorLZ4::Slice(arena, dis_at, P.size);
      dis_at += P.size;
    }
  }
  // each thread's state after its last run of the batch
  for (uint32_t r = 0; r < nruns; r++) L.state[run_tid[r]] = cout[r];
  {  // what the batch's chunks take in the buffer once final, per raw byte
    uint64_t acc = 0;
    for (uint32_t q = 0; q < m; q++)
      acc += parts[q].status == 0 && parts[q].mode != KDB_FLUSH_RAW ? parts[q].size : batch[perm[q]].cn;
    if (raw_bytes) ratio_q16_.store(std::min<uint64_t>((acc << 16) / raw_bytes, 1u << 17), std::memory_order_relaxed);
  }
  if (L.batches == 0) L.first_batch_ms = ms_since(t_start);
  L.batches++;
  gpu_batches_.fetch_add(1, std::memory_order_relaxed);   // (read by watch(), which holds mu_ only)
  L.parts += m;
  L.raw_bytes += raw_bytes;
  L.stage_ms += t_stage;
  L.gpu_ms += t_gpu_ms;
  L.results_ms += ms_since(t_res);
  return KDB_LZ4_OK;
}

void Pipeline::complete(std::vector<Order>& orders) {
  const Clock::time_point t0 = Clock::now();
  // the newest ticket among the orders (every Put order here was deferred)
  bool any = false;
  uint64_t newest = 0;
  {
    std::lock_guard<std::mutex> l(res_mu_);
    for (const Order& o : orders) {
      if (o.type != OrderType::Put) continue;
      const uint64_t t = full_ticket(o.crc32);
      if (!any || t > newest) newest = t;
      any = true;
    }
  }
  if (!any) return;
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (processed_ <= newest) {
      const Clock::time_point tw = Clock::now();
      for (auto& L : lanes_) {
        L->drain = true;
        L->cv_work.notify_one();
      }
      complete_waits_for_.store(newest, std::memory_order_relaxed);
      cv_done_.wait(lk, [&] { return processed_ > newest; });
      complete_waits_for_.store(0, std::memory_order_relaxed);
      stats_.waits++;
      const double w = ms_since(tw);
      stats_.wait_ms += w;
      stats_.max_wait_ms = std::max(stats_.max_wait_ms, w);
    }
  }
  std::lock_guard<std::mutex> l(res_mu_);
  size_t dropped = 0;
  std::vector<char> drop;
  for (size_t i = 0; i < orders.size(); i++) {
    Order& o = orders[i];
    if (o.type != OrderType::Put) continue;
    const uint64_t at = full_ticket(o.crc32) - res_base_;
    Result* rp = at < res_.size() ? &res_[at] : nullptr;
    if (!rp || rp->status != 0) {   // (no result: not an order of this pipeline; never written)
      if (drop.empty()) drop.assign(orders.size(), 0);
      drop[i] = 1;
      dropped++;
      if (rp) rp->consumed = true;
      continue;
    }
    Result& r = *rp;
    r.consumed = true;
    if (r.mode == KDB_FLUSH_FRAME || r.mode == KDB_FLUSH_DISABLED) o.chunk = r.chunk_final;
    o.offset_chunk = r.occ;
    o.size_value_compressed = r.svc;
    o.crc32 = r.crc;
  }
  if (dropped) {
    size_t w = 0;
    for (size_t i = 0; i < orders.size(); i++) {
      if (drop[i]) continue;
      if (w != i) orders[w] = orders[i];
      w++;
    }
    orders.resize(w);
    log::emerg("LZ4FlushOrders()", "%zu orders dropped: their PutPartValidSize failed", dropped);
  }
  stats_.flushes++;
  stats_.orders += orders.size();
  const double c = ms_since(t0);
  stats_.complete_ms += c;
  stats_.max_complete_ms = std::max(stats_.max_complete_ms, c);
  if (stats_.completed_once)
    stats_.max_between_ms = std::max(
        stats_.max_between_ms,
        std::chrono::duration<double, std::milli>(t0 - stats_.last_complete_end).count());
  stats_.last_complete_end = Clock::now();
  stats_.completed_once = true;
  if (stats_.on && stats_.passes.size() < 64)
    stats_.passes.push_back({std::chrono::duration<double, std::milli>(t0 - stats_.born).count(), c, orders.size(),
                             !orders.empty() && orders[0].write_options.sync});
  // the consumed results are dropped by lane 0's worker (drop_consumed), off this thread
  {
    std::lock_guard<std::mutex> l2(mu_);
    garbage_ = true;
  }
  lanes_[0]->cv_work.notify_one();
}

// Lane 0's worker: drops the consumed (or cancelled) results at the front,
// freeing their buffers here rather than on the flush thread.  A cancelled
// ticket a lane has not published yet stays (its slot is still to be filled).
void Pipeline::drop_consumed() {
  std::deque<Result> dead;
  {
    std::lock_guard<std::mutex> l(res_mu_);
    size_t k = 0;
    while (k < res_.size()) {
      const uint32_t t = (uint32_t)(res_base_ + k);
      auto c = cancelled_.find(t);
      if (!res_[k].ready || (!res_[k].consumed && c == cancelled_.end())) break;
      if (c != cancelled_.end()) cancelled_.erase(c);
      k++;
    }
    if (k == 0) return;
    dead.insert(dead.end(), std::make_move_iterator(res_.begin()), std::make_move_iterator(res_.begin() + (long)k));
    res_.erase(res_.begin(), res_.begin() + (long)k);
    res_base_ += k;
  }
}

// ---- registry: one pipeline per write buffer
// LZ4FlushDefer -> WriteBuffer::WritePart on the same client thread: the
// bytes to account for the chunk it just queued (LZ4FlushAccount)
thread_local bool t_account_set = false;
thread_local uint64_t t_account_raw = 0, t_account = 0;

std::mutex g_mu;
std::unordered_map<const void*, std::shared_ptr<Pipeline>> g_pipes;
std::unordered_set<const void*> g_closed;

std::shared_ptr<Pipeline> pipeline_of(const void* wb, bool create) {
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_pipes.find(wb);
  if (it != g_pipes.end()) return it->second;
  if (!create || g_closed.count(wb)) return nullptr;
  int dev = 0;
  if (kdb_lz4_get_device(&dev) != KDB_LZ4_OK) dev = 0;
  auto p = std::make_shared<Pipeline>(dev);
  g_pipes.emplace(wb, p);
  return p;
}

}  // namespace

Status LZ4FlushDefer(const void* wb, const DatabaseOptions& db_options, ByteArray& key, ByteArray& chunk,
                     uint64_t offset_chunk, uint64_t size_value, uint32_t* ticket, ByteArray* staged_chunk) {
  (void)db_options;
  thread_local const void* t_wb = nullptr;
  thread_local std::weak_ptr<Pipeline> t_pipe;
  std::shared_ptr<Pipeline> p = t_wb == wb ? t_pipe.lock() : nullptr;
  if (!p) {
    p = pipeline_of(wb, true);
    if (!p) return Status::IOError("Cannot handle request: WriteBuffer is closing");
    t_wb = wb;
    t_pipe = p;
  }
  const Status s = p->defer(key, chunk, offset_chunk, size_value, ticket, staged_chunk);
  if (s.IsOK()) {
    t_account_raw = chunk.size();
    t_account = p->accounted(chunk.size());
    t_account_set = true;
  }
  return s;
}

uint64_t LZ4FlushAccount(uint64_t chunk_size) {
  const bool mine = t_account_set && t_account_raw == chunk_size;
  t_account_set = false;
  if (mine && g_stats_on) {
    t_accounted = std::chrono::steady_clock::now();
    t_accounted_set = true;
  }
  return mine ? t_account : chunk_size;
}

void LZ4FlushCancel(const void* wb, uint32_t ticket) {
  t_account_set = false;
  std::shared_ptr<Pipeline> p = pipeline_of(wb, false);
  if (p) p->cancel(ticket);
}

void LZ4FlushOrders(const void* wb, const DatabaseOptions& db_options, std::vector<Order>& orders) {
  if (!LZ4FlushDeferrable(db_options) || orders.empty()) return;
  std::shared_ptr<Pipeline> p = pipeline_of(wb, false);
  if (p) p->complete(orders);
}

// The write buffer's constructor (the thread opening the database): the entry
// for this address is the new buffer's from now on, whatever a closed buffer
// at the same address left in g_closed.
void LZ4FlushOpen(const void* wb, const DatabaseOptions& db_options) {
  {
    std::lock_guard<std::mutex> l(g_mu);
    g_closed.erase(wb);
  }
  if (LZ4FlushDeferrable(db_options)) pipeline_of(wb, true);
}

LZ4FlushScope::LZ4FlushScope(const void* wb, const DatabaseOptions& db_options) : wb_(wb) {
#ifdef KDB_LZ4_HANG_DUMP
  signal(SIGUSR2, kdb_dump_one);
  signal(SIGUSR1, kdb_dump_all);
#endif
  // test knob: a ProcessingLoop thread that the scheduler starts late (the
  // put loop of the database that was just opened runs meanwhile)
  if (const char* d = getenv("KDB_LZ4_FLUSH_SCOPE_DELAY_US"))
    std::this_thread::sleep_for(std::chrono::microseconds(strtoul(d, nullptr, 10)));
  {
    std::lock_guard<std::mutex> l(g_mu);
    g_closed.erase(wb);
  }
  if (LZ4FlushDeferrable(db_options)) pipeline_of(wb, true);
}

LZ4FlushScope::~LZ4FlushScope() {
  std::shared_ptr<Pipeline> p;
  {
    std::lock_guard<std::mutex> l(g_mu);
    auto it = g_pipes.find(wb_);
    if (it != g_pipes.end()) {
      p = it->second;
      g_pipes.erase(it);
    }
    g_closed.insert(wb_);
  }
  p.reset();   // the last reference stops and joins the worker (a client still in defer() holds its own)
}

}  // namespace kdb
