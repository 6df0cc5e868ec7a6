// tests/cpp/abi_cpu_model.cc -- TEST INFRASTRUCTURE ONLY: a CPU model of the
// parts of the C ABI (include/kdb_lz4.h, kdb_flush.h, kdb_put.h) that the host
// code above it calls -- kingdb_amd/csrc/compressor.cc (the drop-in),
// flush_hook.cc and read_hook.cc (the KingDB hooks).  It lets those host
// sources run under ThreadSanitizer and AddressSanitizer in this GPU-less
// container (tests/test_sanitizers.py): the sanitizers check the host code's
// threads, locks, staging buffers and ByteArray lifetimes, not the kernels.
//
// Every computation is the oracle's restatement (oracle/lz4_oracle.c, linked
// beside this file); "device" and pinned memory are plain heap memory, copies
// are synchronous, a stream is a token.  This file is never linked into
// libkdb_lz4.so or anything that ships: the product has no CPU path.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "kdb_flush.h"
#include "kdb_lz4.h"
#include "kdb_put.h"

extern "C" {
int orc_compress_bound(int isize);
int orc_compress_limited(const uint8_t* src, uint8_t* dst, int isize, int max_out);
int orc_decompress_safe_partial(const uint8_t* src, uint8_t* dst, int csize, int target, int max_out);
int64_t orc_frame_compress(const uint8_t* src, uint64_t n, uint8_t* frame);
int orc_frame_uncompress(const uint8_t* frame, uint8_t* out, uint64_t* out_n, uint64_t* frame_n);
typedef struct orc_put_state { uint64_t ts_offset, comp_total; uint32_t enabled, crc; } orc_put_state;
int orc_put_part(orc_put_state* st, const uint8_t* key, uint32_t klen, const uint8_t* chunk, uint64_t csz,
                 uint64_t offset_chunk, uint64_t size_value, uint8_t* fin, uint32_t* mode, uint64_t* occ_out,
                 uint64_t* fsz_out, uint64_t* svc_out, uint32_t* crc_out);
int orc_get_value(const uint8_t* stored, uint64_t avail, uint64_t svc, uint64_t size, uint32_t checksum,
                  uint32_t checksum_initial, int verify, uint8_t* out, uint64_t* out_n);
}

static_assert(sizeof(orc_put_state) == sizeof(kdb_flush_state), "state layouts");

extern "C" {

// Devices: KDB_LZ4_CPU_MODEL_DEVICES=<n> models n of them (default 1).  A
// stream belongs to the device bound when it was created, and a batch entry
// point called on a thread bound to another device fails (KDB_LZ4_EINVAL) --
// the HIP rule the host code must keep (a stream is used on its own device).
// KDB_LZ4_CPU_MODEL_STATS=1 prints the batches each device ran at exit.
static thread_local int t_device = 0;
struct ModelStream {
  int device;
};
static std::atomic<unsigned long long> g_batches[64];
static int model_devices() {
  static const int n = [] {
    const char* e = getenv("KDB_LZ4_CPU_MODEL_DEVICES");
    const int v = e && *e ? atoi(e) : 1;
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }();
  return n;
}
static struct ModelStats {
  ~ModelStats() {
    const char* e = getenv("KDB_LZ4_CPU_MODEL_STATS");
    if (!e || !*e || *e == '0') return;
    fprintf(stderr, "cpu_model_batches");
    for (int d = 0; d < model_devices(); d++) fprintf(stderr, " device%d %llu", d, g_batches[d].load());
    fprintf(stderr, "\n");
  }
} g_model_stats;
// the stream's device is the calling thread's (counted per device), or EINVAL
static int on_device(void* stream) {
  if (!stream) return KDB_LZ4_OK;
  const int d = static_cast<ModelStream*>(stream)->device;
  if (d != t_device) return KDB_LZ4_EINVAL;
  g_batches[d].fetch_add(1, std::memory_order_relaxed);
  return KDB_LZ4_OK;
}

int kdb_lz4_device_count(int* count) {
  *count = model_devices();
  return KDB_LZ4_OK;
}
int kdb_lz4_set_device(int device) {
  if (device < 0 || device >= model_devices()) return KDB_LZ4_ENODEV;
  t_device = device;
  return KDB_LZ4_OK;
}
int kdb_lz4_get_device(int* device) {
  *device = t_device;
  return KDB_LZ4_OK;
}
int kdb_lz4_warmup(void) { return KDB_LZ4_OK; }
int kdb_lz4_malloc(void** p, uint64_t n) {
  *p = malloc(n ? n : 1);
  return *p ? KDB_LZ4_OK : KDB_LZ4_EHIP;
}
int kdb_lz4_free(void* p) {
  free(p);
  return KDB_LZ4_OK;
}
int kdb_lz4_host_alloc(void** p, uint64_t n) { return kdb_lz4_malloc(p, n); }
int kdb_lz4_host_free(void* p) { return kdb_lz4_free(p); }
int kdb_lz4_memcpy_h2d(void* d, const void* s, uint64_t n, void*) {
  memcpy(d, s, n);
  return KDB_LZ4_OK;
}
int kdb_lz4_memcpy_d2h(void* d, const void* s, uint64_t n, void*) {
  memcpy(d, s, n);
  return KDB_LZ4_OK;
}
int kdb_lz4_stream_create(void** s) {
  *s = new ModelStream{t_device};
  return KDB_LZ4_OK;
}
int kdb_lz4_stream_destroy(void* s) {
  delete static_cast<ModelStream*>(s);
  return KDB_LZ4_OK;
}
int kdb_lz4_stream_sync(void*) { return KDB_LZ4_OK; }

int kdb_lz4_compressBound(int isize) { return orc_compress_bound(isize); }
int kdb_lz4_compress_limitedOutput(const char* s, char* d, int n, int m) {
  return orc_compress_limited((const uint8_t*)s, (uint8_t*)d, n, m);
}
int kdb_lz4_decompress_safe_partial(const char* s, char* d, int c, int t, int m) {
  return orc_decompress_safe_partial((const uint8_t*)s, (uint8_t*)d, c, t, m);
}
uint64_t kdb_lz4_frame_bound(uint32_t size) { return 8u + (uint64_t)orc_compress_bound((int)size); }

int kdb_lz4_compress_frames_batch(void* stream, const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                  uint32_t n, uint32_t, uint8_t* dst, const uint64_t* dst_off, uint32_t* frame_len,
                                  int32_t* status) {
  if (on_device(stream) != KDB_LZ4_OK) return KDB_LZ4_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    const int64_t f = orc_frame_compress(src + src_off[i], src_len[i], dst + dst_off[i]);
    frame_len[i] = f < 0 ? 0u : (uint32_t)f;
    status[i] = f < 0 ? -1 : 0;
  }
  return KDB_LZ4_OK;
}

int kdb_lz4_decompress_frames_batch(void* stream, const uint8_t* src, const uint64_t* src_off, const uint32_t*,
                                    uint32_t n, uint32_t, uint32_t, uint8_t* dst, const uint64_t* dst_off,
                                    const uint32_t*, uint32_t* out_len, int32_t* status) {
  if (on_device(stream) != KDB_LZ4_OK) return KDB_LZ4_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    uint64_t on = 0, fn = 0;
    status[i] = orc_frame_uncompress(src + src_off[i], dst + dst_off[i], &on, &fn) == 0 ? 0 : -1;
    out_len[i] = (uint32_t)on;
  }
  return KDB_LZ4_OK;
}

uint64_t kdb_flush_scratch_bytes(uint32_t, uint32_t, uint64_t) { return 64; }

// kdb_flush_parts_batch: each run's parts through orc_put_part, in order, from
// the run's carried state; the kept frames packed back to back.
int kdb_flush_parts_batch(void* stream, const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len,
                          const uint8_t* chunks, const uint64_t* chunk_off, const uint32_t* chunk_len,
                          const uint64_t* offset_chunk, const uint64_t* size_value, const uint32_t* seg_first,
                          const uint32_t* run_first, const kdb_flush_state* carry_in, uint32_t nparts, uint32_t,
                          uint32_t nruns, uint32_t max_chunk, uint8_t*, uint64_t, uint64_t, kdb_flush_part* parts,
                          kdb_flush_state* carry_out, uint8_t* frames, uint64_t* frames_total) {
  if (on_device(stream) != KDB_LZ4_OK) return KDB_LZ4_EINVAL;
  uint8_t* fin = static_cast<uint8_t*>(malloc(8 + (size_t)orc_compress_bound((int)max_chunk) + 64));
  uint64_t packed = 0;
  for (uint32_t r = 0; r < nruns; r++) {
    orc_put_state S;
    memcpy(&S, &carry_in[r], sizeof(S));
    for (uint32_t s = run_first[r]; s < run_first[r + 1]; s++)
      for (uint32_t p = seg_first[s]; p < seg_first[s + 1]; p++) {
        uint32_t mode = 0, crc = 0;
        uint64_t occ = 0, fsz = 0, svc = 0;
        const int rc = orc_put_part(&S, keys + key_off[s], key_len[s], chunks + chunk_off[p], chunk_len[p],
                                    offset_chunk[p], size_value[p], fin, &mode, &occ, &fsz, &svc, &crc);
        kdb_flush_part P{};
        P.occ = occ;
        P.svc = svc;
        P.size = (uint32_t)fsz;
        P.crc = crc;
        P.mode = mode;
        P.status = rc;
        if (mode == KDB_FLUSH_FRAME && rc == 0) {
          P.frame_at = packed;
          memcpy(frames + packed, fin, fsz);
          packed += fsz;
        } else {
          P.frame_at = packed;
        }
        parts[p] = P;
      }
    memcpy(&carry_out[r], &S, sizeof(S));
  }
  *frames_total = packed;
  free(fin);
  (void)nparts;
  return KDB_LZ4_OK;
}

uint64_t kdb_get_scratch_bytes(uint32_t, uint64_t) { return 64; }

int kdb_get_values_batch(void* stream, const uint8_t* stored, const uint64_t* stored_off, const uint64_t* avail,
                         const uint64_t* svc, const uint64_t* size, uint32_t n, uint8_t* out, const uint64_t* out_off,
                         int verify, const uint32_t* checksum, const uint32_t* checksum_initial, uint64_t, uint32_t,
                         uint32_t, uint8_t*, uint64_t, uint64_t* out_len, int32_t* status) {
  if (on_device(stream) != KDB_LZ4_OK) return KDB_LZ4_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    uint64_t on = 0;
    const int st = orc_get_value(stored + stored_off[i], avail[i], svc[i], size[i], verify ? checksum[i] : 0,
                                 verify ? checksum_initial[i] : 0, verify, out + out_off[i], &on);
    status[i] = st == 0 ? 0 : st == -2 ? -2 : -1;
    out_len[i] = on;
  }
  return KDB_LZ4_OK;
}

}  // extern "C"
