/*
 * include/kdb_lz4.h -- C ABI of the MI355X (gfx950) LZ4 block codec that drops in
 * behind KingDB's CompressorLZ4 (/root/reference/algorithm/compressor.h:102-176).
 *
 * Plain pointers and sizes only; no HIP or torch types cross this boundary
 * (streams and events are opaque `void*`).  Every function returns an int
 * status (KDB_LZ4_OK or a negative KDB_LZ4_E* code) except where it mirrors an
 * LZ4 r1.3.0 function, whose exact return convention it keeps.  No exception
 * crosses the ABI.  The caller owns all memory.
 *
 * All compute runs in hand-written HIP kernels on the GPU.  There is no CPU
 * codec behind this ABI: without a usable device the compute entry points
 * return KDB_LZ4_ENODEV (scalar LZ4 mirrors: their error value) -- never a
 * CPU result.
 */
#ifndef KDB_LZ4_H_
#define KDB_LZ4_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KDB_LZ4_OK            0
#define KDB_LZ4_EINVAL       -1   /* bad argument */
#define KDB_LZ4_EHIP         -2   /* HIP runtime error (launch, copy, alloc) */
#define KDB_LZ4_ENODEV       -3   /* no usable gfx950 device */
#define KDB_LZ4_EUNSUPPORTED -4   /* size outside what this build's kernels handle */

/* Per-value status word of the batch entry points for a value the launch
 * could not process (e.g. larger than max_len); distinct from LZ4 codes. */
#define KDB_LZ4_VALUE_UNSUPPORTED ((int32_t)0x80000000)

int kdb_lz4_version(void); /* 10000*major + 100*minor + patch */

/* ---------------------------------------------------------------- runtime */
int kdb_lz4_device_count(int* count);
/* Binds `device` for the calling thread and runs its lane-order self-test
 * (kdb_lz4_selftest) if it has not run yet. */
int kdb_lz4_set_device(int device);
int kdb_lz4_get_device(int* device);
/* The compressor's exactness rests on one LDS behaviour: the lanes of one
 * ds_mskor_rtn_b32 that hit the same dword apply in ascending lane order
 * (lz4_compress.hip, the exchange tables).  This runs the device self-test of
 * that behaviour once per device (later calls return the cached verdict):
 * *state = 1 passed, -1 failed (then every compress entry point returns
 * KDB_LZ4_EUNSUPPORTED on that device, never a frame), 0 not run;
 * *bad_lanes (optional) = mismatching lane results seen. */
int kdb_lz4_selftest(int device, int* state, uint32_t* bad_lanes);
/* Readies the current device for the first real call: runs its lane-order
 * self-test and one small batch through every kernel family (so the code
 * object is loaded and the runtime's first-launch costs are paid here, not
 * inside a caller's timed or latency-critical path).  Synchronous; idempotent. */
int kdb_lz4_warmup(void);
/* The per-call decode path's resident service (kingdb_amd/csrc/service.h) on
 * `device`: *launches = instances launched so far, *served = requests the
 * instances that exited served, *alive = 1 while one is resident.  All 0 when
 * the service was never used on the device.  No HIP call. */
int kdb_lz4_service_stats(int device, uint32_t* launches, uint32_t* served, uint32_t* alive);
/* The same device's services' protocol counters (diagnostics; added when the
 * waves exit): polls made, requests taken from their posts (arguments and
 * input read with the doorbells, no second PCIe round trip), and decode
 * results answered by a reply record ahead of the done word (service.h). */
int kdb_lz4_service_counters(int device, uint32_t* polls, uint32_t* from_post, uint32_t* replied);
/* Test hook for the services' request numbers (kdb_lz4_capi.hip,
 * service_call): on the calling thread's device, stops each service created
 * so far, waits for its wave to leave, and sets every slot as if its last
 * request had been number `req` (doorbell, the host's copy, the done word),
 * with a reply record of tags `reply_tag`, return value 0 and a valid
 * checksum (a record a wave wrote `reply_tag` requests ago).  The next call
 * on a slot then takes request number req + 1, skipping 0. */
int kdb_lz4_service_seed_requests(uint32_t req, uint32_t reply_tag);
/* The kernels (rocprof names, ';'-separated) that the calling thread's last
 * compress or decompress batch queued.  No HIP call. */
int kdb_lz4_last_kernels(char* buf, uint64_t cap);
/* The build id of the loaded library: a hash of the HIP and header sources it
 * was compiled from (kingdb_amd/Makefile), so that measurements taken with one
 * build (e.g. committed PMC traffic) can be matched to the build in use. */
int kdb_lz4_build_id(char* buf, uint64_t cap);
int kdb_lz4_malloc(void** ptr, uint64_t bytes);              /* device memory */
int kdb_lz4_free(void* ptr);
int kdb_lz4_host_alloc(void** ptr, uint64_t bytes);          /* pinned host memory */
int kdb_lz4_host_free(void* ptr);
int kdb_lz4_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream);
int kdb_lz4_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream);
int kdb_lz4_memcpy_d2d(void* dst, const void* src, uint64_t bytes, void* stream);
int kdb_lz4_memset(void* ptr, int value, uint64_t bytes, void* stream);
int kdb_lz4_stream_create(void** stream);
int kdb_lz4_stream_destroy(void* stream);
int kdb_lz4_stream_sync(void* stream);
int kdb_lz4_device_sync(void);
int kdb_lz4_event_create(void** event);
int kdb_lz4_event_destroy(void* event);
int kdb_lz4_event_record(void* event, void* stream);
int kdb_lz4_event_sync(void* event);
int kdb_lz4_event_elapsed_ms(void* start, void* stop, float* ms);
/* later work on `stream` waits for `event` (hipStreamWaitEvent): copies on their own
 * streams behind a kernel, so the two PCIe directions overlap (kingdb_amd/hostpipe.py) */
int kdb_lz4_stream_wait_event(void* stream, void* event);

/* ------------------------------------------------ scalar LZ4 r1.3.0 mirrors
 * Host buffers, synchronous, one value per call (a batch of one on the GPU).
 * Same signatures and return conventions as the reference; link-time aliases
 * with the exact LZ4_* names are exported too. */

/* replaces LZ4_compressBound, algorithm/lz4.h:115 (macro lz4.h:103) */
int kdb_lz4_compressBound(int isize);

/* replaces LZ4_compress_limitedOutput, algorithm/lz4.h:129 (lz4.cc:664-682):
 * returns the block size, or 0 if it does not fit in maxOutputSize.  Unlike
 * r1.3.0 this never writes past maxOutputSize. */
int kdb_lz4_compress_limitedOutput(const char* source, char* dest, int inputSize,
                                   int maxOutputSize);

/* replaces LZ4_decompress_safe_partial, algorithm/lz4.h:169 (lz4.cc:1050-1053):
 * returns bytes decoded, or -(input bytes consumed)-1 on malformed input. */
int kdb_lz4_decompress_safe_partial(const char* source, char* dest, int compressedSize,
                                    int targetOutputSize, int maxDecompressedSize);

/* ------------------------------------------------------- batch entry points
 * Device pointers; stream-ordered and asynchronous (`stream` may be NULL for
 * the default stream).  Value v occupies src[src_off[v] .. +len[v]) and writes
 * dst[dst_off[v] ..).  `max_len` (compress) / `max_in`,`max_out` (decompress)
 * bound the per-value sizes of the launch; they size the kernels' LDS. */

/* 8 + LZ4_compressBound(size): the slot a CompressorLZ4 frame needs. */
uint64_t kdb_lz4_frame_bound(uint32_t size);

/* LZ4_compress_limitedOutput per value: ret[v] = block size or 0;
 * dst slot capacity dst_cap[v]. */
int kdb_lz4_compress_blocks_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint32_t n, uint32_t max_len,
                                  uint8_t* dst, const uint64_t* dst_off, const uint32_t* dst_cap,
                                  int32_t* ret);

/* LZ4_decompress_safe_partial(src, dst, in_len, target, dst_cap) per value
 * (target == NULL means target = dst_cap); ret[v] = LZ4 return code. */
int kdb_lz4_decompress_blocks_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                    const uint32_t* in_len, uint32_t n, uint32_t max_in,
                                    uint32_t max_out, uint8_t* dst, const uint64_t* dst_off,
                                    const uint32_t* dst_cap, const uint32_t* target,
                                    int32_t* ret);

/* CompressorLZ4::Compress per value (compressor.cc:15-65): frame = u32le
 * size_compressed_stored, u32le size_source, payload (raw fallback when the
 * block is larger than the value).  Slot capacity >= kdb_lz4_frame_bound(len).
 * frame_len[v] = frame bytes; status[v] = 0, or -1 where the reference returns
 * IOError. */
int kdb_lz4_compress_frames_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint32_t n, uint32_t max_len,
                                  uint8_t* dst, const uint64_t* dst_off, uint32_t* frame_len,
                                  int32_t* status);

/* CompressorLZ4::Uncompress of one frame per value (compressor.cc:75-137):
 * avail[v] = bytes readable at src_off[v]; raw bytes go to dst_off[v] (capacity
 * dst_cap[v]); out_len[v] = *size_dest; status[v] = 0 or -1 (IOError). */
int kdb_lz4_decompress_frames_batch(void* stream, const uint8_t* src, const uint64_t* src_off,
                                    const uint32_t* avail, uint32_t n, uint32_t max_in,
                                    uint32_t max_out, uint8_t* dst, const uint64_t* dst_off,
                                    const uint32_t* dst_cap, uint32_t* out_len, int32_t* status);

/* Compaction of frame slots into one dense stream (additive; the host-side
 * equivalent is KingDB writing frames back to back: hstable_manager.h:656-673,
 * database.cc:143-248).  dst_off[v] = exclusive prefix sum of len (device
 * array), *total = Σ len (device pointer); frame v is copied from
 * src + src_off[v] to dst + dst_off[v]. */
int kdb_lz4_pack_frames(void* stream, const uint8_t* src, const uint64_t* src_off,
                        const uint32_t* len, uint32_t n, uint8_t* dst, uint64_t* dst_off,
                        uint64_t* total);

/* *out (device pointer) = the largest of v[0..n) (device array), 0 for n = 0:
 * e.g. the largest frame of a device-resident batch, for the max_in argument
 * of kdb_lz4_decompress_frames_batch when the caller holds no host copy of
 * the frame lengths. */
int kdb_lz4_max_u32(void* stream, const uint32_t* v, uint32_t n, uint32_t* out);

/* ----------------------------------------------------------- data helpers */

/* Synthetic G1 ("db_bench") data on the device: 100-byte pieces first_piece ..
 * first_piece+npieces-1 of LevelDB Random(seed) CompressibleString(0.5, 100)
 * (doc/bench/db_bench_kingdb.cc:119-131), generated in parallel by jump-ahead. */
int kdb_lz4_gen_g1(uint8_t* dst, uint64_t first_piece, uint64_t npieces, uint32_t seed,
                   void* stream);

#ifdef __cplusplus
}
#endif

#endif /* KDB_LZ4_H_ */
