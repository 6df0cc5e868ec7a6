/*
 * include/kdb_flush.h -- C ABI of the write-buffer flush batch (SURVEY.md §8
 * row f3): Database::PutPartValidSize's tail -- the CompressorLZ4 frame of
 * each part, the disable rule, offset_chunk_compressed, size_value_compressed
 * and the running CRC32C -- for a batch of parts that client threads queued
 * raw, with each thread's state carried in from earlier batches.
 *
 * Replaces, per part, /root/reference/interface/database.cc:143-267 (the
 * compression block, the disable rule :196-209, :237-248 and the CRC :251-257)
 * over the per-thread state the reference keeps in ThreadStorage
 * (ts_compression_enabled_, ts_offset_, CompressorLZ4::ts_compress_, CRC32's
 * ts_; thread/threadstorage.h:23-46).  The KingDB side that uses it is
 * kingdb_amd/csrc/flush_hook.cc (INTEGRATION.md level 4).
 *
 * Plain pointers and sizes; returns KDB_LZ4_OK or a negative KDB_LZ4_E* code;
 * the caller owns all memory.
 */
#ifndef KDB_FLUSH_H_
#define KDB_FLUSH_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One client thread's PutPartValidSize state between parts (ThreadStorage
 * defaults are 0: a thread that never sent a first part has compression
 * disabled, offsets 0 and CRC 0). */
typedef struct kdb_flush_state {
  uint64_t ts_offset;    /* Database::ts_offset_ */
  uint64_t comp_total;   /* CompressorLZ4::size_compressed() (ts_compress_) */
  uint32_t enabled;      /* Database::ts_compression_enabled_ */
  uint32_t crc;          /* Database::crc32_ (the finalized CRC32C so far) */
} kdb_flush_state;

/* chunk_final of a part (what WriteBuffer::PutPart receives as `chunk`) */
#define KDB_FLUSH_FRAME    0  /* the CompressorLZ4 frame (packed into `frames`) */
#define KDB_FLUSH_DISABLED 1  /* 8 zero bytes, then the raw chunk (database.cc:200-208) */
#define KDB_FLUSH_RAW      2  /* the raw chunk itself (compression off for the value, or empty) */
#define KDB_FLUSH_FAILED   3  /* Compress failed (database.cc:189): no state past :171, no CRC */

/* Per-part result: the arguments PutPartValidSize hands to WriteBuffer::PutPart. */
typedef struct kdb_flush_part {
  uint64_t occ;          /* offset_chunk_compressed */
  uint64_t svc;          /* size_value_compressed (0 unless the last part, :237-248) */
  uint64_t frame_at;     /* KDB_FLUSH_FRAME: offset of the frame in `frames` */
  uint32_t size;         /* chunk_final bytes */
  uint32_t crc;          /* crc32 argument: the running CRC32C at a last part, else 0 */
  uint32_t mode;         /* KDB_FLUSH_* */
  int32_t status;        /* 0, or -1 where PutPartValidSize returns IOError */
} kdb_flush_part;

/* Device scratch the batch needs. */
uint64_t kdb_flush_scratch_bytes(uint32_t nparts, uint32_t nseg, uint64_t raw_bytes);

/* A batch, all pointers on the device, stream-ordered.
 *   part p      chunks[chunk_off[p] .. +chunk_len[p]), PutPart(offset_chunk[p], size_value[p])
 *   segment s   parts seg_first[s] .. seg_first[s+1]-1 (nseg+1 entries): one thread's
 *               consecutive parts of one value; a segment whose first part has
 *               offset_chunk 0 starts the value (its CRC restarts from the key
 *               keys[key_off[s] .. +key_len[s])); only a run's first segment may
 *               continue a value, from carry_in[r].crc
 *   run r       segments run_first[r] .. run_first[r+1]-1 (nruns+1): one thread's
 *               segments whose policy state chains (every segment after the
 *               first starts a value with an empty first chunk, which keeps
 *               the compressor's running total); carry_in[r] -> carry_out[r]
 *   max_chunk   largest chunk_len (sizes the compress launch)
 * Outputs: parts[p]; carry_out[r] = the thread's state after the run (the CRC
 * included); the KDB_FLUSH_FRAME chunk_finals packed back to back in `frames`
 * (capacity: the sum of 8 + LZ4_compressBound(chunk_len) rounded to 16),
 * *frames_total = their bytes. */
int kdb_flush_parts_batch(void* stream, const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len,
                          const uint8_t* chunks, const uint64_t* chunk_off, const uint32_t* chunk_len,
                          const uint64_t* offset_chunk, const uint64_t* size_value, const uint32_t* seg_first,
                          const uint32_t* run_first, const kdb_flush_state* carry_in, uint32_t nparts,
                          uint32_t nseg, uint32_t nruns, uint32_t max_chunk, uint8_t* scratch,
                          uint64_t scratch_bytes, uint64_t raw_bytes, kdb_flush_part* parts,
                          kdb_flush_state* carry_out, uint8_t* frames, uint64_t* frames_total);

#ifdef __cplusplus
}
#endif

#endif /* KDB_FLUSH_H_ */
