// kingdb_amd/kingdb_include/cache/lz4_flush.h -- the write-buffer flush hook
// (SURVEY.md §8 row f3): LZ4 compression, the value CRC32C and
// size_value_compressed of single-part puts move from the client thread
// (Database::PutPartValidSize, /root/reference/interface/database.cc:128-276)
// to the write buffer's flush (WriteBuffer::ProcessingLoop,
// /root/reference/cache/write_buffer.cc:228-319), where a whole buffer's worth
// of values goes to the GPU as ONE kdb_put_entries_batch call.
//
// Two call sites in KingDB (oracle/kingdb_hook.py applies them to a copy of
// the reference tree; INTEGRATION.md level 4):
//   * PutPartValidSize: a deferrable chunk (LZ4FlushDeferrable) is handed to
//     WriteBuffer::PutPart raw, with size_value_compressed 0 and crc32 0.  An
//     order like that is self-contained (util/order.h:52-59) and, while it sits
//     in the buffer, WriteBuffer::Get (write_buffer.cc:59-64, 105-110) returns
//     it as an uncompressed value: read-your-writes sees the raw bytes.
//   * ProcessingLoop: the orders handed to the storage engine are a copy of the
//     flush buffer passed through LZ4FlushOrders, which turns every pending
//     order into exactly the order PutPartValidSize would have queued (chunk =
//     the frame or the disabled-compression form, size_value_compressed, crc32).
//     The buffer itself is not modified, so concurrent readers keep seeing the
//     raw bytes until the buffer is cleared.
#ifndef KINGDB_LZ4_FLUSH_H_
#define KINGDB_LZ4_FLUSH_H_

#include <vector>

#include "util/options.h"
#include "util/order.h"

namespace kdb {

// Values above this stay on PutPartValidSize's own path (one GPU call each).
constexpr uint64_t kLZ4FlushMaxValue = 64ull << 20;

// A chunk that is a whole value (first and last part), LZ4 on, not empty.
inline bool LZ4FlushDeferrable(const DatabaseOptions& db_options, uint64_t size_chunk, uint64_t offset_chunk,
                               uint64_t size_value) {
  return db_options.compression.type == kLZ4Compression && offset_chunk == 0 && size_chunk == size_value &&
         size_chunk > 0 && size_chunk <= kLZ4FlushMaxValue;
}

// Completes the deferred orders in `orders` in one GPU batch.  A GPU failure
// is fatal (log::emerg + abort): an order must never reach an HSTable without
// its frame and checksum.
void LZ4FlushOrders(const DatabaseOptions& db_options, std::vector<Order>& orders);

}  // namespace kdb

#endif  // KINGDB_LZ4_FLUSH_H_
