#!/usr/bin/env python3
"""oracle/kingdb_hook.py -- TEST INFRASTRUCTURE: applies the write-buffer flush
hook (kingdb_amd/kingdb_include/cache/lz4_flush.h) to a
COPY of two reference sources outside the repository:

  /root/reference/interface/database.cc  -> <out>/interface/database.cc
  /root/reference/cache/write_buffer.cc  -> <out>/cache/write_buffer.cc

(out defaults to /tmp/kdb_hook_src).  Nothing of the reference is written into
the repo; oracle/Makefile `kingdb_hook` compiles the copies into
oracle/_ref/kingdb_hook/ beside the untouched rest of the tree.

The edits, each anchored on text that must occur exactly once:
  database.cc, Database::PutPartValidSize (:128-276): with LZ4 on, before the
    compression block, the call is queued to the pipeline (LZ4FlushDefer) and
    the chunk goes to WriteBuffer::PutPart raw, with size_value_compressed 0
    and the pipeline's ticket in the crc32 field;
  write_buffer.cc, WriteBuffer::ProcessingLoop (:228-319): the pipeline lives
    as long as the loop (LZ4FlushScope), and before the buffer is handed to the
    storage engine, with its readers held off, LZ4FlushOrders completes the
    deferred orders in place.
INTEGRATION.md level 4 shows the same edits as a diff for a maintainer.
"""
import os
import sys

REF = os.environ.get("REF", "/root/reference")

INCLUDE = '#include "cache/lz4_flush.h"\n'

EDITS = {
    "interface/database.cc": [
        ('#include "interface/database.h"\n', '#include "interface/database.h"\n' + INCLUDE),
        ("  bool do_compression = true;\n  uint64_t size_value_compressed = 0;\n",
         "  if (LZ4FlushDeferrable(db_options_)) {\n"
         "    // frame, offsets, size_value_compressed and CRC32C at the flush (LZ4FlushOrders);\n"
         "    // the order carries its ticket in the crc32 field until then\n"
         "    uint32_t lz4_ticket = 0;\n"
         "    s = LZ4FlushDefer(wb_, db_options_, key, chunk, offset_chunk, size_value, &lz4_ticket);\n"
         "    if (!s.IsOK()) return s;\n"
         "    s = wb_->PutPart(write_options, key, chunk, offset_chunk, size_value, 0, lz4_ticket);\n"
         "    if (!s.IsOK()) LZ4FlushCancel(wb_, lz4_ticket);\n"
         "    return s;\n"
         "  }\n"
         "  bool do_compression = true;\n  uint64_t size_value_compressed = 0;\n"),
    ],
    "cache/write_buffer.cc": [
        ('#include "cache/write_buffer.h"\n', '#include "cache/write_buffer.h"\n' + INCLUDE),
        ("void WriteBuffer::ProcessingLoop() {\n",
         "void WriteBuffer::ProcessingLoop() {\n"
         "  LZ4FlushScope lz4_flush_scope(this, db_options_);   // the LZ4 pipeline lives as long as this loop\n"),
        ("    event_manager_->flush_buffer.StartAndBlockUntilDone(buffers_[im_copy_]);\n",
         "    {\n"
         "      // the deferred puts become the orders PutPartValidSize would have queued;\n"
         "      // the buffer's readers wait outside, as for its clear below\n"
         "      std::unique_lock<std::mutex> lock_copy(mutex_copy_write_level4_);\n"
         "      while (true) {\n"
         "        std::unique_lock<std::mutex> lock_read(mutex_copy_read_level5_);\n"
         "        if (num_readers_ == 0) break;\n"
         "        cv_read_.wait(lock_read);\n"
         "      }\n"
         "      LZ4FlushOrders(this, db_options_, buffers_[im_copy_]);\n"
         "    }\n"
         "    event_manager_->flush_buffer.StartAndBlockUntilDone(buffers_[im_copy_]);\n"),
    ],
}


def apply(out: str) -> None:
    for rel, edits in EDITS.items():
        with open(os.path.join(REF, rel)) as f:
            text = f.read()
        for old, new in edits:
            if text.count(old) != 1:
                sys.exit(f"kingdb_hook: anchor found {text.count(old)} times in {rel}: {old!r}")
            text = text.replace(old, new)
        dst = os.path.join(out, rel)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        tmp = dst + ".tmp"
        with open(tmp, "w") as f:
            f.write(text)
        # keep the copy's mtime when nothing changed, so make does not rebuild
        if os.path.exists(dst) and open(dst).read() == text:
            os.remove(tmp)
        else:
            os.replace(tmp, dst)


if __name__ == "__main__":
    apply(sys.argv[1] if len(sys.argv) > 1 else "/tmp/kdb_hook_src")
