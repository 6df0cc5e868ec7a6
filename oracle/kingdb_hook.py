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
  database.cc, Database::PutPartValidSize (:128-276): before the compression
    block, a deferrable chunk (LZ4FlushDeferrable) goes to WriteBuffer::PutPart
    raw, with size_value_compressed 0 and crc32 0;
  write_buffer.cc, WriteBuffer::ProcessingLoop (:228-319): the storage engine
    receives a copy of the flush buffer passed through LZ4FlushOrders (one
    kdb_put_entries_batch for the deferred orders) instead of the buffer.
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
         "  if (LZ4FlushDeferrable(db_options_, chunk.size(), offset_chunk, size_value)) {\n"
         "    // frame, CRC32C and size_value_compressed at the flush (LZ4FlushOrders)\n"
         "    return wb_->PutPart(write_options, key, chunk, 0, size_value, 0, 0);\n"
         "  }\n"
         "  bool do_compression = true;\n  uint64_t size_value_compressed = 0;\n"),
    ],
    "cache/write_buffer.cc": [
        ('#include "cache/write_buffer.h"\n', '#include "cache/write_buffer.h"\n' + INCLUDE),
        ("    event_manager_->flush_buffer.StartAndBlockUntilDone(buffers_[im_copy_]);\n",
         "    std::vector<Order> flushed(buffers_[im_copy_]);\n"
         "    LZ4FlushOrders(db_options_, flushed);\n"
         "    event_manager_->flush_buffer.StartAndBlockUntilDone(flushed);\n"),
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
