"""Host-inclusive write path (BASELINE configs[4]): puts in pinned host memory
-> HSTable file bytes in host memory, through the GPU.

The reference's sequential-write bench (doc/bench/db_bench_kingdb.cc:457-489:
16-byte "%016d" keys, 100-byte values) drives Database::Put one call at a time;
KingDB buffers the orders (cache/write_buffer.cc) and HSTableManager encodes
and writes them in batches.  Here a batch of puts is the unit: per chunk of
`chunk` puts, over `nstreams` HIP streams,

  H2D keys + values + metadata -> kdb_put_entries_batch (frame policy, LZ4,
  CRC32C, key hash, EntryHeader: csrc/put.hip) -> D2H of the per-entry
  offset/length/hash/kind/status -> host HSTable framing (csrc/hstable.cc),
  in put order, which DMAs the entry bytes (exactly Σ entry_len) from HBM
  straight into the pinned file buffers (direct=True; direct=False lands them
  in a pinned staging buffer and memcpys them into the files)

with the copies and kernels of later chunks overlapping the host framing of
earlier ones.  Timing is host wall clock from the first enqueue to the last
entry byte in its file.  Nothing here computes on the CPU except that framing.
"""
from __future__ import annotations

import time

import numpy as np

from . import _lib
from .hostpipe import PinnedBuffer
from .lz4 import Event, Stream, lib
from .put import HSTableWriter, PutBatch


class PutPipeline:
    """n puts of fixed-size keys and values (the db_bench shape)."""

    def __init__(self, n: int, key_size: int, value_size: int, chunk: int = 1 << 16, nstreams: int = 4,
                 hstable_size: int = 32 << 20, hash_type: int = 1, direct: bool = True):
        self.n, self.ks, self.vs = int(n), int(key_size), int(value_size)
        self.chunk = max(1, min(int(chunk), self.n))
        self.nchunks = (self.n + self.chunk - 1) // self.chunk
        self.hstable_size, self.hash_type, self.direct = hstable_size, hash_type, bool(direct)
        self.streams = [Stream() for _ in range(max(1, nstreams))]
        n, c = self.n, self.chunk
        self.h_keys = PinnedBuffer(n * self.ks)
        self.h_vals = PinnedBuffer(n * self.vs)
        # chunk-local metadata, identical for every full chunk:
        # key_off u64 | key_len u32 | value_off u64 | value_len u64 | part_first u32 (c+1) | chunk_len u32
        idx = np.arange(c, dtype=np.uint64)
        pf = np.arange(c + 1, dtype=np.uint32)
        self.meta = np.concatenate([(idx * np.uint64(self.ks)).view(np.uint8),
                                    np.full(c, self.ks, np.uint32).view(np.uint8),
                                    (idx * np.uint64(self.vs)).view(np.uint8),
                                    np.full(c, self.vs, np.uint64).view(np.uint8), pf.view(np.uint8)])
        self.h_meta = PinnedBuffer(self.meta.nbytes)
        self.h_meta.np[:] = self.meta
        self.h_chunks = PinnedBuffer(4 * c)
        self.h_chunks.np[:] = np.full(c, self.vs, np.uint32).view(np.uint8)
        self.batches = [PutBatch(c, c, c * self.vs, c * self.ks) for _ in self.streams]
        for b in self.batches:
            b.vmeta.upload(self.meta)
            b.chunks.upload(self.h_chunks.np)
        # per stream slot: pinned landing zones for one chunk's outputs
        self.h_ent = [] if self.direct else [PinnedBuffer(b.entries_cap) for b in self.batches]
        self.h_out = [PinnedBuffer(32 * c + 64) for _ in self.batches]
        self.writer: HSTableWriter | None = None

    def _range(self, k: int) -> tuple[int, int]:
        lo = k * self.chunk
        return lo, min(lo + self.chunk, self.n)

    def run(self) -> float:
        """All n puts -> HSTable files (self.writer).  Returns wall seconds."""
        L = lib()
        S = len(self.streams)
        if self.writer is None:
            self.writer = HSTableWriter(self.hstable_size, self.hash_type, pinned=self.direct)
        else:
            self.writer.reset()     # a fresh directory; file buffers (like buffer_raw_) are reused
        w = self.writer
        tot_ev = [Event() for _ in range(self.nchunks)]
        self.stats = {"wait_s": 0.0, "frame_s": 0.0}

        def drain(k: int) -> None:
            lo, hi = self._range(k)
            m = hi - lo
            s = k % S
            st, b = self.streams[s], self.batches[s]
            ta = time.perf_counter()
            _lib.check(L.kdb_lz4_event_sync(tot_ev[k].ptr), "event_sync")
            ho = self.h_out[s]
            p = ho.ptr
            if self.direct:
                tb = time.perf_counter()
                w.append_device(st.ptr, b.entries.ptr, p, p + 8 * m, p + 12 * m, p + 24 * m, p + 28 * m, m)
            else:
                total = int(ho.np[32 * m:32 * m + 8].view(np.uint64)[0])
                if total:
                    _lib.check(L.kdb_lz4_memcpy_d2h(self.h_ent[s].ptr, b.entries.ptr, total, st.ptr), "d2h entries")
                st.sync()
                tb = time.perf_counter()
                w.append_raw(self.h_ent[s].ptr, p, p + 8 * m, p + 12 * m, p + 24 * m, p + 28 * m, m)
            self.stats["wait_s"] += tb - ta
            self.stats["frame_s"] += time.perf_counter() - tb

        t0 = time.perf_counter()
        for k in range(self.nchunks):
            lo, hi = self._range(k)
            m = hi - lo
            s = k % S
            st, b = self.streams[s], self.batches[s]
            _lib.check(L.kdb_lz4_memcpy_h2d(b.keys.ptr, self.h_keys.ptr + lo * self.ks, m * self.ks, st.ptr), "h2d keys")
            _lib.check(L.kdb_lz4_memcpy_h2d(b.values.ptr, self.h_vals.ptr + lo * self.vs, m * self.vs, st.ptr),
                       "h2d values")
            b.run_device(st, m, m, self.vs, m * self.vs, self.hash_type)
            o = b.out.ptr
            for off, width in ((0, 8), (8, 4), (12, 8), (24, 4), (28, 4)):
                # entry_off u64, entry_len u32, hashed u64, kind u32, status i32 (chunk-local layout of PutBatch)
                _lib.check(L.kdb_lz4_memcpy_d2h(self.h_out[s].ptr + off * m, o + off * m, width * m, st.ptr), "d2h out")
            _lib.check(L.kdb_lz4_memcpy_d2h(self.h_out[s].ptr + 32 * m, o + 32 * m, 8, st.ptr), "d2h total")
            tot_ev[k].record(st)
            if k >= S - 1:
                drain(k - (S - 1))
        for k in range(max(0, self.nchunks - (S - 1)), self.nchunks):
            drain(k)
        w.close()                   # + every entry byte landed
        return time.perf_counter() - t0

    def free(self) -> None:
        for b in self.batches:
            b.free()
        for p in [self.h_keys, self.h_vals, self.h_meta, self.h_chunks] + self.h_ent + self.h_out:
            p.free()
