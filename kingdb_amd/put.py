"""The write path around the codec (include/kdb_put.h).

Mirrors what KingDB does with a stream of puts from one client thread --
Database::PutPart's frame policy and CRC32C (interface/database.cc:87-276),
then HSTableManager's entry and file encoding (storage/hstable_manager.h) --
with the per-value work on the GPU (csrc/put.hip) and only the per-file
framing on the host (csrc/hstable.cc).

  put_entries(puts)          one GPU batch: entry bytes, key hashes, CRCs
  HSTableWriter              the HSTable files those entries make
  write_hstables(puts, ...)  both, batch by batch: {file name: bytes}

A put is (key, value) or (key, value, chunks): `chunks` lists the sizes of
the PutPart calls the value arrives in (default: one call, i.e. Database::Put
of a value <= maximum_part_size; use split_parts() for Put's own splitting).
Nothing here computes on the CPU except that host-side framing.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .lz4 import DeviceBuffer, Stream

SELF_CONTAINED, MULTIPART, MULTIPART_UNFINISHED = 0, 1, 2
MAX_PART_SIZE = 1 << 20          # storage__maximum_part_size default (util/options.h:170-172)


def lib():
    return _lib.load()


def padding_size(size_value: int) -> int:
    """EntryHeader::CalculatePaddingSize (storage/format.h:63-71)."""
    return (size_value // 65536 + 1) * 8


def split_parts(size: int, part_size: int = MAX_PART_SIZE) -> list[int]:
    """Database::PutPart's split of a value larger than maximum_part_size
    (interface/database.cc:96-122)."""
    if size <= part_size:
        return [size]
    return [min(part_size, size - o) for o in range(0, size, part_size)]


@dataclass
class PutBatchResult:
    entries: np.ndarray      # dense entry stream (u8)
    entry_off: np.ndarray    # u64
    entry_len: np.ndarray    # u32
    hashed: np.ndarray       # u64
    crc: np.ndarray          # u32
    kind: np.ndarray         # u32
    status: np.ndarray       # i32

    def entry(self, i: int) -> bytes:
        o = int(self.entry_off[i])
        return self.entries[o:o + int(self.entry_len[i])].tobytes()


class PutBatch:
    """Device buffers for batches of up to `n` puts / `raw` value bytes /
    `key_bytes` key bytes / `nparts` chunks, reused across calls."""

    def __init__(self, n: int, nparts: int, raw: int, key_bytes: int):
        self.n, self.nparts, self.raw, self.key_bytes = n, nparts, raw, key_bytes
        self.scratch_bytes = int(lib().kdb_put_scratch_bytes(n, nparts, raw))
        self.scratch = DeviceBuffer(self.scratch_bytes)
        self.keys = DeviceBuffer(key_bytes + 64)
        self.values = DeviceBuffer(raw + 64)
        # per value: key_off u64, key_len u32, value_off u64, value_len u64, part_first u32 (n+1)
        self.vmeta = DeviceBuffer(n * 32 + 8)
        self.chunks = DeviceBuffer(nparts * 4 + 4)
        self.entries_cap = raw + n * 64 + key_bytes + (raw // 65536 + 1) * 8 * 2 + n * 8 + 64
        self.entries = DeviceBuffer(self.entries_cap)
        # outputs: entry_off u64, entry_len u32, hashed u64, crc u32, kind u32, status i32, total u64
        self.out = DeviceBuffer(n * 32 + 64)

    def free(self) -> None:
        for b in (self.scratch, self.keys, self.values, self.vmeta, self.chunks, self.entries, self.out):
            b.free()

    def _optr(self, n: int):
        o = self.out.ptr
        return dict(entry_off=o, entry_len=o + 8 * n, hashed=o + 12 * n, crc=o + 20 * n, kind=o + 24 * n,
                    status=o + 28 * n, total=o + 32 * n)

    def run_device(self, stream, n: int, nparts: int, max_chunk: int, raw: int, hash_type: int) -> None:
        """Launches kdb_put_entries_batch on what is already resident."""
        if n > self.n or nparts > self.nparts or raw > self.raw:
            raise ValueError("batch larger than the buffers")
        v, c = self.vmeta.ptr, self.n     # metadata laid out for the capacity (a short batch uses a prefix)
        o = self._optr(n)
        _lib.check(lib().kdb_put_entries_batch(
            stream.ptr if stream else None, self.keys.ptr, v, v + 8 * c, self.values.ptr, v + 12 * c, v + 20 * c,
            v + 28 * c, self.chunks.ptr, nparts, max_chunk, n, hash_type, self.scratch.ptr, self.scratch_bytes, raw,
            self.entries.ptr, o["entry_off"], o["entry_len"], o["total"], o["hashed"], o["crc"], o["kind"],
            o["status"]), "kdb_put_entries_batch")


def _layout(puts):
    keys = [p[0] for p in puts]
    vals = [p[1] for p in puts]
    chunks = [list(p[2]) if len(p) > 2 and p[2] is not None else [len(p[1])] for p in puts]
    for v, ch in zip(vals, chunks):
        if sum(ch) != len(v):
            raise ValueError("chunk sizes must add up to the value size")
    n = len(puts)
    klen = np.array([len(k) for k in keys], np.uint32)
    vlen = np.array([len(v) for v in vals], np.uint64)
    koff = np.zeros(n, np.uint64)
    voff = np.zeros(n, np.uint64)
    if n > 1:
        koff[1:] = np.cumsum(klen[:-1].astype(np.uint64))
        voff[1:] = np.cumsum(vlen[:-1])
    nch = np.array([len(c) for c in chunks], np.uint32)
    pf = np.zeros(n + 1, np.uint32)
    pf[1:] = np.cumsum(nch)
    clen = np.array([c for ch in chunks for c in ch], np.uint32)
    kbuf = np.frombuffer(b"".join(keys), np.uint8) if n else np.zeros(0, np.uint8)
    vbuf = np.frombuffer(b"".join(vals), np.uint8) if n else np.zeros(0, np.uint8)
    return kbuf, vbuf, koff, klen, voff, vlen, pf, clen


def put_entries(puts, hash_type: int = 1, stream: Stream | None = None) -> PutBatchResult:
    """One GPU batch: the HSTable entry bytes of every put (see kdb_put.h)."""
    kbuf, vbuf, koff, klen, voff, vlen, pf, clen = _layout(puts)
    n = len(puts)
    nparts = len(clen)
    raw = int(vlen.sum()) if n else 0
    b = PutBatch(max(n, 1), max(nparts, 1), max(raw, 1), max(len(kbuf), 1))
    try:
        st = stream.ptr if stream else None
        if len(kbuf):
            b.keys.upload(kbuf, stream=st)
        if len(vbuf):
            b.values.upload(vbuf, stream=st)
        meta = np.concatenate([koff.view(np.uint8), klen.view(np.uint8), voff.view(np.uint8), vlen.view(np.uint8),
                               pf.view(np.uint8)])
        b.vmeta.upload(meta, stream=st)
        if nparts:
            b.chunks.upload(clen, stream=st)
        b.run_device(stream, n, nparts, int(clen.max()) if nparts else 0, raw, hash_type)
        o = b._optr(n)
        # the copies back ride the caller's stream (see get_values)
        out = b.out.download(32 * n + 8, 0, stream=st)
        total = int(out[32 * n:32 * n + 8].view(np.uint64)[0])
        ents = b.entries.download(total, stream=st) if total else np.zeros(0, np.uint8)
        del o
        return PutBatchResult(
            entries=ents, entry_off=out[0:8 * n].view(np.uint64).copy(), entry_len=out[8 * n:12 * n].view(np.uint32).copy(),
            hashed=out[12 * n:20 * n].view(np.uint64).copy(), crc=out[20 * n:24 * n].view(np.uint32).copy(),
            kind=out[24 * n:28 * n].view(np.uint32).copy(), status=out[28 * n:32 * n].view(np.int32).copy())
    finally:
        b.free()


class HSTableWriter:
    """HSTable files for one database directory (csrc/hstable.cc)."""

    def __init__(self, hstable_size: int = 32 << 20, hash_type: int = 1, pinned: bool = False):
        h = ctypes.c_void_p()
        _lib.check(lib().kdb_hstable_writer_create2(hstable_size, hash_type, 1 if pinned else 0, ctypes.byref(h)),
                   "hstable_writer_create")
        self.h = h.value
        self.hstable_size, self.hash_type = hstable_size, hash_type

    def append(self, r: PutBatchResult) -> None:
        n = len(r.entry_len)
        ents = r.entries if len(r.entries) else np.zeros(1, np.uint8)
        _lib.check(lib().kdb_hstable_writer_append(
            self.h, ents.ctypes.data, r.entry_off.ctypes.data, r.entry_len.ctypes.data, r.hashed.ctypes.data,
            r.kind.ctypes.data, r.status.ctypes.data, n), "hstable_writer_append")

    def append_raw(self, entries_ptr: int, entry_off_ptr: int, entry_len_ptr: int, hashed_ptr: int, kind_ptr: int,
                   status_ptr: int, n: int) -> None:
        """append() from host pointers (pinned buffers of the bench pipeline)."""
        _lib.check(lib().kdb_hstable_writer_append(self.h, entries_ptr, entry_off_ptr, entry_len_ptr, hashed_ptr,
                                                   kind_ptr, status_ptr, n), "hstable_writer_append")

    def append_device(self, stream_ptr: int, d_entries: int, entry_off_ptr: int, entry_len_ptr: int,
                      hashed_ptr: int, kind_ptr: int, status_ptr: int, n: int) -> None:
        """append() with the entry bytes still on the device: DMA on `stream`
        straight into the files (host pointers for the per-entry arrays)."""
        _lib.check(lib().kdb_hstable_writer_append_device(self.h, stream_ptr, d_entries, entry_off_ptr, entry_len_ptr,
                                                          hashed_ptr, kind_ptr, status_ptr, n),
                   "hstable_writer_append_device")

    def close(self) -> None:
        _lib.check(lib().kdb_hstable_writer_close(self.h), "hstable_writer_close")

    def reset(self) -> None:
        """A fresh directory; the file buffers' memory is kept for reuse."""
        _lib.check(lib().kdb_hstable_writer_reset(self.h), "hstable_writer_reset")

    def files(self) -> dict[str, bytes]:
        c = ctypes.c_uint32(0)
        _lib.check(lib().kdb_hstable_writer_file_count(self.h, ctypes.byref(c)), "file_count")
        out = {}
        for i in range(c.value):
            fid, p, sz = ctypes.c_uint32(), ctypes.c_void_p(), ctypes.c_uint64()
            _lib.check(lib().kdb_hstable_writer_file(self.h, i, ctypes.byref(fid), ctypes.byref(p), ctypes.byref(sz)),
                       "file")
            out["%08x" % fid.value] = ctypes.string_at(p.value, sz.value) if sz.value else b""
        return out

    def file_bytes(self) -> int:
        c = ctypes.c_uint32(0)
        _lib.check(lib().kdb_hstable_writer_file_count(self.h, ctypes.byref(c)), "file_count")
        tot = 0
        for i in range(c.value):
            fid, p, sz = ctypes.c_uint32(), ctypes.c_void_p(), ctypes.c_uint64()
            _lib.check(lib().kdb_hstable_writer_file(self.h, i, ctypes.byref(fid), ctypes.byref(p), ctypes.byref(sz)),
                       "file")
            tot += sz.value
        return tot

    def save(self, directory: str) -> None:
        _lib.check(lib().kdb_hstable_writer_save(self.h, directory.encode()), "hstable_writer_save")

    def __del__(self):
        try:
            if self.h:
                lib().kdb_hstable_writer_destroy(self.h)
                self.h = None
        except Exception:
            pass


def db_options(hstable_size: int = 32 << 20, hash_type: int = 1) -> bytes:
    """The 48-byte db_options file (DatabaseOptionEncoder, storage/format.h:324-340)."""
    out = np.zeros(48, np.uint8)
    _lib.check(lib().kdb_hstable_db_options(hstable_size, hash_type, out.ctypes.data), "db_options")
    return out.tobytes()


def write_hstables(puts, hstable_size: int = 32 << 20, hash_type: int = 1, batch: int | None = None
                   ) -> dict[str, bytes]:
    """The HSTable files KingDB writes for `puts` (one writer thread), with
    the puts handed to the GPU `batch` at a time (one write-buffer flush each)."""
    w = HSTableWriter(hstable_size, hash_type)
    step = batch or max(len(puts), 1)
    for i in range(0, len(puts), step):
        w.append(put_entries(puts[i:i + step], hash_type))
    w.close()
    return w.files()
