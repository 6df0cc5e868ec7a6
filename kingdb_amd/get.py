"""The read path around the codec (kdb_get_values_batch, csrc/get.hip):
CompressorLZ4::UncompressByteArray for a batch of stored values, plus the
HSTable entry reader that finds them.

  read_hstable(bytes)         the entries of one HSTable file (EntryHeader::DecodeFrom,
                              storage/format.h:182-222; offset array, hstable_manager.h:380-420)
  get_values(items, verify)   GPU batch decode: [(status, value bytes)]

status: 0 OK, -1 IOError (a frame failed to decode, or sizes outside the
value), -2 IOError "Invalid checksum." (verify 1 = the reference's check with
its double-streamed CRC, 2 = the corrected one).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

from . import _lib
from .lz4 import DeviceBuffer, Stream

HEADER_SIZE = 8192
MAGIC = 0x4D454F57


def lib():
    return _lib.load()


def _varint(b: bytes, i: int) -> tuple[int, int]:
    v, s = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 127) << s
        if c < 128:
            return v, i
        s += 7


@dataclass
class Entry:
    offset: int                # entry offset in the file
    flags: int
    checksum: int
    key: bytes
    size_value: int
    size_value_compressed: int
    size_padding: int
    hashed: int
    value_at: int              # file offset of the value region
    header_size: int

    @property
    def stored_len(self) -> int:
        """Bytes of the value region that hold data (EntryHeader::size_value_used)."""
        return self.size_value_compressed if self.size_value_compressed else self.size_value


def decode_entry(f: bytes, off: int) -> Entry:
    """EntryHeader::DecodeFrom with compression on (storage/format.h:182-222)."""
    (checksum,) = struct.unpack_from("<I", f, off + 1)
    i = off + 5
    flags, i = _varint(f, i)
    klen, i = _varint(f, i)
    size, i = _varint(f, i)
    (svc,) = struct.unpack_from("<Q", f, i)
    i += 8
    pad, i = _varint(f, i)
    (hashed,) = struct.unpack_from("<Q", f, i)
    i += 8
    return Entry(off, flags, checksum, f[i:i + klen], size, svc, pad, hashed, i + klen, i - off)


def read_hstable(f: bytes) -> list[Entry]:
    """Every entry the file's offset array lists, in order (HSTableFooter,
    storage/format.h:480-493; rows: varint64 hash, varint32 offset)."""
    if len(f) < HEADER_SIZE + 36:
        return []
    ftype, fflags, oidx, num, magic = struct.unpack_from("<IIQQQ", f, len(f) - 36)
    if magic != MAGIC:
        # no offset array (a multipart entry never finished, hstable_manager.h:361-378):
        # walk the entries from the header block, as recovery would
        out, o = [], HEADER_SIZE
        while o < len(f):
            e = decode_entry(f, o)
            out.append(e)
            o = e.value_at + (e.size_value + e.size_padding if (e.flags & 0x2) else e.stored_len)
        return out
    out, i = [], oidx
    for _ in range(num):
        _, i = _varint(f, i)
        o, i = _varint(f, i)
        out.append(decode_entry(f, o))
    return out


def get_values(items, verify: int = 0, stream: Stream | None = None,
               frame_cap: int | None = None) -> list[tuple[int, bytes]]:
    """items: (stored bytes, size_value_compressed, size_value[, checksum, checksum_initial]).
    One GPU batch of CompressorLZ4::UncompressByteArray."""
    n = len(items)
    if n == 0:
        return []
    stored = [it[0] for it in items]
    avail = np.array([len(s) for s in stored], np.uint64)
    svc = np.array([it[1] for it in items], np.uint64)
    size = np.array([it[2] for it in items], np.uint64)
    ck = np.array([it[3] if len(it) > 3 else 0 for it in items], np.uint32)
    ci = np.array([it[4] if len(it) > 4 else 0 for it in items], np.uint32)
    soff = np.zeros(n, np.uint64)
    soff[1:] = np.cumsum((avail[:-1] + 63) & ~np.uint64(63))
    sbytes = int(soff[-1] + avail[-1]) + 64
    buf = np.zeros(sbytes, np.uint8)
    for s, o in zip(stored, soff):
        buf[int(o):int(o) + len(s)] = np.frombuffer(s, np.uint8)
    ooff = np.zeros(n, np.uint64)
    ooff[1:] = np.cumsum((size[:-1] + 63) & ~np.uint64(63))
    obytes = int(ooff[-1] + size[-1]) + 64
    # frames are at least 8 bytes: Σ(avail/8 + 1) bounds them (values KingDB
    # writes hold one frame per part, far fewer)
    if frame_cap is None:   # frames are >= 8 bytes: this many always suffice
        frame_cap = int((avail // 8 + 1).sum())
        if frame_cap > (4 << 20):
            frame_cap = max(4 * n + int(avail.sum()) // 4096, 4 << 20)
    max_in = int(avail.max())
    max_out = int(size.max()) if n else 0
    sb = int(lib().kdb_get_scratch_bytes(n, frame_cap))
    d_st, d_out, d_scr = DeviceBuffer(sbytes), DeviceBuffer(obytes), DeviceBuffer(sb)
    meta = DeviceBuffer(n * (8 * 5 + 4 * 2 + 8 + 4))
    try:
        st = stream.ptr if stream else None
        d_st.upload(buf, stream=st)
        m = np.concatenate([soff.view(np.uint8), avail.view(np.uint8), svc.view(np.uint8), size.view(np.uint8),
                            ooff.view(np.uint8), ck.view(np.uint8), ci.view(np.uint8)])
        meta.upload(m, stream=st)
        b = meta.ptr
        p_outlen, p_status = b + 48 * n, b + 56 * n
        _lib.check(lib().kdb_get_values_batch(
            st, d_st.ptr, b, b + 8 * n, b + 16 * n, b + 24 * n, n, d_out.ptr, b + 32 * n, verify, b + 40 * n,
            b + 44 * n, frame_cap, max_in, max_out, d_scr.ptr, sb, p_outlen, p_status), "kdb_get_values_batch")
        # the copies back ride the same stream (a download on the null stream
        # would not wait for a non-blocking caller stream)
        res = meta.download(12 * n, 48 * n, stream=st)
        olen = res[: 8 * n].view(np.uint64)
        stat = res[8 * n:].view(np.int32)
        out = d_out.download(obytes, stream=st)
        return [(int(stat[i]), out[int(ooff[i]):int(ooff[i]) + int(olen[i])].tobytes()) for i in range(n)]
    finally:
        for d in (d_st, d_out, d_scr, meta):
            d.free()


def entry_items(f: bytes, entries: list[Entry] | None = None, crc32c=None):
    """get_values() items for a file's entries: the value region as stored,
    with checksum and checksum_initial = crc32c(key) when `crc32c` is given."""
    entries = read_hstable(f) if entries is None else entries
    items = []
    for e in entries:
        region = e.size_value + e.size_padding if (e.flags & 0x2) else e.stored_len
        stored = f[e.value_at:e.value_at + region]
        ci = crc32c(e.key) if crc32c else 0
        items.append((stored, e.size_value_compressed, e.size_value, e.checksum, ci))
    return items
