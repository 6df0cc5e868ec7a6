"""Python face of the gfx950 LZ4 codec (a thin layer over include/kdb_lz4.h).

Mirrors the reference's operator interface for this path:
  * ``compress_bound``, ``compress_limited_output``, ``decompress_safe_partial``
    -- LZ4 r1.3.0 (algorithm/lz4.h:115,129,169), same return conventions;
  * ``compress_frames`` / ``decompress_frames`` -- CompressorLZ4::Compress /
    Uncompress frames (algorithm/compressor.cc:15-137), batched;
  * ``DeviceBatch`` -- device-resident batches for the benchmark and for
    callers that keep values in HBM.

Every call runs the HIP kernels; nothing here computes LZ4 on the CPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib



def lib():
    return _lib.load()


def compress_bound(n: int) -> int:
    return lib().kdb_lz4_compressBound(n)


def frame_bound(n: int) -> int:
    return int(lib().kdb_lz4_frame_bound(n))


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().kdb_lz4_device_count(ctypes.byref(n))
    return n.value if rc == _lib.OK else 0


def set_device(dev: int) -> None:
    _lib.check(lib().kdb_lz4_set_device(dev), "set_device")


def get_device() -> int:
    d = ctypes.c_int(-1)
    _lib.check(lib().kdb_lz4_get_device(ctypes.byref(d)), "get_device")
    return d.value


def selftest(dev: int) -> tuple:
    """(state, bad_lanes) of the device's lane-order self-test (kdb_lz4_selftest):
    state 1 passed, -1 failed, 0 not run."""
    st, bad = ctypes.c_int(0), ctypes.c_uint32(0)
    _lib.check(lib().kdb_lz4_selftest(dev, ctypes.byref(st), ctypes.byref(bad)), "selftest")
    return st.value, bad.value


def last_kernels() -> list:
    """Kernels (rocprof names) the calling thread's last compress/decompress batch queued."""
    buf = ctypes.create_string_buffer(1024)
    _lib.check(lib().kdb_lz4_last_kernels(buf, len(buf)), "last_kernels")
    return [k for k in buf.value.decode().split(";") if k]


def build_id() -> str:
    """Hash of the sources the loaded library was compiled from (kdb_lz4_build_id)."""
    buf = ctypes.create_string_buffer(64)
    _lib.check(lib().kdb_lz4_build_id(buf, len(buf)), "build_id")
    return buf.value.decode()


# ------------------------------------------------------------ device memory
class DeviceBuffer:
    """A hipMalloc'd byte range owned by Python."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _lib.check(lib().kdb_lz4_malloc(ctypes.byref(p), max(self.nbytes, 1)), "kdb_lz4_malloc")
        self.ptr = p.value

    def free(self) -> None:
        if self.ptr:
            lib().kdb_lz4_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr: np.ndarray, offset: int = 0, stream=None) -> None:
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        _lib.check(lib().kdb_lz4_memcpy_h2d(self.ptr + offset, a.ctypes.data, a.nbytes, stream), "h2d")
        if stream is None:
            _lib.check(lib().kdb_lz4_stream_sync(None), "sync")

    def download(self, nbytes: int | None = None, offset: int = 0, dtype=np.uint8, stream=None) -> np.ndarray:
        nb = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(nb, dtype=np.uint8)
        if nb:
            _lib.check(lib().kdb_lz4_memcpy_d2h(out.ctypes.data, self.ptr + offset, nb, stream), "d2h")
        _lib.check(lib().kdb_lz4_stream_sync(stream), "sync")
        return out.view(dtype)

    def memset(self, value: int = 0, stream=None) -> None:
        _lib.check(lib().kdb_lz4_memset(self.ptr, value, self.nbytes, stream), "memset")


class Stream:
    def __init__(self):
        p = ctypes.c_void_p()
        _lib.check(lib().kdb_lz4_stream_create(ctypes.byref(p)), "stream_create")
        self.ptr = p.value

    def sync(self) -> None:
        _lib.check(lib().kdb_lz4_stream_sync(self.ptr), "stream_sync")

    def __del__(self):
        try:
            if self.ptr:
                lib().kdb_lz4_stream_destroy(self.ptr)
        except Exception:
            pass


class Event:
    def __init__(self):
        p = ctypes.c_void_p()
        _lib.check(lib().kdb_lz4_event_create(ctypes.byref(p)), "event_create")
        self.ptr = p.value

    def record(self, stream: "Stream | None" = None) -> None:
        _lib.check(lib().kdb_lz4_event_record(self.ptr, stream.ptr if stream else None), "event_record")

    def elapsed_ms(self, end: "Event") -> float:
        _lib.check(lib().kdb_lz4_event_sync(end.ptr), "event_sync")
        ms = ctypes.c_float(0)
        _lib.check(lib().kdb_lz4_event_elapsed_ms(self.ptr, end.ptr, ctypes.byref(ms)), "elapsed")
        return ms.value

    def __del__(self):
        try:
            if self.ptr:
                lib().kdb_lz4_event_destroy(self.ptr)
        except Exception:
            pass


def _a16(x):
    return (np.asarray(x, dtype=np.uint64) + 15) & ~np.uint64(15)


def _pack(values: list[bytes], slot: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate values into 16-aligned slots; returns (buffer, offsets)."""
    slot = _a16(slot)
    off = np.zeros(len(values), dtype=np.uint64)
    if len(values) > 1:
        off[1:] = np.cumsum(slot[:-1])
    total = int(slot.sum()) if len(values) else 0
    buf = np.zeros(max(total, 16), dtype=np.uint8)
    for v, o in zip(values, off):
        if len(v):
            buf[int(o): int(o) + len(v)] = np.frombuffer(v, dtype=np.uint8)
    return buf, off


# ------------------------------------------------------------- scalar mirrors
def compress_limited_output(data: bytes, max_out: int) -> tuple[int, bytes]:
    """LZ4_compress_limitedOutput on the GPU: (ret, block[:ret])."""
    dst = ctypes.create_string_buffer(max(max_out, 1))
    r = lib().kdb_lz4_compress_limitedOutput(data, ctypes.addressof(dst), len(data), max_out)
    return r, dst.raw[: max(r, 0)]


def decompress_safe_partial(block: bytes, target: int, max_out: int) -> tuple[int, bytes]:
    """LZ4_decompress_safe_partial on the GPU: (ret, out[:ret])."""
    dst = ctypes.create_string_buffer(max(max_out, 1))
    r = lib().kdb_lz4_decompress_safe_partial(block, ctypes.addressof(dst), len(block), target, max_out)
    return r, dst.raw[: max(r, 0)]


# -------------------------------------------------------------------- batches
def compress_blocks(values: list[bytes], caps: list[int] | None = None) -> list[tuple[int, bytes]]:
    """LZ4_compress_limitedOutput per value (one launch): [(ret, block)]."""
    n = len(values)
    if n == 0:
        return []
    lens = np.array([len(v) for v in values], dtype=np.uint32)
    caps_a = np.array([compress_bound(len(v)) for v in values] if caps is None else caps, dtype=np.uint32)
    src, src_off = _pack(values, lens.astype(np.uint64) + 16)
    dst_off = np.zeros(n, dtype=np.uint64)
    slots = _a16(caps_a.astype(np.uint64) + 16)
    if n > 1:
        dst_off[1:] = np.cumsum(slots[:-1])
    dbytes = int(slots.sum())
    d_src = DeviceBuffer(src.nbytes)
    d_src.upload(src)
    d_dst = DeviceBuffer(dbytes)
    meta = DeviceBuffer(n * (8 + 4 + 8 + 4 + 4))
    m = np.concatenate([src_off.view(np.uint8), lens.view(np.uint8), dst_off.view(np.uint8),
                        caps_a.view(np.uint8), np.zeros(4 * n, np.uint8)])
    meta.upload(m)
    b = meta.ptr
    _lib.check(lib().kdb_lz4_compress_blocks_batch(
        None, d_src.ptr, b, b + 8 * n, n, int(lens.max()), d_dst.ptr, b + 12 * n, b + 20 * n, b + 24 * n),
        "compress_blocks_batch")
    out = d_dst.download()
    ret = meta.download(4 * n, 24 * n).view(np.int32)
    res = []
    for i in range(n):
        r = int(ret[i])
        o = int(dst_off[i])
        res.append((r, out[o:o + max(r, 0)].tobytes()))
    return res


def decompress_blocks(blocks: list[bytes], sizes: list[int], targets: list[int] | None = None
                      ) -> list[tuple[int, bytes]]:
    """LZ4_decompress_safe_partial(block, dst, len, target, size) per value (one launch)."""
    n = len(blocks)
    if n == 0:
        return []
    inl = np.array([len(b) for b in blocks], dtype=np.uint32)
    caps = np.array(sizes, dtype=np.uint32)
    tg = np.array(sizes if targets is None else targets, dtype=np.int64).astype(np.int32).view(np.uint32)
    src, src_off = _pack(blocks, inl.astype(np.uint64) + 16)
    slots = _a16(caps.astype(np.uint64) + 16)
    dst_off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        dst_off[1:] = np.cumsum(slots[:-1])
    d_src = DeviceBuffer(src.nbytes)
    d_src.upload(src)
    d_dst = DeviceBuffer(int(slots.sum()))
    meta = DeviceBuffer(n * (8 + 4 + 8 + 4 + 4 + 4))
    m = np.concatenate([src_off.view(np.uint8), inl.view(np.uint8), dst_off.view(np.uint8),
                        caps.view(np.uint8), tg.view(np.uint8), np.zeros(4 * n, np.uint8)])
    meta.upload(m)
    b = meta.ptr
    _lib.check(lib().kdb_lz4_decompress_blocks_batch(
        None, d_src.ptr, b, b + 8 * n, n, int(inl.max()), int(caps.max()), d_dst.ptr, b + 12 * n,
        b + 20 * n, b + 24 * n, b + 28 * n), "decompress_blocks_batch")
    out = d_dst.download()
    ret = meta.download(4 * n, 28 * n).view(np.int32)
    res = []
    for i in range(n):
        r = int(ret[i])
        o = int(dst_off[i])
        res.append((r, out[o:o + max(r, 0)].tobytes()))
    return res


def compress_frames(values: list[bytes], max_len: int | None = None) -> list[bytes]:
    """CompressorLZ4::Compress per value (one launch); raises on IOError.
    max_len: the launch's bound on the values' lengths (default: the largest)."""
    n = len(values)
    if n == 0:
        return []
    lens = np.array([len(v) for v in values], dtype=np.uint32)
    src, src_off = _pack(values, lens.astype(np.uint64) + 16)
    slots = _a16(np.array([frame_bound(int(x)) for x in lens], dtype=np.uint64))
    dst_off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        dst_off[1:] = np.cumsum(slots[:-1])
    d_src = DeviceBuffer(src.nbytes)
    d_src.upload(src)
    d_dst = DeviceBuffer(int(slots.sum()))
    meta = DeviceBuffer(n * (8 + 4 + 8 + 4 + 4))
    m = np.concatenate([src_off.view(np.uint8), lens.view(np.uint8), dst_off.view(np.uint8),
                        np.zeros(8 * n, np.uint8)])
    meta.upload(m)
    b = meta.ptr
    _lib.check(lib().kdb_lz4_compress_frames_batch(
        None, d_src.ptr, b, b + 8 * n, n, int(lens.max()) if max_len is None else max_len, d_dst.ptr, b + 12 * n,
        b + 20 * n, b + 24 * n), "compress_frames_batch")
    out = d_dst.download()
    md = meta.download(8 * n, 20 * n)
    flen = md[: 4 * n].view(np.uint32)
    st = md[4 * n:].view(np.int32)
    res = []
    for i in range(n):
        if st[i] != 0:
            raise _lib.HipError(f"LZ4_compress_limitedOutput() failed for value {i} (status {st[i]})")
        o = int(dst_off[i])
        res.append(out[o:o + int(flen[i])].tobytes())
    return res


def decompress_frames(frames: list[bytes], sizes: list[int]) -> list[tuple[int, bytes]]:
    """CompressorLZ4::Uncompress of one frame per value: [(status, data)]."""
    n = len(frames)
    if n == 0:
        return []
    avail = np.array([len(f) for f in frames], dtype=np.uint32)
    caps = np.array(sizes, dtype=np.uint32)
    src, src_off = _pack(frames, avail.astype(np.uint64) + 16)
    slots = _a16(caps.astype(np.uint64) + 16)
    dst_off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        dst_off[1:] = np.cumsum(slots[:-1])
    d_src = DeviceBuffer(src.nbytes)
    d_src.upload(src)
    d_dst = DeviceBuffer(int(slots.sum()))
    meta = DeviceBuffer(n * (8 + 4 + 8 + 4 + 4 + 4))
    m = np.concatenate([src_off.view(np.uint8), avail.view(np.uint8), dst_off.view(np.uint8),
                        caps.view(np.uint8), np.zeros(8 * n, np.uint8)])
    meta.upload(m)
    b = meta.ptr
    _lib.check(lib().kdb_lz4_decompress_frames_batch(
        None, d_src.ptr, b, b + 8 * n, n, int(avail.max()), int(caps.max()), d_dst.ptr, b + 12 * n,
        b + 20 * n, b + 24 * n, b + 28 * n), "decompress_frames_batch")
    out = d_dst.download()
    md = meta.download(8 * n, 24 * n)
    olen = md[: 4 * n].view(np.uint32)
    st = md[4 * n:].view(np.int32)
    return [(int(st[i]), out[int(dst_off[i]):int(dst_off[i]) + int(olen[i])].tobytes()) for i in range(n)]


# ------------------------------------------------------ device-resident batch
# the mixed batch, by count 90% 100 B values, 9% 4 KiB
# values and 1% 64 KiB parts (network/server.cc:258 cuts 64 KiB parts).
MIX_CONFIG4 = ((100, 0.90), (4096, 0.09), (65536, 0.01))


def mixed_sizes(n: int, mix=MIX_CONFIG4, seed: int = 4) -> np.ndarray:
    """n value sizes with the given by-count mix, in a seeded shuffled order
    (the exact counts are round(n * share), the remainder going to the first class)."""
    counts = [int(round(n * f)) for _, f in mix]
    counts[0] += n - sum(counts)
    sizes = np.concatenate([np.full(c, sz, np.uint32) for (sz, _), c in zip(mix, counts)])
    np.random.default_rng(seed).shuffle(sizes)
    return sizes


@dataclass
class DeviceBatch:
    """A batch of n values resident in HBM (sizes may differ per value), with
    frame slots and the metadata arrays the kernels take.  Values are packed
    back to back in `src`; decoded values land at the same offsets in `out`.
    Used by bench.py and the large parity tests; nothing here touches host
    memory after construction."""

    n: int
    size: int                  # largest value size of the batch
    sizes: np.ndarray          # u32 per value
    src_off: np.ndarray        # u64 per value (same offsets in `out`)
    frame_off: np.ndarray      # u64 per value (16-aligned frame slots)
    src: DeviceBuffer
    frames: DeviceBuffer
    out: DeviceBuffer
    meta: DeviceBuffer
    slot: int                  # largest frame slot
    max_in: int = 0            # largest frame decompress() is told to expect (0: the slot)
    exact_max_in: bool = False # decompress(): find the largest frame on the device first (one 4-byte read back)

    @property
    def raw_bytes(self) -> int:
        return int(self.sizes.astype(np.int64).sum())

    @classmethod
    def g1_long(cls, n: int, size: int, first_piece: int = 0, stream: Stream | None = None) -> "DeviceBatch":
        """n consecutive `size`-byte slices of the G1-long pool (piece-aligned start)."""
        return cls.g1_long_sizes(np.full(n, size, np.uint32), first_piece=first_piece, stream=stream)

    @classmethod
    def g1_long_sizes(cls, sizes: np.ndarray, first_piece: int = 0, stream: Stream | None = None) -> "DeviceBatch":
        """Values of the given sizes, consecutive slices of the G1-long pool."""
        sizes = np.asarray(sizes, dtype=np.uint32)
        total = int(sizes.astype(np.int64).sum())
        npieces = (total + 99) // 100
        src = DeviceBuffer(npieces * 100 + 64)
        st = stream.ptr if stream else None
        _lib.check(lib().kdb_lz4_gen_g1(src.ptr, first_piece, npieces, 301, st), "gen_g1")
        return cls._layout(sizes, src, stream)

    @classmethod
    def from_host(cls, values: np.ndarray, size: int, stream: Stream | None = None) -> "DeviceBatch":
        n = values.nbytes // size
        src = DeviceBuffer(values.nbytes + 64)
        src.upload(values)
        return cls._layout(np.full(n, size, np.uint32), src, stream)

    @classmethod
    def _layout(cls, sizes: np.ndarray, src: DeviceBuffer, stream) -> "DeviceBatch":
        n = len(sizes)
        src_off = np.zeros(n, dtype=np.uint64)
        if n > 1:
            src_off[1:] = np.cumsum(sizes[:-1].astype(np.uint64))
        uniq, inv = np.unique(sizes, return_inverse=True)
        fslot = np.array([frame_bound(int(x)) for x in uniq], dtype=np.uint64)
        slots = ((fslot + 15) & ~np.uint64(15))[inv]
        frame_off = np.zeros(n, dtype=np.uint64)
        if n > 1:
            frame_off[1:] = np.cumsum(slots[:-1])
        frames = DeviceBuffer(int(slots.sum()) + 64)
        out = DeviceBuffer(src.nbytes)
        # meta: src_off u64 | len u32 | frame_off u64 | frame_len u32 | status i32 |
        #       out_off u64 | out_cap u32 | out_len u32 | dstatus i32
        m = np.concatenate([
            src_off.view(np.uint8),
            sizes.view(np.uint8),
            frame_off.view(np.uint8),
            np.zeros(n, np.uint32).view(np.uint8),
            np.zeros(n, np.int32).view(np.uint8),
            src_off.view(np.uint8),
            sizes.view(np.uint8),
            np.zeros(n, np.uint32).view(np.uint8),
            np.zeros(n, np.int32).view(np.uint8),
        ])
        meta = DeviceBuffer(m.nbytes)
        meta.upload(m, stream=stream.ptr if stream else None)
        if stream:
            stream.sync()
        return cls(n=n, size=int(sizes.max()) if n else 0, sizes=sizes, src_off=src_off, frame_off=frame_off,
                   src=src, frames=frames, out=out, meta=meta, slot=int(slots.max()) if n else 16)

    # metadata views (device pointers)
    def _p(self, k: int) -> int:
        n = self.n
        offs = [0, 8 * n, 12 * n, 20 * n, 24 * n, 28 * n, 36 * n, 40 * n, 44 * n]
        return self.meta.ptr + offs[k]

    def compress(self, stream: Stream | None = None) -> None:
        _lib.check(lib().kdb_lz4_compress_frames_batch(
            stream.ptr if stream else None, self.src.ptr, self._p(0), self._p(1), self.n, self.size,
            self.frames.ptr, self._p(2), self._p(3), self._p(4)), "compress_frames_batch")

    def largest_frame(self, stream: Stream | None = None) -> int:
        """The largest frame length of the batch, reduced on the device
        (kdb_lz4_max_u32) and read back: the max_in a caller with no host copy
        of the frame lengths passes to the decoder."""
        if getattr(self, "_maxbuf", None) is None:
            self._maxbuf = DeviceBuffer(4)
        st = stream.ptr if stream else None
        _lib.check(lib().kdb_lz4_max_u32(st, self._p(3), self.n, self._maxbuf.ptr), "max_u32")
        v = ctypes.c_uint32(0)
        _lib.check(lib().kdb_lz4_memcpy_d2h(ctypes.addressof(v), self._maxbuf.ptr, 4, st), "d2h")
        _lib.check(lib().kdb_lz4_stream_sync(st), "sync")
        return int(v.value)

    def decompress(self, stream: Stream | None = None) -> None:
        if self.exact_max_in:
            # the decoder's LDS staging is sized by max_in: the frames' true
            # largest (about 0.56 x 4 KiB for G1) instead of the slot bound
            # (8 + compressBound) leaves room for more waves per CU
            self.max_in = max(self.largest_frame(stream), 1)
        _lib.check(lib().kdb_lz4_decompress_frames_batch(
            stream.ptr if stream else None, self.frames.ptr, self._p(2), self._p(3), self.n,
            self.max_in or self.slot, self.size, self.out.ptr, self._p(5), self._p(6), self._p(7), self._p(8)),
            "decompress_frames_batch")

    def frame_lens(self) -> np.ndarray:
        return self.meta.download(4 * self.n, 20 * self.n).view(np.uint32)

    def status(self) -> tuple[np.ndarray, np.ndarray]:
        c = self.meta.download(4 * self.n, 24 * self.n).view(np.int32)
        d = self.meta.download(4 * self.n, 44 * self.n).view(np.int32)
        return c, d

    def out_lens(self) -> np.ndarray:
        return self.meta.download(4 * self.n, 40 * self.n).view(np.uint32)

    def poison(self, stream: Stream | None = None) -> None:
        """Overwrite every output of compress() and decompress() -- frame slots,
        decoded bytes, frame lengths, decoded lengths and both status words --
        with bytes no correct pass leaves there (0xA5 / all ones), so that a
        later roundtrip_ok() proves the passes after this call wrote them."""
        st = stream.ptr if stream else None
        n = self.n
        for ptr, nbytes, val in ((self.frames.ptr, self.frames.nbytes, 0xA5), (self.out.ptr, self.out.nbytes, 0xA5),
                                 (self._p(3), 8 * n, 0xFF), (self._p(7), 8 * n, 0xFF)):
            _lib.check(lib().kdb_lz4_memset(ptr, val, nbytes, st), "memset")

    def roundtrip_ok(self) -> bool:
        """Every status 0, every decoded length right, every decoded byte equal."""
        cst, dst = self.status()
        if not ((cst == 0).all() and (dst == 0).all() and np.array_equal(self.out_lens(), self.sizes)):
            return False
        t = self.raw_bytes
        return bool(np.array_equal(self.src.download(t), self.out.download(t)))

    def free(self) -> None:
        for b in (self.src, self.frames, self.out, self.meta, getattr(self, "_maxbuf", None)):
            if b is not None:
                b.free()
