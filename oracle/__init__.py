"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU restatement of KingDB's LZ4 r1.3.0 codec
(`oracle/lz4_oracle.c`) and, where it has been built in this container, for
the reference's own codec (`oracle/_ref/libkdbref.so`, built from
/root/reference by `make -C oracle ref`).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product package `kingdb_amd` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liblz4_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libkdbref.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(ref: bool = False) -> None:
    """Compile the oracle (and, if asked and /root/reference exists, _ref)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


class Oracle:
    """The C restatement (lz4_oracle.c)."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        lib.orc_compress_bound.argtypes = [ctypes.c_int]
        lib.orc_compress_bound.restype = ctypes.c_int
        lib.orc_compress_limited.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int]
        lib.orc_compress_limited.restype = ctypes.c_int
        lib.orc_decompress_safe_partial.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.orc_decompress_safe_partial.restype = ctypes.c_int
        lib.orc_crc32c_extend.argtypes = [ctypes.c_uint32, _u8p, ctypes.c_size_t]
        lib.orc_crc32c_extend.restype = ctypes.c_uint32
        lib.orc_frame_compress.argtypes = [_u8p, ctypes.c_uint64, _u8p]
        lib.orc_frame_compress.restype = ctypes.c_int64
        lib.orc_frame_uncompress.argtypes = [_u8p, _u8p, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_uint64)]
        lib.orc_frame_uncompress.restype = ctypes.c_int
        lib.orc_g1_pieces.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u8p]
        lib.orc_g1_pieces.restype = None
        c = ctypes
        lib.orc_crc8.argtypes = [c.c_uint, _u8p, c.c_size_t]
        lib.orc_crc8.restype = c.c_uint8
        lib.orc_xxh64.argtypes = [_u8p, c.c_size_t, c.c_uint64]
        lib.orc_xxh64.restype = c.c_uint64
        lib.orc_murmur3_64.argtypes = [_u8p, c.c_size_t]
        lib.orc_murmur3_64.restype = c.c_uint64
        lib.orc_entry_header.argtypes = [c.c_uint32, c.c_uint32, c.c_uint64, c.c_uint64, c.c_uint64, c.c_uint64,
                                         c.c_uint64, _u8p]
        lib.orc_entry_header.restype = c.c_int
        lib.orc_padding.argtypes = [c.c_uint64]
        lib.orc_padding.restype = c.c_uint64
        lib.orc_put_value.argtypes = [_u8p, c.c_uint32, _u8p, c.c_uint64, ctypes.POINTER(c.c_uint32), c.c_uint32,
                                      _u8p, ctypes.POINTER(c.c_uint64), ctypes.POINTER(c.c_uint32),
                                      ctypes.POINTER(c.c_uint64), ctypes.POINTER(c.c_uint32)]
        lib.orc_put_value.restype = c.c_int
        lib.orc_get_value.argtypes = [_u8p, c.c_uint64, c.c_uint64, c.c_uint64, c.c_uint32, c.c_uint32, c.c_int, _u8p,
                                      ctypes.POINTER(c.c_uint64)]
        lib.orc_get_value.restype = c.c_int
        lib.orc_put_part.argtypes = [c.c_void_p, _u8p, c.c_uint32, _u8p, c.c_uint64, c.c_uint64, c.c_uint64, _u8p,
                                     ctypes.POINTER(c.c_uint32), ctypes.POINTER(c.c_uint64),
                                     ctypes.POINTER(c.c_uint64), ctypes.POINTER(c.c_uint64),
                                     ctypes.POINTER(c.c_uint32)]
        lib.orc_put_part.restype = c.c_int
        self.lib = lib

    def compress_bound(self, n: int) -> int:
        return self.lib.orc_compress_bound(n)

    def compress(self, data: bytes, max_out: int | None = None) -> bytes | None:
        """LZ4_compress_limitedOutput; None where the reference returns 0."""
        src = np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        cap = self.compress_bound(len(data)) if max_out is None else max_out
        # r1.3.0 limitedOutput can run past max_out on chains of zero-literal
        # sequences before a later check returns 0, so size the scratch by bound.
        dst = np.zeros(max(cap, self.compress_bound(len(data)), 1) + 64, dtype=np.uint8)
        r = self.lib.orc_compress_limited(_ptr(src), _ptr(dst), len(data), cap)
        return None if r == 0 else dst[:r].tobytes()

    def decompress(self, block: bytes, size: int, target: int | None = None) -> tuple[int, bytes]:
        """LZ4_decompress_safe_partial(block, dst, len(block), target, size); target defaults to size."""
        src = np.zeros(len(block) + 64, dtype=np.uint8)
        src[: len(block)] = np.frombuffer(block, dtype=np.uint8)
        dst = np.zeros(size + 64, dtype=np.uint8)
        r = self.lib.orc_decompress_safe_partial(_ptr(src), _ptr(dst), len(block), size if target is None else target,
                                                 size)
        return r, (dst[:r].tobytes() if r > 0 else b"")

    def frame(self, data: bytes) -> bytes:
        """CompressorLZ4::Compress frame bytes."""
        src = np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        out = np.zeros(8 + max(self.compress_bound(len(data)), len(data)) + 64, dtype=np.uint8)
        n = self.lib.orc_frame_compress(_ptr(src), len(data), _ptr(out))
        if n < 0:
            raise RuntimeError("LZ4_compress_limitedOutput() failed")
        return out[:n].tobytes()

    def crc32c(self, data: bytes, crc: int = 0) -> int:
        a = np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        return self.lib.orc_crc32c_extend(crc, _ptr(a), len(data))

    def crc32c_array(self, a: np.ndarray, crc: int = 0) -> int:
        """CRC32C of a contiguous uint8 array, no copy (GB-sized streams)."""
        a = np.ascontiguousarray(a, dtype=np.uint8)
        return self.lib.orc_crc32c_extend(crc, _ptr(a), a.nbytes) if a.nbytes else crc

    def frames_digest(self, src: np.ndarray, off: np.ndarray, lens: np.ndarray) -> tuple[int, int]:
        """(sum of frame bytes, CRC32C of the frames concatenated) of CompressorLZ4
        frames of values src[off[i] .. +lens[i]) (tests/golden/digests.json)."""
        return _digest(self.lib.orc_frames_digest, src, off, lens)

    def g1_pieces(self, npieces: int, seed: int = 301) -> np.ndarray:
        out = np.empty(npieces * 100, dtype=np.uint8)
        self.lib.orc_g1_pieces(seed, npieces, _ptr(out))
        return out

    # ------------------------------------------------ write path
    @staticmethod
    def _buf(data: bytes) -> np.ndarray:
        return np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)

    def crc8(self, data: bytes, crc: int = 0) -> int:
        return self.lib.orc_crc8(crc, _ptr(self._buf(data)), len(data))

    def xxh64(self, data: bytes, seed: int = 0) -> int:
        return self.lib.orc_xxh64(_ptr(self._buf(data)), len(data), seed)

    def murmur3_64(self, data: bytes) -> int:
        return self.lib.orc_murmur3_64(_ptr(self._buf(data)), len(data))

    def entry_header(self, crc: int, flags: int, size_key: int, size_value: int, svc: int, padding: int,
                     hashed: int) -> bytes:
        out = np.zeros(64, np.uint8)
        n = self.lib.orc_entry_header(crc, flags, size_key, size_value, svc, padding, hashed, _ptr(out))
        return out[:n].tobytes()

    def padding(self, size_value: int) -> int:
        return self.lib.orc_padding(size_value)

    def get_value(self, stored: bytes, svc: int, size: int, checksum: int = 0, checksum_initial: int = 0,
                  verify: int = 0) -> tuple[int, bytes]:
        """CompressorLZ4::UncompressByteArray of one stored value: (status, defined output bytes)."""
        src = np.zeros(len(stored) + 64, np.uint8)
        src[: len(stored)] = np.frombuffer(stored, np.uint8)
        out = np.zeros(size + 64, np.uint8)
        n = ctypes.c_uint64(0)
        st = self.lib.orc_get_value(_ptr(src), len(stored), svc, size, checksum, checksum_initial, verify, _ptr(out),
                                    ctypes.byref(n))
        return st, out[: n.value].tobytes()

    def put_value(self, key: bytes, value: bytes, chunks: list[int] | None = None) -> dict:
        """Database::PutPart over `chunks` (default: one chunk) of one value:
        {"parts": [(offset_chunk_compressed, chunk_final bytes)], "svc", "crc",
        "stored": the value region (size_value + padding bytes)}; raises on IOError."""
        chunks = [len(value)] if chunks is None else list(chunks)
        assert sum(chunks) == len(value)
        n = len(chunks)
        cl = (ctypes.c_uint32 * max(n, 1))(*chunks)
        po = (ctypes.c_uint64 * max(n, 1))()
        pl = (ctypes.c_uint32 * max(n, 1))()
        svc, crc = ctypes.c_uint64(0), ctypes.c_uint32(0)
        stored = np.zeros(len(value) + self.padding(len(value)) + 64, np.uint8)
        rc = self.lib.orc_put_value(_ptr(self._buf(key)), len(key), _ptr(self._buf(value)), len(value), cl, n,
                                    _ptr(stored), po, pl, ctypes.byref(svc), ctypes.byref(crc))
        if rc != 0:
            raise RuntimeError("PutPartValidSize IOError")
        parts = [(int(po[i]), stored[int(po[i]):int(po[i]) + int(pl[i])].tobytes()) for i in range(n)]
        return {"parts": parts, "svc": svc.value, "crc": crc.value,
                "stored": stored[: len(value) + self.padding(len(value))].tobytes()}


class PutState(ctypes.Structure):
    """orc_put_state: one client thread's PutPartValidSize state (all 0 = ThreadStorage defaults)."""
    _fields_ = [("ts_offset", ctypes.c_uint64), ("comp_total", ctypes.c_uint64), ("enabled", ctypes.c_uint32),
                ("crc", ctypes.c_uint32)]


def put_part(orc: "Oracle", state: PutState, key: bytes, chunk: bytes, offset_chunk: int, size_value: int) -> dict:
    """One Database::PutPartValidSize call (orc_put_part): {"rc", "mode", "occ", "chunk_final", "svc", "crc"}."""
    fin = np.zeros(8 + orc.compress_bound(len(chunk)) + 64, np.uint8)
    mode, crc = ctypes.c_uint32(0), ctypes.c_uint32(0)
    occ, fsz, svc = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = orc.lib.orc_put_part(ctypes.byref(state), _ptr(orc._buf(key)), len(key), _ptr(orc._buf(chunk)), len(chunk),
                              offset_chunk, size_value, _ptr(fin), ctypes.byref(mode), ctypes.byref(occ),
                              ctypes.byref(fsz), ctypes.byref(svc), ctypes.byref(crc))
    return {"rc": rc, "mode": mode.value, "occ": occ.value, "chunk_final": fin[: fsz.value].tobytes(),
            "svc": svc.value, "crc": crc.value}


def _digest(fn, src: np.ndarray, off: np.ndarray, lens: np.ndarray) -> tuple[int, int]:
    c = ctypes
    fn.argtypes = [_u8p, c.POINTER(c.c_uint64), c.POINTER(c.c_uint32), c.c_uint64, c.POINTER(c.c_uint64),
                   c.POINTER(c.c_uint32)]
    fn.restype = c.c_int
    src = np.ascontiguousarray(src, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    tot, crc = c.c_uint64(0), c.c_uint32(0)
    r = fn(_ptr(src), off.ctypes.data_as(c.POINTER(c.c_uint64)), lens.ctypes.data_as(c.POINTER(c.c_uint32)),
           len(lens), c.byref(tot), c.byref(crc))
    if r != 0:
        raise RuntimeError("frames_digest: IOError")
    return tot.value, crc.value


class Reference:
    """The reference's own codec (oracle/_ref/libkdbref.so); container only."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = ctypes.CDLL(path)
        c = ctypes
        lib.ref_compress_bound.argtypes = [c.c_int]
        lib.ref_compress_bound.restype = c.c_int
        lib.ref_compress_limited.argtypes = [_u8p, _u8p, c.c_int, c.c_int]
        lib.ref_compress_limited.restype = c.c_int
        lib.ref_decompress_partial.argtypes = [_u8p, c.c_int, _u8p, c.c_int, c.c_int]
        lib.ref_decompress_partial.restype = c.c_int
        lib.ref_frame_compress.argtypes = [_u8p, c.c_uint64, _u8p]
        lib.ref_frame_compress.restype = c.c_int64
        lib.ref_frames_uncompress.argtypes = [_u8p, c.c_uint64, _u8p, c.POINTER(c.c_uint64)]
        lib.ref_frames_uncompress.restype = c.c_int64
        lib.ref_crc32c_extend.argtypes = [c.c_uint32, _u8p, c.c_uint64]
        lib.ref_crc32c_extend.restype = c.c_uint32
        lib.ref_uncompress_value.argtypes = [_u8p, c.c_uint64, c.c_uint64, c.c_uint64, c.c_uint32, c.c_uint32,
                                             c.c_int, _u8p, ctypes.POINTER(c.c_uint64)]
        lib.ref_uncompress_value.restype = c.c_int
        lib.ref_gen_g2.argtypes = [_u8p, c.c_int, c.c_int]
        lib.ref_gen_g3.argtypes = [_u8p, c.c_int, c.c_int]
        self.lib = lib

    def compress_bound(self, n: int) -> int:
        return self.lib.ref_compress_bound(n)

    def compress(self, data: bytes, max_out: int | None = None) -> bytes | None:
        src = np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        cap = self.compress_bound(len(data)) if max_out is None else max_out
        dst = np.zeros(max(cap, self.compress_bound(len(data)), 1) + 64, dtype=np.uint8)
        r = self.lib.ref_compress_limited(_ptr(src), _ptr(dst), len(data), cap)
        return None if r == 0 else dst[:r].tobytes()

    def decompress(self, block: bytes, size: int) -> tuple[int, bytes]:
        src = np.frombuffer(block, dtype=np.uint8).copy() if len(block) else np.zeros(1, np.uint8)
        dst = np.zeros(size + 64, dtype=np.uint8)
        r = self.lib.ref_decompress_partial(_ptr(src), len(block), _ptr(dst), size, size)
        return r, (dst[:r].tobytes() if r > 0 else b"")

    def frame(self, data: bytes) -> bytes:
        src = np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        out = np.zeros(8 + max(self.compress_bound(len(data)), len(data)) + 64, dtype=np.uint8)
        n = self.lib.ref_frame_compress(_ptr(src), len(data), _ptr(out))
        if n < 0:
            raise RuntimeError("LZ4_compress_limitedOutput() failed")
        return out[:n].tobytes()

    def frames_uncompress(self, frames: bytes, out_cap: int) -> tuple[int, bytes]:
        src = np.frombuffer(frames, dtype=np.uint8).copy()
        out = np.zeros(out_cap + 64, dtype=np.uint8)
        tot = ctypes.c_uint64(0)
        n = self.lib.ref_frames_uncompress(_ptr(src), len(frames), _ptr(out), ctypes.byref(tot))
        return n, out[: tot.value].tobytes()

    def crc32c(self, data: bytes, crc: int = 0) -> int:
        a = np.frombuffer(data, dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        return self.lib.ref_crc32c_extend(crc, _ptr(a), len(data))

    def frames_digest(self, src: np.ndarray, off: np.ndarray, lens: np.ndarray) -> tuple[int, int]:
        """The reference's CompressorLZ4::Compress over every value: (sum of frame
        bytes, CRC32C of the frames concatenated)."""
        return _digest(self.lib.ref_frames_digest, src, off, lens)

    def uncompress_value(self, stored: bytes, svc: int, size: int, checksum: int = 0, checksum_initial: int = 0,
                         verify: bool = False) -> tuple[int, bytes]:
        """CompressorLZ4::UncompressByteArray: (0 OK / 1 Invalid checksum / 2 IOError, value bytes)."""
        src = np.frombuffer(stored, np.uint8).copy() if len(stored) else np.zeros(1, np.uint8)
        out = np.zeros(size + 64, np.uint8)
        n = ctypes.c_uint64(0)
        st = self.lib.ref_uncompress_value(_ptr(src), len(stored), svc, size, checksum, checksum_initial,
                                           1 if verify else 0, _ptr(out), ctypes.byref(n))
        return st, out[: n.value].tobytes()

    def g2(self, size: int, count: int) -> np.ndarray:
        out = np.empty(size * count, dtype=np.uint8)
        self.lib.ref_gen_g2(_ptr(out), size, count)
        return out

    def g3(self, size: int, count: int) -> np.ndarray:
        out = np.empty(size * count, dtype=np.uint8)
        self.lib.ref_gen_g3(_ptr(out), size, count)
        return out


def g1_pool(orc: Oracle, min_bytes: int = 1048576, seed: int = 301) -> np.ndarray:
    """db_bench RandomGenerator pool: 100-byte pieces until >= min_bytes
    (doc/bench/db_bench_kingdb.cc:119-131)."""
    npieces = (min_bytes + 99) // 100
    return orc.g1_pieces(npieces, seed)


def g1_values(pool: np.ndarray, size: int, count: int) -> list[bytes]:
    """RandomGenerator::Generate (db_bench_kingdb.cc:134-141): consecutive
    slices, wrapping to 0 when pos + len > pool size."""
    out = []
    pos = 0
    for _ in range(count):
        if pos + size > len(pool):
            pos = 0
        out.append(pool[pos:pos + size].tobytes())
        pos += size
    return out
