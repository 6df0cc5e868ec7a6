#!/usr/bin/env python3
"""Golden fixtures for the write path: put streams and the HSTable
files the REFERENCE writes for them.

Runs oracle/_ref/ref_db -- KingDB's own Database::PutPart -> WriteBuffer ->
HSTableManager, compiled from /root/reference by `make -C oracle ref` -- on
each stream in a scratch directory, and stores the stream and every HSTable
file it leaves (container only; the fixture travels, the reference does not).

    python tests/golden/make_golden_put.py      -> tests/golden/hstable_streams.npz

Streams (name: what it exercises):
  small     1000 x (16 B "%016d" key, 100 B G1 value): the config-5 shape
  edge      empty / 1..14-byte / incompressible values (raw fallback -> disabled
            frame), keys of 1..300 bytes (multi-byte varints)
  rollover  300 mixed-size values, 64 KiB HSTables: file renewal, offset arrays
  murmur    300 small puts with MurmurHash3-64 keys
  multipart 64 KiB PutPart chunks of compressible, incompressible and mixed
            values (the disable rule mid-value), interleaved with small puts
"""
from __future__ import annotations

import os
import shutil
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "hstable_streams.npz")
REF_DB = os.path.join(ROOT, "oracle", "_ref", "ref_db")


def encode_stream(puts) -> bytes:
    """ref_db's stream format: u32 klen, key, u64 size, u32 nchunks, (u32 len, bytes)*."""
    out = bytearray()
    for k, v, ch in puts:
        ch = [len(v)] if ch is None else ch
        out += struct.pack("<I", len(k)) + k + struct.pack("<QI", len(v), len(ch))
        o = 0
        for c in ch:
            out += struct.pack("<I", c) + v[o:o + c]
            o += c
    return bytes(out)


def decode_stream(b: bytes):
    puts, i = [], 0
    while i < len(b):
        (kl,) = struct.unpack_from("<I", b, i)
        i += 4
        k = b[i:i + kl]
        i += kl
        size, nch = struct.unpack_from("<QI", b, i)
        i += 12
        v, ch = bytearray(), []
        for _ in range(nch):
            (cl,) = struct.unpack_from("<I", b, i)
            i += 4
            v += b[i:i + cl]
            i += cl
            ch.append(cl)
        assert len(v) == size
        puts.append((k, bytes(v), ch))
    return puts


def run_ref(stream: bytes, hstable_size: int, hash_type: int, part_size: int) -> dict[str, bytes]:
    d = tempfile.mkdtemp(prefix="kdbgold")
    try:
        sp = os.path.join(d, "stream.bin")
        open(sp, "wb").write(stream)
        db = os.path.join(d, "db")
        subprocess.run([REF_DB, db, sp, str(part_size), str(hstable_size), str(hash_type)], check=True,
                       capture_output=True)
        return {f: open(os.path.join(db, f), "rb").read() for f in sorted(os.listdir(db))
                if len(f) == 8 and all(c in "0123456789abcdef" for c in f)}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def streams(orc, ref):
    pool = oracle.g1_pool(orc, 4 << 20)
    pos = [0]

    def g1(n):
        if pos[0] + n > len(pool):
            pos[0] = 0
        v = pool[pos[0]:pos[0] + n].tobytes()
        pos[0] += n
        return v

    g3 = ref.g3(65536 * 2, 1).tobytes()
    rng = np.random.default_rng(8)
    out = {}
    out["small"] = ([(b"%016d" % i, g1(100), None) for i in range(1000)], 32 << 20, 1, 1 << 20)
    edge = []
    for i, sz in enumerate([0, 1, 2, 12, 13, 14, 50, 100, 101, 255, 256, 1000, 4096]):
        edge.append((b"e%015d" % i, g3[:sz], None))                  # incompressible
        edge.append((b"k" * (1 + 23 * i), g1(sz), None))              # keys 1..277 bytes
    edge.append((b"x" * 300, b"a" * 5000, None))
    edge.append((b"y", bytes(20000), None))
    out["edge"] = (edge, 32 << 20, 1, 1 << 20)
    sizes = rng.choice([1, 13, 100, 1000, 4096, 12000], 300)
    out["rollover"] = ([(b"%016d" % i, g1(int(s)), None) for i, s in enumerate(sizes)], 64 << 10, 1, 32 << 10)
    out["murmur"] = ([(b"%016d" % i, g1(100), None) for i in range(300)], 32 << 20, 0, 1 << 20)
    mp = []
    for i in range(12):
        kind = i % 4
        if kind == 0:
            v = g1(100000)
        elif kind == 1:
            v = g3[:70000]
        elif kind == 2:
            v = g1(65536 + 1000) + g3[:40000] + g1(9000)
        else:
            v = g1(3000)
        ch = [65536] * (len(v) // 65536) + ([len(v) % 65536] if len(v) % 65536 else [])
        mp.append((b"mp%014d" % i, v, ch))
        mp.append((b"sm%014d" % i, g1(100), None))
    out["multipart"] = (mp, 32 << 20, 1, 1 << 20)
    return out


def main() -> None:
    orc, ref = oracle.Oracle(), oracle.Reference()
    arrs = {}
    names = []
    for name, (puts, hs, ht, mps) in streams(orc, ref).items():
        s = encode_stream(puts)
        files = run_ref(s, hs, ht, mps)
        names.append(name)
        arrs[f"{name}__stream"] = np.frombuffer(s, np.uint8)
        arrs[f"{name}__opts"] = np.array([hs, ht, mps], np.uint64)
        arrs[f"{name}__files"] = np.array(list(files), dtype="U16")
        for f, b in files.items():
            arrs[f"{name}__file_{f}"] = np.frombuffer(b, np.uint8)
        print(f"{name}: {len(puts)} puts, {len(files)} file(s), {sum(map(len, files.values()))} bytes")
    arrs["names"] = np.array(names, dtype="U16")
    np.savez_compressed(OUT, **arrs)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
