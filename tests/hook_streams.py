"""Put streams for kdb_db (oracle/ref_db.cc) and the helpers that compare two
KingDB builds on them -- shared by the CPU-model tests (test_hook_contract.py)
and the GPU tests (test_kingdb_dropin.py).

Record format (oracle/ref_db.cc): u32 key_len, key, u64 size_value, u32
nchunks, then per chunk u32 len (+ u64 offset when bit 31 of nchunks is set),
bytes.
"""
import os
import struct
import subprocess

import numpy as np

# bytes [72, 8192) of an HSTable's header block are left as the write buffer's
# memory held them (see test_kingdb_dropin.py): undefined, masked
HEADER_DEFINED, HEADER_BLOCK = 72, 8192


def defined_bytes(b: bytes) -> bytes:
    return b[:HEADER_DEFINED] + b[HEADER_BLOCK:] if len(b) >= HEADER_BLOCK else b


def record(key: bytes, size_value: int, chunks, offsets=None) -> bytes:
    """One record; `offsets` (one per chunk) makes them explicit."""
    out = [struct.pack("<I", len(key)), key, struct.pack("<Q", size_value)]
    n = len(chunks) | (0x80000000 if offsets is not None else 0)
    out.append(struct.pack("<I", n))
    for i, c in enumerate(chunks):
        out.append(struct.pack("<I", len(c)))
        if offsets is not None:
            out.append(struct.pack("<Q", offsets[i]))
        out.append(c)
    return b"".join(out)


def _payload(rng, n: int) -> bytes:
    kind = rng.integers(0, 3)
    if kind == 0:                                   # incompressible
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == 1:                                   # runs
        return (bytes([int(rng.integers(97, 100))]) * n)
    base = rng.integers(97, 123, max(1, n // 8 + 1), dtype=np.uint8).tobytes()   # repetitive text
    return (base * 9)[:n]


def irregular_stream(seed: int, n_records: int = 160) -> bytes:
    """Puts PutPartValidSize may refuse (database.cc:261-266) next to regular
    ones: parts out of order, gaps, overlaps, a value's last part sent twice,
    parts past the value's end, empty parts, two values interleaved on the one
    client thread, single-part values in between."""
    rng = np.random.default_rng(seed)
    recs = []
    open_values = []          # (key, size_value, next offset) of values left unfinished
    for r in range(n_records):
        choice = rng.integers(0, 6)
        if choice == 1 or (choice > 1 and not open_values):   # start a multipart value, leave it open
            V = int(rng.choice([8192, 16384, 65536, 70000, 140000]))
            n = int(rng.choice([4096, 8192, min(V, 16384)]))
            key = b"m%07d" % r
            recs.append(record(key, V, [_payload(rng, n)], [0]))
            open_values.append([key, V, n])
        elif choice == 0:                           # a regular single-part value
            n = int(rng.choice([0, 1, 13, 100, 4096, 5000]))
            recs.append(record(b"s%07d" % r, n, [_payload(rng, n)]))
        else:                                       # continue an open value, regularly or not
            i = int(rng.integers(0, len(open_values)))
            key, V, nxt = open_values[i]
            how = rng.integers(0, 6)
            if how == 0:
                off = nxt                           # regular
            elif how == 1:
                off = max(0, nxt - int(rng.integers(1, 4097)))   # overlap
            elif how == 2:
                off = min(V, nxt + int(rng.integers(1, 4097)))   # gap
            elif how == 3:
                off = V                             # at the end (an empty part, or past it)
            elif how == 4:
                off = int(rng.integers(0, V + 1))   # anywhere
            else:
                off = nxt
            room = V - off
            n = int(rng.choice([0, 1, 100, 4096, 8192])) if room > 0 else 0
            if rng.integers(0, 8) == 0:
                n += 1                              # sometimes past the value's end (PutPart refuses)
            n = min(n, max(room, 0) + 1)
            recs.append(record(key, V, [_payload(rng, n)], [off]))
            open_values[i][2] = off + n
            if off + n >= V and rng.integers(0, 2) == 0:
                open_values.pop(i)
    return b"".join(recs)


def overrun_stream() -> bytes:
    """Hand-made refusals (database.cc:261-266), each at a value's last part
    and in the middle of a stream of regular puts:
      * 16 x 4 KiB incompressible parts of a 64 KiB value (the disable rule
        switches at the second part), then an empty part at offset 65536 --
        its offset is ts_offset = 65552 > 65536 + 0 padding;
      * a 4-part value whose last part is sent twice."""
    rng = np.random.default_rng(11)
    rnd = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()   # noqa: E731
    recs = [record(b"before%04d" % i, 100, [b"x%099d" % i]) for i in range(50)]
    recs.append(record(b"overrun-empty", 65536, [rnd(4096) for _ in range(16)] + [b""]))
    recs += [record(b"between%04d" % i, 4096, [rnd(4096)]) for i in range(20)]
    parts = [rnd(4096) for _ in range(4)]
    recs.append(record(b"overrun-dup", 16384, parts + [parts[3]], [0, 4096, 8192, 12288, 12288]))
    recs += [record(b"after%04d" % i, 100, [b"y%099d" % i]) for i in range(50)]
    return b"".join(recs)


def run_kdb_db(exe, db, stream, opts, env_extra=None, timeout=300):
    hs, ht, mps = opts
    env = dict(os.environ, **(env_extra or {}))
    return subprocess.run([exe, str(db), str(stream), str(mps), str(hs), str(ht)], capture_output=True, text=True,
                          timeout=timeout, env=env)


def verify_kdb_db(exe, db, stream, opts, timeout=300):
    hs, ht, mps = opts
    return subprocess.run([exe, "--verify", str(db), str(stream), str(mps), str(hs), str(ht)], capture_output=True,
                          text=True, timeout=timeout)


def refusals(stderr: str):
    return [ln for ln in stderr.splitlines() if ln.startswith("put ")]


def hstables(db):
    return sorted(f for f in os.listdir(db) if len(f) == 8 and all(c in "0123456789abcdef" for c in f))


def same_database(a, b):
    fa, fb = hstables(a), hstables(b)
    assert fa == fb, (fa, fb)
    for f in fa:
        assert defined_bytes((a / f).read_bytes()) == defined_bytes((b / f).read_bytes()), f
