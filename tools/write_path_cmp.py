#!/usr/bin/env python3
"""KingDB's own write path, like for like, with three codecs behind it.

configs[4] (BASELINE.json): the sequential-write bench shape, 16 B keys /
100 B values (and 4 KiB values beside it), sent through Database::PutPart ->
WriteBuffer -> HSTableManager by oracle/ref_db.cc (built as kdb_db) in three
builds of the SAME KingDB sources (oracle/Makefile):

  kingdb_ref     the reference codec (algorithm/compressor.cc + lz4.cc) on the CPU
  kingdb_dropin  the drop-in CompressorLZ4: one GPU call per PutPart (zero-copy
                 scalar path, kdb_lz4_capi.hip)
  kingdb_hook    the drop-in plus the flush hook (lz4_flush.h): one
                 kdb_put_entries_batch per write-buffer flush

Each build writes its HSTables into its own fresh directory under the SAME
parent (--dir; default: the current directory, i.e. the box's local disk;
/dev/shm for tmpfs), and the three databases' files must be identical.
Prints one JSON object per (workload, build) and a summary line.

  python tools/write_path_cmp.py [--n 1048576] [--sizes 100,4096,mp3072x262144/65536] [--dir DIR]

(mp<N>x<V>/<P>: N values of V bytes, each sent as PutPart calls of P bytes.)
"""
import argparse
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BUILDS = ["kingdb_ref", "kingdb_dropin", "kingdb_hook"]


def stream(n: int, ks: int, vs: int) -> np.ndarray:
    """n single-chunk puts, keys %016d-style, G1 values (oracle's generator)."""
    import oracle  # the data generator only (checker infrastructure)
    orc = oracle.Oracle()
    pool = np.frombuffer(oracle.g1_pool(orc, 8 << 20), np.uint8)
    rng = np.random.default_rng(7)
    starts = rng.integers(0, len(pool) - vs, n)
    vals = pool[starts[:, None] + np.arange(vs)[None, :]]
    keys = np.frombuffer(b"".join(b"%016d" % i for i in range(n)), np.uint8).reshape(n, 16)[:, :ks]
    rec = np.zeros((n, 4 + ks + 8 + 4 + 4 + vs), np.uint8)
    rec[:, 0:4] = np.frombuffer(struct.pack("<I", ks), np.uint8)
    rec[:, 4:4 + ks] = keys
    rec[:, 4 + ks:12 + ks] = np.frombuffer(struct.pack("<Q", vs), np.uint8)
    rec[:, 12 + ks:16 + ks] = np.frombuffer(struct.pack("<I", 1), np.uint8)
    rec[:, 16 + ks:20 + ks] = np.frombuffer(struct.pack("<I", vs), np.uint8)
    rec[:, 20 + ks:] = vals
    return rec


def mp_stream(n: int, ks: int, vs: int, part: int) -> np.ndarray:
    """n values of vs bytes, each sent as PutPart calls of `part` bytes
    (KingServer's 64 KiB receive parts, network/server.cc:258; MultipartWriter,
    interface/multipart.h:200-224), keys %016d-style, G1 values."""
    import oracle
    orc = oracle.Oracle()
    pool = np.frombuffer(oracle.g1_pool(orc, 8 << 20), np.uint8)
    rng = np.random.default_rng(9)
    starts = rng.integers(0, len(pool) - vs, n)
    nch = (vs + part - 1) // part
    rec_len = 4 + ks + 8 + 4 + nch * 4 + vs
    rec = np.zeros((n, rec_len), np.uint8)
    rec[:, 0:4] = np.frombuffer(struct.pack("<I", ks), np.uint8)
    rec[:, 4:4 + ks] = np.frombuffer(b"".join(b"%016d" % i for i in range(n)), np.uint8).reshape(n, 16)[:, :ks]
    rec[:, 4 + ks:12 + ks] = np.frombuffer(struct.pack("<Q", vs), np.uint8)
    rec[:, 12 + ks:16 + ks] = np.frombuffer(struct.pack("<I", nch), np.uint8)
    at = 16 + ks
    for c in range(nch):
        cl = min(part, vs - c * part)
        rec[:, at:at + 4] = np.frombuffer(struct.pack("<I", cl), np.uint8)
        for i in range(n):
            rec[i, at + 4:at + 4 + cl] = pool[starts[i] + c * part:starts[i] + c * part + cl]
        at += 4 + cl
    return rec


# Bytes [72, 8192) of an HSTable's header block are whatever the reference's
# write buffer held there (hstable_manager.h:77, 280-289: never written), so
# they are not compared (tests/test_kingdb_dropin.py, HEADER_DEFINED).
def files_of(db: str) -> dict:
    out = {}
    for f in sorted(os.listdir(db)):
        if len(f) == 8 and all(c in "0123456789abcdef" for c in f):
            b = open(os.path.join(db, f), "rb").read()
            out[f] = b[:72] + b[8192:] if len(b) >= 8192 else b
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--sizes", default="100,4096,mp3072x262144/65536")
    ap.add_argument("--dir", default=".")
    ap.add_argument("--builds", default=",".join(BUILDS))
    ap.add_argument("--out", default=None)
    ap.add_argument("--ceiling", action="store_true", help="also run the reference with compression off")
    ap.add_argument("--timeout", type=float, default=120.0,
                    help="seconds per run; a run past it is killed and reported as hung (the reference "
                         "KingDB itself can stop making progress, see mp3072 below)")
    ap.add_argument("--repeat", type=int, default=1, help="runs of each build per workload")
    a = ap.parse_args()
    rows = []
    for size in a.sizes.split(","):
        d = tempfile.mkdtemp(prefix="kdbwp", dir=a.dir)
        try:
            sp = os.path.join(d, "s.bin")
            args = []
            if size.startswith("mp"):            # mp<count>x<value bytes>/<part bytes>: multipart values
                cnt, rest = size[2:].split("x")
                vs, part = (int(x) for x in rest.split("/"))
                n = int(cnt)
                mp_stream(n, 16, vs, part).tofile(sp)
                what = f"{n} values of {vs} B in {part} B PutPart parts, 16 B keys, G1"
                # 256 MiB HSTables, and under the 1 GB of uncompacted data that starts a
                # compaction (util/options.h:192): with the default 32 MiB HSTables the
                # reference itself stops making progress on this stream once a third
                # file opens (measured: 256 x 256 KiB values hang, 240 do not)
                args = [str(1 << 20), str(256 << 20)]
            else:
                vs = int(size)
                n = a.n if vs <= 1024 else max(1, a.n // 8)
                stream(n, 16, vs).tofile(sp)
                what = f"{n} puts 16 B keys / {vs} B G1 values"
            ref_files = None
            for b in [x for x in a.builds.split(",") for _ in range(max(1, a.repeat))]:
                exe = os.path.join(ROOT, "oracle", "_ref", b, "kdb_db")
                db = os.path.join(d, "db_" + b)
                t0 = time.perf_counter()
                env = dict(os.environ, KDB_LZ4_FLUSH_STATS="1") if b == "kingdb_hook" else None
                try:
                    r = subprocess.run([exe, db, sp] + args, capture_output=True, text=True, timeout=a.timeout,
                                       env=env)
                except subprocess.TimeoutExpired as e:
                    err = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else (e.stderr or "")
                    row = {"workload": what, "build": b, "hung": True, "killed_after_s": a.timeout,
                           "stderr_tail": err[-1500:], "dir": os.path.abspath(a.dir)}
                    print(json.dumps(row), flush=True)
                    rows.append(row)
                    shutil.rmtree(db, ignore_errors=True)
                    continue
                wall = time.perf_counter() - t0
                if r.returncode != 0:
                    print(r.stderr[-2000:], file=sys.stderr)
                    sys.exit(f"{b} failed rc={r.returncode}")
                f = r.stdout.split()
                t_put, t_all = float(f[2]), float(f[5])
                files = files_of(db)
                if ref_files is None:
                    ref_files = files
                same = files == ref_files
                row = {"workload": what, "build": b,
                       "puts_per_s": round(n / t_put, 1), "puts_per_s_with_close": round(n / t_all, 1),
                       "seconds_put": round(t_put, 4), "seconds_with_close": round(t_all, 4),
                       "process_wall_s": round(wall, 3), "hstable_files": len(files),
                       "hstable_bytes": sum(map(len, files.values())), "files_identical_to_first_build": same,
                       "dir": os.path.abspath(a.dir)}
                for ln in r.stderr.splitlines():
                    if ln.startswith("lz4_flush_stats "):
                        w = ln.split()[1:]
                        row["flush_stats"] = {k: float(v) for k, v in zip(w[::2], w[1::2])}
                print(json.dumps(row), flush=True)
                rows.append(row)
                shutil.rmtree(db, ignore_errors=True)
                if not same:
                    sys.exit(f"{b}: HSTable files differ from {a.builds.split(',')[0]}")
            if a.ceiling:
                # the same write path with compression off (reference build): what
                # KingDB's write buffer and storage engine cost without any codec --
                # the most any codec change can reach on this workload
                exe = os.path.join(ROOT, "oracle", "_ref", "kingdb_ref", "kdb_db")
                db = os.path.join(d, "db_none")
                ca = args + [str(1 << 20), str(32 << 20)][len(args):] + ["1", "none"]
                try:
                    r = subprocess.run([exe, db, sp] + ca, capture_output=True, text=True, timeout=a.timeout)
                except subprocess.TimeoutExpired:
                    r = None
                if r is not None and r.returncode == 0:
                    f = r.stdout.split()
                    t_put, t_all = float(f[2]), float(f[5])
                    row = {"workload": what, "build": "kingdb_ref, compression off (ceiling)",
                           "puts_per_s": round(n / t_put, 1), "puts_per_s_with_close": round(n / t_all, 1),
                           "seconds_put": round(t_put, 4), "seconds_with_close": round(t_all, 4),
                           "dir": os.path.abspath(a.dir)}
                    print(json.dumps(row), flush=True)
                    rows.append(row)
                shutil.rmtree(db, ignore_errors=True)
        finally:
            shutil.rmtree(d, ignore_errors=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
