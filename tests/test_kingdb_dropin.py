"""GPU: KingDB's own unit tests, compiled from the reference tree against the
drop-in (oracle/Makefile `kingdb`, INTEGRATION.md level 2).

In `oracle/_ref/kingdb_dropin/` every translation unit of KingDB sees
kingdb_amd/kingdb_include/algorithm/compressor.h (the drop-in
kdb::CompressorLZ4) instead of the reference's, algorithm/compressor.o and
algorithm/lz4.o are not linked, and every LZ4 block goes through
libkdb_lz4.so's HIP kernels.  `oracle/_ref/kingdb_ref/` is the same build
with the reference codec, run beside it as the checker.

  * unit-tests/test_compression.cc: `Verify(): ok`, and the frame stream it
    prints equals the reference's (tests/golden/test_compression.npz, KAT T1).
  * unit-tests/test_db.cc (LevelDB harness, 11 tests x 13 option stages, 10 of
    them LZ4): `==== PASSED` with the same test list as the reference build.
  * unit-tests/client_embedded.cc: 1 M puts of 16 B keys / 100 B values through
    Database::PutPart, then an iteration with GetValue: all 1 M items back.

`oracle/_ref/kingdb_hook/` is the drop-in build plus the write-buffer flush
hook (kingdb_amd/kingdb_include/cache/lz4_flush.h): every
part of every put -- single-part values and multipart parts alike -- is
queued raw, and a per-database pipeline batches them through
kdb_flush_parts_batch while the buffer fills; the flush completes the orders.
The same test_db stages run against it, and the write-path driver
oracle/ref_db.cc (built as kdb_db) must write the HSTable files the reference
wrote for the golden put streams (tests/golden/hstable_streams.npz, multipart
streams included) byte for byte, through both builds.  The reference's put contract:
a GPU batch failure injected into the hook (KDB_LZ4_FLUSH_INJECT) is retried,
and the files are still the reference's; a permanent one completes the
batches on the host in the disabled-compression form, so every acknowledged
put is read back by the reference build; irregular parts are refused at the
same put as by the reference build, with identical files.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT, load_golden

pytestmark = pytest.mark.gpu

DROP = os.path.join(ROOT, "oracle", "_ref", "kingdb_dropin")
HOOK = os.path.join(ROOT, "oracle", "_ref", "kingdb_hook")
BUILDS = {"dropin": DROP, "hook": HOOK}
REF = os.path.join(ROOT, "oracle", "_ref", "kingdb_ref")


def _bin(d, name):
    p = os.path.join(d, name)
    if not os.path.exists(p):
        pytest.fail(f"{p} missing: build it here with `make -C oracle kingdb` (needs /root/reference)")
    return p


def _frames_from_stderr(err: bytes) -> bytes:
    # unit-tests/test_compression.cc:86-90 prints the frame stream between these markers
    m = re.search(rb"--- stream compressed data \(size:(\d+)\):\n", err)
    assert m, "no frame stream in test_compression's output"
    n = int(m.group(1))
    body = err[m.end():m.end() + n]
    assert err[m.end() + n:m.end() + n + 10] == b"\n--- done\n"
    return body


def test_kingdb_test_compression(tmp_path, gpu):
    r = subprocess.run([_bin(DROP, "test_compression")], cwd=tmp_path, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert b"Verify(): ok" in r.stderr
    stream = _frames_from_stderr(r.stderr)
    g = load_golden("test_compression.npz")
    assert stream == g["frames"].tobytes()
    assert len(stream) == 1947
    rr = subprocess.run([_bin(REF, "test_compression")], cwd=tmp_path, capture_output=True, timeout=120)
    assert _frames_from_stderr(rr.stderr) == stream


def _passed(err: str):
    tests = re.findall(r"==== Test (\S+)", err)
    m = re.search(r"==== PASSED (\d+) tests", err)
    return tests, int(m.group(1)) if m else None


# The LevelDB harness's filter (LEVELDB_TESTS, a substring of "DBTest.<name>",
# unit-tests/testharness.cc:39): every one of unit-tests/test_db.cc's 11 tests,
# one entry per test and build (the SingleThreadSmallEntries filter also matches
# SingleThreadSmallEntriesCompaction, so that one runs twice);
# KDB_DROPIN_FULL=1 runs the whole file in one process instead.
TEST_DB = ["CloseAndReopen", "KeysWithNullBytes", "MultipartReader", "SingleThreadSmallEntries",
           "SingleThreadSnapshot", "SingleThreadSingleLargeEntry", "FileUtil", "RepairInvalidDatabaseOptionFile",
           "TestStringInterface", "SingleThreadSmallEntriesCompaction", "SequentialIterator"]


@pytest.mark.parametrize("build", sorted(BUILDS))
@pytest.mark.parametrize("name", [None] if os.environ.get("KDB_DROPIN_FULL") else TEST_DB)
def test_kingdb_test_db(tmp_path, gpu, name, build):
    env = dict(os.environ)
    if name:
        env["LEVELDB_TESTS"] = name
    r = subprocess.run([_bin(BUILDS[build], "test_db")], cwd=tmp_path, capture_output=True, text=True, env=env,
                       timeout=1500, errors="replace")
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    tests, passed = _passed(r.stderr)
    assert passed is not None and passed == len(tests) and passed >= 1, r.stderr[-3000:]
    if name is None:
        assert passed == 11
    # every LZ4 option stage ran (unit-tests/test_db.cc:185-266)
    if name not in ("CloseAndReopen", "KeysWithNullBytes", "FileUtil", "RepairInvalidDatabaseOptionFile"):
        for stage in (0, 1, 3, 4, 5, 7, 9, 10, 11, 12):
            assert f"Stage {stage} -" in r.stdout


@pytest.mark.skipif(not os.environ.get("KDB_DROPIN_FULL"), reason="1 M puts; KDB_DROPIN_FULL=1")
@pytest.mark.parametrize("build", sorted(BUILDS))
def test_kingdb_client_embedded(tmp_path, gpu, build):
    r = subprocess.run([_bin(BUILDS[build], "client_emb")], cwd=tmp_path, capture_output=True, text=True,
                       timeout=1500)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "count items: 1000000" in r.stdout
    print(build, r.stdout)


# The reference leaves bytes [72, 8192) of every HSTable's header block as the
# write buffer's memory held them: HSTableManager::OpenNewFile encodes the
# 72-byte HSTableHeader + DatabaseOptions into buffer_raw_ (hstable_manager.h:
# 280-289, format.h:415-425) and the block's other bytes are never written --
# `new char[2 * size_block]` (:77) is zero only when the allocator maps fresh
# pages.  With 64 KiB HSTables that depends on the process's earlier heap use
# (glibc's dynamic mmap threshold), so those bytes are undefined and masked.
HEADER_DEFINED, HEADER_BLOCK = 72, 8192


def _defined_bytes(b: bytes) -> bytes:
    return b[:HEADER_DEFINED] + b[HEADER_BLOCK:] if len(b) >= HEADER_BLOCK else b


def _defined(path) -> bytes:
    return _defined_bytes(path.read_bytes())


def _golden_streams():
    import numpy as np
    z = np.load(os.path.join(ROOT, "tests", "golden", "hstable_streams.npz"))
    return z, [str(n) for n in z["names"]]


@pytest.mark.parametrize("build", sorted(BUILDS))
@pytest.mark.parametrize("name", _golden_streams()[1])
def test_kingdb_write_path_reference_hstables(tmp_path, gpu, build, name):
    z, _ = _golden_streams()
    hs, ht, mps = (int(x) for x in z[f"{name}__opts"])
    (tmp_path / "s.bin").write_bytes(z[f"{name}__stream"].tobytes())
    db = tmp_path / "db"
    r = subprocess.run([_bin(BUILDS[build], "kdb_db"), str(db), str(tmp_path / "s.bin"), str(mps), str(hs), str(ht)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    want = [str(f) for f in z[f"{name}__files"]]
    got = sorted(f for f in os.listdir(db) if len(f) == 8 and all(c in "0123456789abcdef" for c in f))
    assert got == want
    for f in want:
        assert _defined(db / f) == _defined_bytes(z[f"{name}__file_{f}"].tobytes()), f


def _run_stream(exe, db, stream, opts, env=None):
    hs, ht, mps = opts
    return subprocess.run([exe, str(db), str(stream), str(mps), str(hs), str(ht)], capture_output=True, text=True,
                          timeout=300, env=env)


@pytest.mark.parametrize("name", ["small", "multipart", "murmur"])
def test_hook_retry_after_injected_gpu_failure(tmp_path, gpu, name):
    """The first GPU batch attempt fails (KDB_LZ4_FLUSH_INJECT=1:1): the
    pipeline retries on a fresh stream and staging, and the files are still the
    reference's, byte for byte."""
    z, _ = _golden_streams()
    opts = tuple(int(x) for x in z[f"{name}__opts"])
    (tmp_path / "s.bin").write_bytes(z[f"{name}__stream"].tobytes())
    env = dict(os.environ, KDB_LZ4_FLUSH_INJECT="1:1")
    r = _run_stream(_bin(HOOK, "kdb_db"), tmp_path / "db", tmp_path / "s.bin", opts, env)
    assert r.returncode == 0, r.stderr[-2000:]
    want = [str(f) for f in z[f"{name}__files"]]
    for f in want:
        assert _defined(tmp_path / "db" / f) == _defined_bytes(z[f"{name}__file_{f}"].tobytes()), f


def _big_stream(n):
    import struct
    import numpy as np
    rng = np.random.default_rng(5)
    vals = rng.integers(97, 101, (n, 100), dtype=np.uint8)
    rec = np.zeros((n, 4 + 16 + 8 + 4 + 4 + 100), np.uint8)
    rec[:, 0:4] = np.frombuffer(struct.pack("<I", 16), np.uint8)
    rec[:, 4:20] = np.frombuffer(b"".join(b"%016d" % i for i in range(n)), np.uint8).reshape(n, 16)
    rec[:, 20:28] = np.frombuffer(struct.pack("<Q", 100), np.uint8)
    rec[:, 28:32] = np.frombuffer(struct.pack("<I", 1), np.uint8)
    rec[:, 32:36] = np.frombuffer(struct.pack("<I", 100), np.uint8)
    rec[:, 36:] = vals
    return rec.tobytes()


@pytest.mark.parametrize("first", [1, 3])
def test_hook_permanent_gpu_failure_is_survived(tmp_path, gpu, first):
    """Every GPU batch attempt from `first` on fails: each such batch is
    completed on the host in the reference's disabled-compression form
    (database.cc:199-209), so every put is acknowledged AND stored: the
    reference build then reads back all 300 000 values intact (the reference's
    put contract: nothing acknowledged is lost)."""
    (tmp_path / "s.bin").write_bytes(_big_stream(300000))
    opts = (32 << 20, 1, 1 << 20)
    env = dict(os.environ, KDB_LZ4_FLUSH_INJECT=f"{first}:1000000000", KDB_LZ4_FLUSH_STATS="1")
    r = _run_stream(_bin(HOOK, "kdb_db"), tmp_path / "db", tmp_path / "s.bin", opts, env)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "stored uncompressed" in r.stderr
    v = subprocess.run([_bin(REF, "kdb_db"), "--verify", str(tmp_path / "db"), str(tmp_path / "s.bin"),
                        str(opts[2]), str(opts[0]), str(opts[1])], capture_output=True, text=True, timeout=300)
    assert v.returncode == 0, v.stdout + v.stderr[-2000:]
    print(v.stdout.strip(), [ln for ln in r.stderr.splitlines() if "contract" in ln])
    f = [int(x) for x in v.stdout.split()[1::2]]
    assert f[0] == 300000 and f[1:3] == [0, 0] and f[4:] == [0, 0], v.stdout


@pytest.mark.parametrize("stream", ["overrun", "irregular1", "irregular2", "irregular3-mps16k"])
def test_hook_refuses_the_puts_the_reference_refuses(tmp_path, gpu, stream):
    """Irregular part shapes (tests/hook_streams.py: overlaps, gaps, a last
    part sent twice, empty parts past the value, interleaved values, PutPart's
    own splits): the GPU hook build refuses exactly the puts the reference
    build refuses, with the same status (database.cc:261-266, settled inside
    LZ4FlushDefer), and writes the same HSTable files."""
    from hook_streams import irregular_stream, overrun_stream, refusals, run_kdb_db, same_database
    data = overrun_stream() if stream == "overrun" else irregular_stream(int(stream[9]))
    opts = (4 << 20, 1, 16384 if stream.endswith("mps16k") else 1 << 20)
    (tmp_path / "s.bin").write_bytes(data)
    keep = {"KDB_DB_KEEP_GOING": "1"}
    rr = run_kdb_db(_bin(REF, "kdb_db"), tmp_path / "ref", tmp_path / "s.bin", opts, keep)
    rh = run_kdb_db(_bin(HOOK, "kdb_db"), tmp_path / "hook", tmp_path / "s.bin", opts,
                    dict(keep, KDB_LZ4_FLUSH_STATS="1"))
    assert rr.returncode in (0, 3), rr.stderr[-2000:]
    assert rh.returncode == rr.returncode, (rh.returncode, rh.stderr[-2000:])
    assert refusals(rh.stderr) == refusals(rr.stderr)
    if stream == "overrun":
        assert len(refusals(rh.stderr)) == 2
    same_database(tmp_path / "ref", tmp_path / "hook")


def _verify(exe, db, stream, opts):
    hs, ht, mps = opts
    return subprocess.run([exe, "--verify", str(db), str(stream), str(mps), str(hs), str(ht)], capture_output=True,
                          text=True, timeout=300)


@pytest.mark.parametrize("name", ["small", "edge", "murmur", "multipart"])
def test_hook_read_path_matches_reference_reads(tmp_path, gpu, name):
    """The read hooks (INTEGRATION.md level 5): the hook build reads a database
    back three ways -- Database::Get, the iterator's GetValue (LZ4ReadAhead: the
    next entries decoded in one GPU batch) and MultipartReader (LZ4MultipartDecode:
    all frames of a value in one launch) -- and every value equals the one put,
    with the same found / missing / iterated counts as the reference build
    reading the reference's own files."""
    z, _ = _golden_streams()
    opts = tuple(int(x) for x in z[f"{name}__opts"])
    (tmp_path / "s.bin").write_bytes(z[f"{name}__stream"].tobytes())
    r = _run_stream(_bin(REF, "kdb_db"), tmp_path / "ref", tmp_path / "s.bin", opts)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _verify(_bin(REF, "kdb_db"), tmp_path / "ref", tmp_path / "s.bin", opts)
    assert want.returncode == 0, want.stdout + want.stderr[-2000:]
    r = _run_stream(_bin(HOOK, "kdb_db"), tmp_path / "hook", tmp_path / "s.bin", opts)
    assert r.returncode == 0, r.stderr[-2000:]
    got = _verify(_bin(HOOK, "kdb_db"), tmp_path / "hook", tmp_path / "s.bin", opts)
    assert got.returncode == 0, got.stdout + got.stderr[-2000:]
    assert got.stdout.split() == want.stdout.split()


def test_hook_client_embedded_iteration_vs_reference(tmp_path, gpu):
    """unit-tests/client_embedded.cc (1 M puts of 16 B keys / 100 B values, then
    one iteration with GetValue) through the reference build and through the
    hook build, on the same box in the same test: all items back in both, and
    the times are printed (the read hooks' claim is the hook build's iteration
    <= the reference's)."""
    out = {}
    for b, d in (("reference", REF), ("hook", HOOK)):
        wd = tmp_path / b
        wd.mkdir()
        r = subprocess.run([_bin(d, "client_emb")], cwd=wd, capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, KDB_LZ4_FLUSH_STATS="1", KDB_LZ4_READ_STATS="1"))
        for ln in r.stderr.splitlines():
            if ln.startswith(("lz4_flush_stats", "lz4_read_stats")):
                print(b, ln)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "count items: 1000000" in r.stdout
        it = re.search(r"iteration done in (\d+) ms", r.stdout)
        out[b] = int(it.group(1))
        print(b, r.stdout.strip().replace("\n", " | "))
    print("iteration ms", out)


def test_hook_concurrent_writers_and_readers(tmp_path, gpu):
    """oracle/hook_mt.cc on the GPU build: 8 client threads put single-part and
    multipart values at once (the flush pipeline carries each thread's
    PutPartValidSize state), then 8 readers (Get, MultipartReader) and an
    iteration get every value back byte for byte."""
    r = subprocess.run([_bin(HOOK, "hook_mt"), str(tmp_path / "db"), "8", "150"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, KDB_LZ4_READ_BATCH="64"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.startswith("ok:"), r.stdout
