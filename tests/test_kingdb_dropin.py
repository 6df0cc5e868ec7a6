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
hook (kingdb_amd/kingdb_include/cache/lz4_flush.h): single-part
puts are queued raw and compressed, checksummed and sized at the flush in one
kdb_put_entries_batch call.  The same test_db stages run against it, and the
write-path driver oracle/ref_db.cc (built as kdb_db) must write the HSTable
files the reference wrote for the golden put streams
(tests/golden/hstable_streams.npz) byte for byte, through both builds.
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
# unit-tests/testharness.cc:39).  The default run takes the tests whose
# IterateOverOptions() loop is short; KDB_DROPIN_FULL=1 runs the whole file.
QUICK = ["CloseAndReopen", "KeysWithNullBytes", "MultipartReader", "SingleThreadSmallEntries",
         "SingleThreadSnapshot", "SingleThreadSingleLargeEntry", "FileUtil"]


@pytest.mark.parametrize("build", sorted(BUILDS))
@pytest.mark.parametrize("name", [None] if os.environ.get("KDB_DROPIN_FULL") else QUICK)
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
        assert (db / f).read_bytes() == z[f"{name}__file_{f}"].tobytes(), f
