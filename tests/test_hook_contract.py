"""CPU: the flush hook keeps the reference's put contract (database.cc:128-276)
-- checked on the CPU-model build of KingDB + hooks (oracle/Makefile
`kingdb_san SAN=none`: the same flush_hook.cc over tests/cpp/abi_cpu_model.cc,
whose batch entry point computes with the oracle) against the reference build
(`kingdb_ref`), both driving the same put streams through oracle/ref_db.cc.
The GPU twins are in test_kingdb_dropin.py.

  * A put the reference refuses is refused by the hook build at the same put,
    with the same status, and the HSTable files of both builds are identical
    (irregular part shapes: overlaps, gaps, a last part sent twice, empty parts
    past the value, interleaved values, PutPart's own splits).
  * A GPU batch that fails twice (KDB_LZ4_FLUSH_INJECT) loses nothing: its
    parts are stored in the reference's disabled-compression form and every
    acknowledged put reads back through the reference's own reader.
"""
import os

import numpy as np
import pytest

from conftest import ROOT
from hook_streams import (irregular_stream, overrun_stream, refusals, run_kdb_db, same_database, verify_kdb_db)

pytestmark = pytest.mark.skipif(not os.path.isdir("/root/reference"),
                                reason="the KingDB builds compile the reference tree in place")

CPUM = os.path.join(ROOT, "oracle", "_ref", "kingdb_cpumodel", "kdb_db")
REFB = os.path.join(ROOT, "oracle", "_ref", "kingdb_ref", "kdb_db")
KEEP = {"KDB_DB_KEEP_GOING": "1", "KDB_LZ4_FLUSH_STATS": "1"}


@pytest.fixture(scope="module")
def builds():
    import subprocess
    for args in (["kingdb_san", "SAN=none"], ["kingdb"]):
        b = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle")] + args, capture_output=True,
                           text=True, timeout=1200)
        assert b.returncode == 0, b.stderr[-3000:]
    return CPUM, REFB


def _contract(builds, tmp_path, stream: bytes, opts):
    hook, ref = builds
    (tmp_path / "s.bin").write_bytes(stream)
    rr = run_kdb_db(ref, tmp_path / "ref", tmp_path / "s.bin", opts, {"KDB_DB_KEEP_GOING": "1"})
    rh = run_kdb_db(hook, tmp_path / "hook", tmp_path / "s.bin", opts, KEEP)
    assert rr.returncode in (0, 3), rr.stderr[-2000:]
    assert rh.returncode == rr.returncode, (rh.returncode, rr.returncode, rh.stderr[-2000:])
    assert refusals(rh.stderr) == refusals(rr.stderr)
    same_database(tmp_path / "ref", tmp_path / "hook")
    return rr, rh


def test_overrun_refused_at_the_same_put(builds, tmp_path):
    rr, rh = _contract(builds, tmp_path, overrun_stream(), (4 << 20, 1, 1 << 20))
    got = refusals(rh.stderr)
    assert len(got) == 2 and all("Prevented write to occur outside of the allocated memory" in g for g in got), got
    assert "refused_parts 2" in rh.stderr


@pytest.mark.parametrize("seed,mps", [(1, 1 << 20), (2, 1 << 20), (3, 16384), (4, 1 << 20)])
def test_irregular_parts_same_status_same_files(builds, tmp_path, seed, mps):
    rr, rh = _contract(builds, tmp_path, irregular_stream(seed), (4 << 20, 1, mps))
    print(len(refusals(rr.stderr)), "refusals;", [ln for ln in rh.stderr.splitlines() if "contract" in ln])


def _stream_100b(n):
    import struct
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


def _golden(name):
    z = np.load(os.path.join(ROOT, "tests", "golden", "hstable_streams.npz"))
    return z[f"{name}__stream"].tobytes(), tuple(int(x) for x in z[f"{name}__opts"])


@pytest.mark.parametrize("case", ["all-100b", "mid-100b", "multipart-2:2", "multipart-all", "small-3:2", "edge-1:2"])
def test_double_gpu_failure_loses_no_acknowledged_put(builds, tmp_path, case):
    """KDB_LZ4_FLUSH_INJECT=<first>:<count> fails GPU batch attempts: a batch
    whose two attempts both fail is completed on the host in the disabled
    form.  Every put is acknowledged, and the reference build's reader
    (Database::Get, the iterator, MultipartReader) finds every value intact."""
    hook, ref = builds
    if case.startswith("all-") or case.startswith("mid-"):
        # (the mid case: > 64 Ki puts, so there are several batches and the second fails twice)
        stream, opts = _stream_100b(20000 if case.startswith("all-") else 150000), (32 << 20, 1, 1 << 20)
        inject = "1:1000000000" if case.startswith("all-") else "2:2"
    else:
        name = case.split("-")[0]
        stream, opts = _golden(name)
        inject = "1:1000000000" if case.endswith("-all") else case.split("-")[1]
    (tmp_path / "s.bin").write_bytes(stream)
    env = {"KDB_LZ4_FLUSH_INJECT": inject, "KDB_LZ4_FLUSH_STATS": "1"}
    if not case.endswith("100b"):
        env["KDB_LZ4_FLUSH_MAX_PARTS"] = "5"       # multipart values straddle batches; a middle one fails
    r = run_kdb_db(hook, tmp_path / "db", tmp_path / "s.bin", opts, env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "stored uncompressed" in r.stderr
    host = [ln for ln in r.stderr.splitlines() if ln.startswith("lz4_flush_contract")]
    assert host and " host_batches 0 " not in host[0] + " ", host
    v = verify_kdb_db(ref, tmp_path / "db", tmp_path / "s.bin", opts)
    assert v.returncode == 0, v.stdout + v.stderr[-2000:]
    # no read of any value is wrong (Get, iterator, MultipartReader), and at
    # least the values the reference build finds in its own database are
    # found.  (The reference itself loses 9 of the multipart stream's 24
    # values to its frame-size quirks -- a first frame of exactly size_value
    # bytes makes the entry self-contained and drops the later parts,
    # DESIGN.md §4.6 -- which the disabled form does not hit: with every batch
    # failed, all 24 read back.)
    w = run_kdb_db(ref, tmp_path / "ref", tmp_path / "s.bin", opts)
    assert w.returncode == 0, w.stderr[-2000:]
    want = verify_kdb_db(ref, tmp_path / "ref", tmp_path / "s.bin", opts)
    assert want.returncode == 0
    f, g = [int(x) for x in v.stdout.split()[1::2]], [int(x) for x in want.stdout.split()[1::2]]
    found, missing, bad, iterated, it_bad, mp_bad = f
    assert (bad, it_bad, mp_bad) == (0, 0, 0), v.stdout
    assert found >= g[0] and found + missing == g[0] + g[1], (v.stdout, want.stdout)
    if case.endswith("100b"):
        assert found == _count_keys(stream)
    print(case, "hook:", v.stdout.strip(), "| reference:", want.stdout.strip())


def _count_keys(stream: bytes) -> int:
    import struct
    keys, i = set(), 0
    while i < len(stream):
        (kl,) = struct.unpack_from("<I", stream, i)
        i += 4
        key = stream[i:i + kl]
        i += kl + 8
        (nc,) = struct.unpack_from("<I", stream, i)
        i += 4
        ex = nc & 0x80000000
        for _ in range(nc & 0x7FFFFFFF):
            (cl,) = struct.unpack_from("<I", stream, i)
            i += 4 + (8 if ex else 0) + cl
        keys.add(key)
    return len(keys)
