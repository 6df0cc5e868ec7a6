"""CPU: the flush hook and the read-ahead over several devices (CPU-model
build, tests/cpp/abi_cpu_model.cc with KDB_LZ4_CPU_MODEL_DEVICES=4).

The flush pipeline runs one lane per device (worker thread, staging, stream,
the carried PutPartValidSize state of the client threads it takes); a client
thread moves between lanes only at a value's first part, where the reference
resets that state (database.cc:159-179, 252-255); results are published by
ticket and the flush completes the buffer in ticket order.  So the HSTable
files are the reference's, byte for byte, whatever the number of devices --
checked on the golden streams, with batches capped small so that lanes
interleave.  Execution on distinct real GPUs is the driver's 8-GPU run.
"""
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from hook_streams import defined_bytes, run_kdb_db

pytestmark = pytest.mark.skipif(not os.path.isdir("/root/reference"),
                                reason="the KingDB builds compile the reference tree in place")

CPUM = os.path.join(ROOT, "oracle", "_ref", "kingdb_cpumodel")


@pytest.fixture(scope="module")
def cpumodel():
    import subprocess
    b = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "kingdb_san", "SAN=none"],
                       capture_output=True, text=True, timeout=1200)
    assert b.returncode == 0, b.stderr[-3000:]
    return CPUM


@pytest.mark.parametrize("name", ["small", "edge", "rollover", "murmur", "multipart"])
@pytest.mark.parametrize("devices", [1, 4])
def test_golden_hstables_on_n_devices(cpumodel, tmp_path, name, devices):
    z = np.load(os.path.join(ROOT, "tests", "golden", "hstable_streams.npz"))
    opts = tuple(int(x) for x in z[f"{name}__opts"])
    (tmp_path / "s.bin").write_bytes(z[f"{name}__stream"].tobytes())
    env = {"KDB_LZ4_CPU_MODEL_DEVICES": str(devices), "KDB_LZ4_FLUSH_DEVICES": str(devices),
           "KDB_LZ4_READ_DEVICES": str(devices), "KDB_LZ4_CPU_MODEL_STATS": "1", "KDB_LZ4_FLUSH_STATS": "1",
           "KDB_LZ4_FLUSH_MAX_PARTS": "7"}
    r = run_kdb_db(os.path.join(cpumodel, "kdb_db"), tmp_path / "db", tmp_path / "s.bin", opts, env)
    assert r.returncode == 0, r.stderr[-2000:]
    for f in z[f"{name}__files"]:
        got = (tmp_path / "db" / str(f)).read_bytes()
        assert defined_bytes(got) == defined_bytes(z[f"{name}__file_{f}"].tobytes()), (name, f)
    lanes = [ln for ln in r.stderr.splitlines() if ln.startswith("lz4_flush_lanes")][0]
    assert lanes.startswith(f"lz4_flush_lanes {devices}")


def test_one_writer_spreads_over_devices(cpumodel, tmp_path):
    """One client thread, 64 MiB of 4 KiB values: it moves to the next lane
    every 2 MiB (at a value's first part), so all 4 devices take batches."""
    import struct
    rng = np.random.default_rng(3)
    base = rng.integers(97, 123, 512, dtype=np.uint8).tobytes()
    recs = []
    for i in range(16384):
        v = (base * 10)[i % 97:i % 97 + 4096]
        recs.append(struct.pack("<I", 16) + b"%016d" % i + struct.pack("<QII", 4096, 1, 4096) + v)
    (tmp_path / "s.bin").write_bytes(b"".join(recs))
    opts = (32 << 20, 1, 1 << 20)
    env = {"KDB_LZ4_CPU_MODEL_DEVICES": "4", "KDB_LZ4_FLUSH_DEVICES": "4", "KDB_LZ4_CPU_MODEL_STATS": "1",
           "KDB_LZ4_FLUSH_STATS": "1"}
    r = run_kdb_db(os.path.join(cpumodel, "kdb_db"), tmp_path / "one", tmp_path / "s.bin", opts, env)
    assert r.returncode == 0, r.stderr[-2000:]
    lanes = [ln for ln in r.stderr.splitlines() if ln.startswith("lz4_flush_lanes")][0]
    parts = [int(x) for x in re.findall(r"parts (\d+)", lanes)]
    assert len(parts) == 4 and all(p > 0 for p in parts) and sum(parts) == 16384, lanes
    # and the files equal a single-device run's
    env1 = dict(env, KDB_LZ4_CPU_MODEL_DEVICES="1", KDB_LZ4_FLUSH_DEVICES="1")
    r1 = run_kdb_db(os.path.join(cpumodel, "kdb_db"), tmp_path / "ref", tmp_path / "s.bin", opts, env1)
    assert r1.returncode == 0
    fa = sorted(os.listdir(tmp_path / "one"))
    assert fa == sorted(os.listdir(tmp_path / "ref"))
    for f in fa:
        if len(f) == 8:
            assert defined_bytes((tmp_path / "one" / f).read_bytes()) == defined_bytes((tmp_path / "ref" / f).read_bytes())


def _multipart_stream(seed: int, n: int) -> bytes:
    """n values of 48-200 KiB in 16 KiB parts (text-like, compressible)."""
    from hook_streams import record
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        V = int(rng.integers(48, 200)) << 10
        base = rng.integers(97, 123, 700, dtype=np.uint8).tobytes()
        v = (base * (V // 700 + 2))[int(rng.integers(0, 700)):][:V]
        recs.append(record(b"k%02d%06d" % (seed, i), V, [v[o:o + 16384] for o in range(0, V, 16384)]))
    return b"".join(recs)


def test_one_thread_interleaves_two_databases(cpumodel, tmp_path):
    """one client thread writes the parts of multipart
    values into TWO databases in turn, over 4 modelled devices.  The hook's
    per-thread lane and value tracking are kept per database (pipeline), so
    each database gets the files of a run of its stream alone: a reset lane on
    every switch would compress a part from another lane's carried
    PutPartValidSize state (wrong offsets, sizes or CRCs)."""
    import subprocess
    sa, sb = tmp_path / "a.bin", tmp_path / "b.bin"
    sa.write_bytes(_multipart_stream(1, 40))
    sb.write_bytes(_multipart_stream(2, 40))
    opts = (2 << 20, 1, 256 << 10)   # hstable 2 MiB, xxhash, 256 KiB maximum part size
    env = {"KDB_LZ4_CPU_MODEL_DEVICES": "4", "KDB_LZ4_FLUSH_DEVICES": "4", "KDB_LZ4_FLUSH_MAX_PARTS": "5"}
    exe = os.path.join(cpumodel, "kdb_db")
    r = subprocess.run([exe, "--two", str(tmp_path / "A"), str(tmp_path / "B"), str(sa), str(sb), str(opts[2]),
                        str(opts[0]), str(opts[1])], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    from hook_streams import same_database
    for s, d in ((sa, "A"), (sb, "B")):
        r1 = run_kdb_db(exe, tmp_path / f"{d}1", s, opts, dict(env, KDB_LZ4_CPU_MODEL_DEVICES="1", KDB_LZ4_FLUSH_DEVICES="1"))
        assert r1.returncode == 0, r1.stderr[-2000:]
        same_database(tmp_path / d, tmp_path / f"{d}1")
