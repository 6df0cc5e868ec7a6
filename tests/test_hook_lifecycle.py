"""CPU: the flush hook's pipeline belongs to the write buffer that is open, from
the moment Database::Open returns -- not from the moment WriteBuffer's
ProcessingLoop thread first runs.

Round 5's GPU suite failed once in test_db's SingleThreadSmallEntriesCompaction
(hook build): in one option stage every Put returned "IO error: Cannot handle
request: WriteBuffer is closing" and the iteration found 0 of 1000 items
(/root/reference/unit-tests/test_db.cc:652).  Cause: the pipeline registry is
keyed by the WriteBuffer's address, and the allocator hands the next stage's
WriteBuffer the address of the previous, closed one, which the registry still
listed as closed.  The pipeline used to be created by LZ4FlushScope, a local of
ProcessingLoop, i.e. on the buffer's own thread; when the scheduler started
that thread late, the stage's puts ran first and were refused.  The fix creates
the pipeline in WriteBuffer's constructor (LZ4FlushOpen, one more anchored edit
of oracle/kingdb_hook.py), before the thread starts.

KDB_LZ4_FLUSH_SCOPE_DELAY_US (a test knob of flush_hook.cc) holds the
ProcessingLoop thread back for 200 ms, which makes the old failure
deterministic: every stage after the first loses all of its puts.  The test
runs KingDB's own test on the CPU-model build of KingDB + hooks
(oracle/Makefile `kingdb_san SAN=none`: the same flush_hook.cc over
tests/cpp/abi_cpu_model.cc).
"""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.skipif(not os.path.isdir("/root/reference"),
                                reason="the KingDB builds compile the reference tree in place")

TEST_DB = os.path.join(ROOT, "oracle", "_ref", "kingdb_cpumodel", "test_db")


@pytest.fixture(scope="module")
def cpumodel_test_db():
    b = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "kingdb_san", "SAN=none"],
                       capture_output=True, text=True, timeout=1200)
    assert b.returncode == 0, b.stderr[-3000:]
    return TEST_DB


def test_puts_right_after_open_are_accepted_when_the_flush_thread_starts_late(cpumodel_test_db, tmp_path):
    env = dict(os.environ, LEVELDB_TESTS="SingleThreadSmallEntriesCompaction", KDB_LZ4_FLUSH_SCOPE_DELAY_US="200000")
    r = subprocess.run([cpumodel_test_db], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600,
                       errors="replace")
    assert "WriteBuffer is closing" not in r.stderr, r.stderr[-2000:]
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-1500:])
    assert "PASSED 1 tests" in r.stderr
    # every option stage ran (13: IterateOverOptions, test_db.cc:185-266)
    assert r.stdout.count("Database Options: Stage") == 13
