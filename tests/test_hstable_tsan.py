"""CPU: the host-side HSTable writer (kingdb_amd/csrc/hstable.cc) under
ThreadSanitizer -- its parallel append path (append_fast on the worker pool)
and the pooled offset-array encoding, driven by 4 host threads with a writer
each (tests/cpp/test_hstable_tsan.cc).  TSan reports make it exit 66; every
writer's files must equal a writer fed one entry per call (the serial path)."""
import os
import subprocess

import pytest

from conftest import ROOT

CPP = os.path.join(ROOT, "tests", "cpp")


def test_hstable_parallel_append_tsan():
    b = subprocess.run(["make", "-s", "-C", CPP, "tsan"], capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "tsan" in (b.stderr + b.stdout).lower() and "cannot find" in b.stderr:
        pytest.skip("no ThreadSanitizer runtime: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([os.path.join(CPP, "test_hstable_tsan"), "4", "300000"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("ok:")
