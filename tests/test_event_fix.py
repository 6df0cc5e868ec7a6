"""CPU: the hook build's fix of KingDB's lost wake-up at Close,
made deterministic.

StorageEngine::Close notifies the data thread with Event::NotifyWait
(/root/reference/storage/storage_engine.h:110-111).  In the reference that is
a bare notify_one (thread/event_manager.h:44-46): if the data thread is still
in the last flush's index update, the notification is lost and its next
Event::Wait (:30-36) sleeps forever.  tests/cpp/test_event.cc forces exactly
that interleaving with a barrier (NotifyWait, then Wait) and is built against
the hook build's patched header (oracle/kingdb_hook.py: a flag set under the
event's mutex, Wait on the predicate) and against the reference's.
"""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="builds against the reference tree")


def test_notify_before_wait(tmp_path):
    src = tmp_path / "hook_src"
    subprocess.run(["python3", os.path.join(ROOT, "oracle", "kingdb_hook.py"), str(src)], check=True)
    cpp = os.path.join(ROOT, "tests", "cpp")
    b = subprocess.run(["make", "-s", "-B", "-C", cpp, "event", f"HOOK_SRC={src}"], capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-2000:]
    fixed = subprocess.run([os.path.join(cpp, "test_event_hook")], capture_output=True, text=True, timeout=60)
    assert (fixed.returncode, fixed.stdout.strip()) == (0, "returned")
    # the reference's Event under the same interleaving: the wake-up is lost
    ref = subprocess.run([os.path.join(cpp, "test_event_ref")], capture_output=True, text=True, timeout=60)
    assert (ref.returncode, ref.stdout.strip()) == (2, "lost wake-up")
