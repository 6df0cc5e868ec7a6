"""CPU: the host code around the kernels under ThreadSanitizer and
AddressSanitizer (race detection).

The host code is what has threads and buffers of its own: the drop-in
kdb::CompressorLZ4 (csrc/compressor.cc -- ThreadStorageLZ4 maps, per-thread
BatchStaging), the flush hook (csrc/flush_hook.cc -- client threads' intake,
the pipeline's worker, the flush thread's completion, the per-thread policy
state, the staging pool), the read hooks (csrc/read_hook.cc) and the HSTable
writer (csrc/hstable.cc).  Here they run over a CPU model of the C ABI
(tests/cpp/abi_cpu_model.cc, computing with the oracle), so the sanitizers see
every host-side access in this GPU-less container; the kernels are covered by
the GPU tests.

KingDB itself has data races of its own (e.g. WriteBuffer::WritePart reads
im_live_ outside its mutexes, write_buffer.cc:178; StorageEngine flags read
without locks); a TSan report counts against this build only when the access
it reports happens in our code (the first frame outside the C++ library).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CPP = os.path.join(ROOT, "tests", "cpp")
ORACLE = os.path.join(ROOT, "oracle")
OURS = ("flush_hook.cc", "read_hook.cc", "compressor.cc", "compressor.h", "lz4_flush.h", "lz4_read.h",
        "abi_cpu_model.cc", "hstable.cc", "hook_mt.cc", "ref_db.cc")


def _make(args, timeout=900):
    b = subprocess.run(["make", "-s", "-j8"] + args, capture_output=True, text=True, timeout=timeout)
    if b.returncode != 0 and "cannot find" in b.stderr and "san" in b.stderr:
        pytest.skip("no sanitizer runtime: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-3000:]


def _our_races(stderr: str) -> list:
    """TSan reports whose racy access is in our code: in each access's stack,
    the first frame outside the C++ library and the sanitizer runtime."""
    ours = []
    for block in stderr.split("=================="):
        if "WARNING: ThreadSanitizer" not in block:
            continue
        for stack in re.split(r"\n\s*\n", block):
            frames = re.findall(r"#\d+ ([^\n]+)", stack)
            first = next((f for f in frames if "/usr/include/" not in f and "libsanitizer" not in f
                          and "libtsan" not in f and "libstdc++" not in f), None)
            if first and any(o in first for o in OURS):
                ours.append(block.strip()[:3000])
                break
    return ours


def test_dropin_compressor_threads_tsan():
    _make(["-C", CPP, "compressor_san"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([os.path.join(CPP, "test_compressor_tsan"), "/tmp"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    assert "all checks passed" in r.stdout + r.stderr


def test_dropin_compressor_asan():
    _make(["-C", CPP, "compressor_san"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([os.path.join(CPP, "test_compressor_asan"), "/tmp"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    assert "all checks passed" in r.stdout + r.stderr


def test_hstable_writer_asan():
    _make(["-C", CPP, "asan"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([os.path.join(CPP, "test_hstable_asan"), "4", "100000"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    assert r.stdout.startswith("ok:")


needs_ref = pytest.mark.skipif(not os.path.isdir("/root/reference"),
                               reason="the KingDB sanitizer builds compile the reference tree in place")


@needs_ref
@pytest.mark.parametrize("devices", [1, 4])
def test_kingdb_hook_threads_tsan(tmp_path, devices):
    """4 client threads writing single-part and multipart values through the
    flush hook, then 4 readers (Get, MultipartReader) and an iteration through
    the read hooks; no race in our code.  With 4 modelled devices the flush
    pipeline runs one lane (worker, staging, stream) per device and the
    read-ahead spreads its batches over them: every batch ran on the device
    its stream belongs to (the model refuses any other), all four devices
    took batches, and every value reads back."""
    _make(["-C", ORACLE, "kingdb_san", "SAN=thread"])
    # small read-ahead batches, so the iteration runs its helper threads too
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=0 history_size=4", KDB_LZ4_READ_BATCH="32",
               KDB_LZ4_CPU_MODEL_DEVICES=str(devices), KDB_LZ4_FLUSH_DEVICES=str(devices),
               KDB_LZ4_READ_DEVICES=str(devices), KDB_LZ4_CPU_MODEL_STATS="1", KDB_LZ4_FLUSH_STATS="1")
    r = subprocess.run([os.path.join(ORACLE, "_ref", "kingdb_tsan", "hook_mt"), str(tmp_path / "db"), "4", "60"],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("ok:"), r.stdout
    ours = _our_races(r.stderr)
    assert not ours, "\n\n".join(ours[:3])
    per_dev = re.search(r"cpu_model_batches(( device\d+ \d+)+)", r.stderr)
    assert per_dev, r.stderr[-2000:]
    counts = [int(x) for x in re.findall(r"device\d+ (\d+)", per_dev.group(1))]
    assert len(counts) == devices and all(c > 0 for c in counts), per_dev.group(0)
    lanes = [ln for ln in r.stderr.splitlines() if ln.startswith("lz4_flush_lanes")]
    assert lanes and lanes[0].startswith(f"lz4_flush_lanes {devices}"), lanes


@needs_ref
def test_kingdb_hook_asan(tmp_path):
    """The same driver and the golden write streams (kdb_db, then --verify's
    Get / iterator / MultipartReader reads) under AddressSanitizer."""
    _make(["-C", ORACLE, "kingdb_san", "SAN=address"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", KDB_LZ4_READ_BATCH="32")
    exe = os.path.join(ORACLE, "_ref", "kingdb_asan")
    r = subprocess.run([os.path.join(exe, "hook_mt"), str(tmp_path / "mt"), "4", "40"], capture_output=True,
                       text=True, timeout=900, env=env)
    assert r.returncode == 0 and r.stdout.startswith("ok:"), r.stderr[-4000:]
    z = np.load(os.path.join(ROOT, "tests", "golden", "hstable_streams.npz"))
    for name in ("small", "edge", "multipart"):
        hs, ht, mps = (int(x) for x in z[f"{name}__opts"])
        s = tmp_path / f"{name}.bin"
        s.write_bytes(z[f"{name}__stream"].tobytes())
        db = tmp_path / f"db_{name}"
        args = [str(db), str(s), str(mps), str(hs), str(ht)]
        w = subprocess.run([os.path.join(exe, "kdb_db")] + args, capture_output=True, text=True, timeout=300, env=env)
        assert w.returncode == 0, w.stderr[-4000:]
        for f in z[f"{name}__files"]:
            got = (db / str(f)).read_bytes()
            want = z[f"{name}__file_{f}"].tobytes()
            assert got[:72] + got[8192:] == want[:72] + want[8192:], (name, f)
        v = subprocess.run([os.path.join(exe, "kdb_db"), "--verify"] + args, capture_output=True, text=True,
                           timeout=300, env=env)
        assert v.returncode == 0, v.stdout + v.stderr[-4000:]
