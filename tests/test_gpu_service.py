"""GPU: the resident services of the per-call path (kingdb_amd/csrc/
service.h): LZ4_decompress_safe_partial (lz4.cc:1050-1053) and
LZ4_compress_limitedOutput (lz4.cc:664-682) one value per call, served by
waves that stay on the device between calls.

Parity is the batch kernels' (the same decode_block / compress_block): every
return code of the reference's malformed-block fixtures at the per-call sizes
(tests/golden/malformed.npz), the reference's limited-output return codes and
blocks (limited_output.npz), outputs equal to the oracle's, from one thread
and from 16 threads at once; the waves leave once idle, and with
KDB_LZ4_SERVICE=0 (one launch per call) the results are the same.
"""
import ctypes
import os
import random
import subprocess
import sys
import threading
import time

import pytest

import oracle
from conftest import ROOT, load_golden, split

pytestmark = pytest.mark.gpu

SMALL = 8192   # the service's class (service.h kSvcMaxOut)


def _stats(gpu, dev=0):
    from kingdb_amd import _lib
    a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    assert _lib.load().kdb_lz4_service_stats(dev, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == 0
    return a.value, b.value, c.value


def test_service_malformed_codes(gpu):
    g = load_golden("malformed.npz")
    blocks = split(g["blk"], g["blk_off"], g["blk_len"])
    n = 0
    for i, b in enumerate(blocks):
        size, tgt = int(g["size"][i]), int(g["target"][i])
        if size > SMALL or len(b) > SMALL + SMALL // 255 + 24:
            continue
        r, out = gpu.decompress_safe_partial(b, tgt, size)
        assert r == int(g["ret"][i]), (i, r, int(g["ret"][i]))
        if r > 0 and g["cmp"][i]:
            o = int(g["out_off"][i])
            assert out == g["out"][o:o + r].tobytes(), i
        n += 1
    launches, served, alive = _stats(gpu)
    assert n > 1000 and launches >= 1, (n, launches)


def test_service_g1_and_random(gpu, orc):
    rng = random.Random(9)
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, 100, 300) + oracle.g1_values(pool, 4096, 100) + [b"", b"a" * 13, b"q" * 8192]
    vals += [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 8192))) for _ in range(20)]
    t0 = time.perf_counter()
    for v in vals:
        b = orc.compress(v)
        assert gpu.decompress_safe_partial(b, len(v), len(v)) == (len(v), v)
    dt = (time.perf_counter() - t0) / len(vals) * 1e6
    print(f"{len(vals)} calls, {dt:.1f} us per call (python included)")
    time.sleep(0.05)   # idle: the wave has left (KDB_LZ4_SERVICE_IDLE_US, 2 ms)
    launches, served, alive = _stats(gpu)
    assert alive == 0 and served >= len(vals), (launches, served, alive)


def test_service_compress_limited_output(gpu, orc):
    """The reference's limitedOutput return codes and blocks (values <= 4 KiB
    go to the compress service), and the G1 values at the bound."""
    g = load_golden("limited_output.npz")
    inputs = split(g["inp"], g["inp_off"], g["inp_len"])
    n = 0
    for i, x in enumerate(inputs):
        cap = int(g["cap"][i])
        r, b = gpu.compress_limited_output(x, cap)
        assert r == int(g["ret"][i]), (i, r, int(g["ret"][i]))
        if r:
            o = int(g["blk_off"][i])
            assert b == g["blk"][o:o + r].tobytes(), i
        n += len(x) <= 4096
    pool = oracle.g1_pool(orc)
    for x in oracle.g1_values(pool, 100, 200) + oracle.g1_values(pool, 4096, 50) + [b"", b"a", b"a" * 13]:
        r, b = gpu.compress_limited_output(x, orc.compress_bound(len(x)))
        assert b == orc.compress(x), len(x)
    launches, served, alive = _stats(gpu)
    assert n > 100 and launches >= 1, (n, launches)


def test_service_many_threads(gpu, orc):
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, 100, 64) + oracle.g1_values(pool, 4096, 64)
    blocks = [orc.compress(v) for v in vals]
    bad = []

    def worker(t):
        gpu.set_device(0)
        rng = random.Random(t)
        for _ in range(300):
            i = rng.randrange(len(vals))
            r = gpu.decompress_safe_partial(blocks[i], len(vals[i]), len(vals[i]))
            if r != (len(vals[i]), vals[i]):
                bad.append((t, i))
            c = gpu.compress_limited_output(vals[i], len(vals[i]) + len(vals[i]) // 255 + 16)
            if c[1] != blocks[i]:
                bad.append((t, i, "compress"))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not bad, bad[:5]


def test_service_off_is_the_launch_path(gpu, orc):
    code = ("import sys; sys.path.insert(0, %r); import kingdb_amd as K, oracle, ctypes; "
            "from kingdb_amd import _lib; K.set_device(0); o = oracle.Oracle(); "
            "v = oracle.g1_values(oracle.g1_pool(o), 4096, 20); "
            "assert all(K.decompress_safe_partial(o.compress(x), 4096, 4096) == (4096, x) for x in v); "
            "a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(); "
            "_lib.load().kdb_lz4_service_stats(0, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)); "
            "assert a.value == 0, a.value; print('ok')") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, KDB_LZ4_SERVICE="0"))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def _counters(dev=0):
    from kingdb_amd import _lib
    a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    assert _lib.load().kdb_lz4_service_counters(dev, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == 0
    return a.value, b.value, c.value


def test_service_posts_and_replies(gpu, orc):
    """Round 5's protocol (service.h): a request whose input fits its slot's
    post (<= 108 bytes) is taken from the poll itself, and a decode result of
    <= 108 bytes comes back in a reply record ahead of the done word.  Both
    paths must be the ones that ran (the counters, summed as waves exit), and
    give the oracle's bytes -- short values, values at the 108-byte edges,
    longer ones (fetched as before), and 40 threads at once, so that slots
    past the 16 posted ones take the fetch path beside them."""
    pool = oracle.g1_pool(orc)
    rng = random.Random(5)
    vals = oracle.g1_values(pool, 100, 200) + [b"", b"z", b"a" * 13]
    vals += [bytes(rng.randrange(256) for _ in range(n)) for n in (92, 93, 107, 108, 109, 110, 120, 200)]
    vals += [bytes(rng.choice(b"ab") for _ in range(n)) for n in (108, 109, 500, 3000)]
    time.sleep(0.05)
    p0, f0, r0 = _counters()
    for v in vals:
        b = orc.compress(v)
        assert gpu.decompress_safe_partial(b, len(v), len(v)) == (len(v), v), len(v)
        c = gpu.compress_limited_output(v, orc.compress_bound(len(v)))
        assert c == (len(b), b) or (len(v) == 0 and c[0] == len(b)), len(v)
    bad = []

    def worker(t):
        gpu.set_device(0)
        r = random.Random(t)
        for _ in range(100):
            v = vals[r.randrange(len(vals))]
            if gpu.decompress_safe_partial(orc.compress(v), len(v), len(v)) != (len(v), v):
                bad.append((t, len(v)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(40)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not bad, bad[:5]
    time.sleep(0.05)   # the waves leave (2 ms idle) and add their counters
    p1, f1, r1 = _counters()
    short = sum(1 for v in vals if len(v) <= 108)
    assert f1 - f0 >= short and r1 - r0 >= short // 2, (p1 - p0, f1 - f0, r1 - r0, short)


@pytest.mark.parametrize("busy", [0, 1])
def test_service_stress_threads(gpu, busy):
    """tests/cpp/svc_stress: 8 threads of per-call decodes and compressions of
    hook_mt-shaped values, each checked against the oracle's blocks; with
    `busy`, batch compressions run on the device meanwhile and the callers
    pause past the idle time (waves leave and are relaunched)."""
    exe = os.path.join(ROOT, "tests", "cpp", "svc_stress")
    if not os.path.exists(exe):
        pytest.fail("tests/cpp/svc_stress is not built (make -C tests/cpp)")
    r = subprocess.run([exe, "8", "300", "7", str(busy)], cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, KDB_ORACLE_SO=os.path.join(ROOT, "oracle", "liblz4_oracle.so")))
    assert r.returncode == 0 and "ok:" in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])


def test_service_request_numbers_wrap(gpu, orc):
    """A slot's request number wraps after 2^32 calls: 0 is never
    used (a zero-filled reply record or done word would pass for its answer),
    and a reply record left from the previous wrap cannot be taken for the
    first requests after it.  kdb_lz4_service_seed_requests puts every slot
    just before the wrap, with reply records of tag 0 (never written) and then
    of tag 1 (written one wrap ago), each with a valid checksum and return 0."""
    from kingdb_amd import _lib
    lib = _lib.load()
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, 100, 8)
    blocks = [orc.compress(v) for v in vals]
    for v, b in zip(vals, blocks):   # the services exist, this thread holds its slots
        assert gpu.decompress_safe_partial(b, len(v), len(v)) == (len(v), v)
        assert gpu.compress_limited_output(v, orc.compress_bound(len(v))) == (len(b), b)
    for req, tag in ((0xFFFFFFFF, 0), (0xFFFFFFFE, 1), (0xFFFFFFFD, 2)):
        assert lib.kdb_lz4_service_seed_requests(ctypes.c_uint32(req), ctypes.c_uint32(tag)) == 0
        for v, b in zip(vals, blocks):   # numbers req+1, ... across the wrap
            assert gpu.decompress_safe_partial(b, len(v), len(v)) == (len(v), v), (hex(req), tag)
            assert gpu.compress_limited_output(v, orc.compress_bound(len(v))) == (len(b), b), (hex(req), tag)
