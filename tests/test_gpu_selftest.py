"""GPU: the compressor's lane-order guard (kingdb_amd/csrc/selftest.hip).

The exchange tables of lz4_compress.hip rest on one LDS behaviour (the lanes
of one ds_mskor_rtn_b32 that hit the same dword apply in ascending lane
order).  Every device the library binds runs a self-test of it first:
* kdb_lz4_set_device runs it, and it passes on MI355X;
* a device that fails it compresses nothing -- every compress entry point
  returns KDB_LZ4_EUNSUPPORTED (the scalar mirror: 0), never a frame
  (KDB_LZ4_SELFTEST_FORCE_FAIL=1 drives that path in a child process);
* decompression does not depend on it and keeps working.
Also: the library names the kernels a batch queued (kdb_lz4_last_kernels),
which bench.py uses for its roofline label.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_selftest_ran_and_passed(gpu):
    import kingdb_amd as K
    K.set_device(0)
    state, bad = K.selftest(0)
    assert state == 1 and bad == 0
    assert K.get_device() == 0


def test_selftest_failure_blocks_compression():
    code = r'''
import sys
sys.path.insert(0, %r)
import kingdb_amd as K
from kingdb_amd import _lib
K.set_device(0)
state, bad = K.selftest(0)
assert state == -1 and bad >= 1, (state, bad)
try:
    K.compress_frames([b"abc" * 100])
    raise SystemExit("compress_frames returned frames on a failed device")
except RuntimeError as e:
    assert str(_lib.EUNSUPPORTED) in str(e) or "EUNSUPPORTED" in str(e), e
assert K.compress_limited_output(b"abc" * 100, 400) == (0, b"")
frame = bytes([0, 0, 0, 0, 3, 0, 0, 0]) + b"xyz"          # a raw-fallback frame decodes without the table
st, out = K.decompress_frames([frame], [3])[0]
assert st == 0 and out == b"xyz", (st, out)
print("ok")
''' % ROOT
    env = dict(os.environ, KDB_LZ4_SELFTEST_FORCE_FAIL="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_last_kernels_names(gpu):
    """A launch queues one kernel per size class its length bounds allow (the
    batch API's lower bound is 0, so the classes below max_len launch too and
    return at once): the names are rocprof's."""
    import kingdb_amd as K
    K.compress_frames([b"x" * 4096] * 4)
    assert K.last_kernels() == ["lz4_compress_kernel<true, true, 1u, 10u>"]   # batched emission
    K.compress_frames([b"x" * 100] * 4)
    assert K.last_kernels() == ["lz4_compress_kernel<true, true, 0u, 10u>"]   # short values: per sequence
    K.compress_frames([b"x" * 6000] * 4)
    assert K.last_kernels() == ["lz4_compress_kernel<true, true, 1u, 10u>", "lz4_compress_kernel<true, false, 1u, 1u>"]
    K.compress_frames([b"x" * 4096, b"y" * 20000])
    assert K.last_kernels() == ["lz4_compress_mixed_kernel<true, 10u>", "lz4_compress_kernel<true, false, 1u, 1u>"]
    K.compress_frames([b"x" * 100000])                  # byU32, every value <= 1 MiB: the compact table
    assert "lz4_compress_big_compact_kernel<true>" in K.last_kernels()
    K.compress_frames([b"x" * 100000, b"z" * ((1 << 20) + 1)])
    assert "lz4_compress_big_kernel<true, true>" in K.last_kernels()
    K.decompress_frames(K.compress_frames([b"x" * 4096] * 4), [4096] * 4)
    assert K.last_kernels() == ["lz4_decompress_kernel<true, 3u>"]     # every frame <= 3 057 B
    import numpy as np
    noise = np.random.default_rng(7).integers(0, 256, 4096, dtype=np.uint8).tobytes()   # a 4 104 B raw frame
    K.decompress_frames(K.compress_frames([noise, b"x" * 4096]), [4096] * 2)
    assert K.last_kernels() == ["lz4_decompress_kernel<true, 5u>"]


@pytest.mark.parametrize("n,shift", [(0, 0), (1, 0), (3, 1), (5, 0), (1023, 3), (4096, 0), (65537, 2),
                                     ((1 << 20) + 3, 1)])
def test_max_u32_reduction(gpu, n, shift):
    """kdb_lz4_max_u32 (the decoder's max_in for a device-resident batch):
    the exact maximum at ragged lengths, 16-byte-aligned or not (shift dwords)."""
    import ctypes

    import numpy as np

    import kingdb_amd as K
    from kingdb_amd import _lib
    from kingdb_amd.lz4 import DeviceBuffer, lib
    K.set_device(0)
    rng = np.random.default_rng(n + shift)
    v = rng.integers(0, 1 << 20, size=n, dtype=np.uint32)
    if n:
        v[rng.integers(0, n)] = (1 << 31) + 7          # one large value anywhere (tail included)
    buf = DeviceBuffer(4 * (n + shift) + 64)
    if n:
        buf.upload(v, offset=4 * shift)
    out = DeviceBuffer(4)
    _lib.check(lib().kdb_lz4_max_u32(None, buf.ptr + 4 * shift, n, out.ptr), "max_u32")
    r = ctypes.c_uint32(123)
    _lib.check(lib().kdb_lz4_memcpy_d2h(ctypes.addressof(r), out.ptr, 4, None), "d2h")
    _lib.check(lib().kdb_lz4_stream_sync(None), "sync")
    assert r.value == (int(v.max()) if n else 0)
