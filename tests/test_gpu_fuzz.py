"""A seeded fuzz batch through the device path against the oracle (GPU), and the
oracle against the reference on the same values (CPU).

Several thousand values in one DeviceBatch -- every size class of the
compressor and decoder (<= 4 KiB LDS-staged, 4-8 KiB, the in-place 8 KiB -
65 546 B class with its register window, byU32 above), the class boundaries
exactly, and data shaped to reach the rare paths: incompressible bytes (raw
fallback frames), tiny alphabets, periodic data with sparse mutations (long
matches: the in-place window's ml <= 187 test on both sides, literal runs
that do and do not end inside the previous match's window), far copies from
a shared pool (matches across the whole 64 KiB window), byte runs (long
run-length bytes).  The packed frame stream must have the oracle's length
and CRC32C (oracle/lz4_oracle.c, pinned to the reference's goldens), and
every value must round-trip through the device decoder.
"""
import numpy as np
import pytest


BOUNDARIES = [0, 1, 12, 13, 14, 63, 64, 4095, 4096, 4097, 6144, 8191, 8192, 8193, 65535, 65536, 65546, 65547,
              65548, 131072]


def _values(seed: int, n: int):
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    pool[::3] = rng.integers(97, 101, pool[::3].size, dtype=np.uint8)      # some structure in the pool
    sizes = []
    for i in range(n):
        r = rng.random()
        if r < 0.10:
            s = int(rng.integers(0, 64))
        elif r < 0.45:
            s = int(rng.integers(64, 4097))
        elif r < 0.60:
            s = int(rng.integers(4097, 8193))
        elif r < 0.97:
            s = int(rng.integers(8193, 65547))
        else:
            s = int(rng.integers(65547, 200000))
        sizes.append(s)
    sizes = BOUNDARIES + sizes
    out = []
    for s in sizes:
        kind = int(rng.integers(0, 6))
        if s == 0:
            v = np.zeros(0, np.uint8)
        elif kind == 0:                                  # incompressible: raw fallback frames
            v = rng.integers(0, 256, s, dtype=np.uint8)
        elif kind == 1:                                  # tiny alphabet
            v = rng.integers(0, int(rng.integers(2, 5)), s, dtype=np.uint8) + 65
        elif kind == 2:                                  # periodic + sparse mutations: long matches
            p = int(rng.integers(1, 400))
            base = rng.integers(0, 256, p, dtype=np.uint8)
            v = np.tile(base, s // p + 1)[:s].copy()
            m = int(rng.integers(0, max(1, s // 150)))
            if m:
                v[rng.integers(0, s, m)] = rng.integers(0, 256, m, dtype=np.uint8)
        elif kind == 3:                                  # far copies from a shared pool
            pieces, got = [], 0
            while got < s:
                ln = int(rng.integers(4, 600))
                at = int(rng.integers(0, pool.size - ln))
                pieces.append(pool[at:at + ln])
                got += ln
            v = np.concatenate(pieces)[:s]
        elif kind == 4:                                  # byte runs of every length
            lens = rng.integers(1, 2000, s // 8 + 2)
            vals = rng.integers(0, 256, lens.size, dtype=np.uint8)
            v = np.repeat(vals, lens)[:s]
            if v.size < s:
                v = np.concatenate([v, np.zeros(s - v.size, np.uint8)])
        else:                                            # text-like: words from a small vocabulary
            words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9)), dtype=np.uint8)) + b" "
                     for _ in range(64)]
            pick = rng.integers(0, 64, s // 3 + 1)
            v = np.frombuffer(b"".join(words[k] for k in pick), np.uint8)[:s]
        out.append(np.ascontiguousarray(v, dtype=np.uint8))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n", [(1, 3000), (2, 3000)])
def test_fuzz_batch_vs_oracle(gpu, orc, seed, n):
    import kingdb_amd as K
    from kingdb_amd import _lib
    from kingdb_amd.lz4 import DeviceBatch, DeviceBuffer, lib
    K.set_device(0)
    vals = _values(seed, n)
    sizes = np.array([v.size for v in vals], dtype=np.uint32)
    host = np.concatenate(vals) if sizes.sum() else np.zeros(1, np.uint8)
    off = np.zeros(len(vals), np.uint64)
    off[1:] = np.cumsum(sizes[:-1].astype(np.uint64))
    src = DeviceBuffer(host.nbytes + 64)
    src.upload(host)
    b = DeviceBatch._layout(sizes, src, None)
    st = K.Stream()
    b.compress(st)
    b.decompress(st)
    st.sync()
    cst, dst = b.status()
    assert (cst == 0).all() and (dst == 0).all()
    dense, doff, tot = DeviceBuffer(b.frames.nbytes), DeviceBuffer(8 * b.n), DeviceBuffer(8)
    _lib.check(lib().kdb_lz4_pack_frames(None, b.frames.ptr, b._p(2), b._p(3), b.n, dense.ptr, doff.ptr, tot.ptr),
               "pack")
    total = int(tot.download(8).view(np.uint64)[0])
    got = (total, orc.crc32c_array(dense.download(total)))
    exp = orc.frames_digest(host, off, sizes)
    assert got == tuple(exp), (got, exp)
    assert b.roundtrip_ok()
    for x in (dense, doff, tot):
        x.free()
    b.free()


@pytest.mark.parametrize("seed", [1, 2])
def test_fuzz_oracle_equals_reference(seed):
    """CPU (not gpu): on the same fuzz values the oracle's frame digest equals
    the reference's own CompressorLZ4::Compress (oracle/_ref, compiled from
    /root/reference), so the GPU test above is pinned to the reference."""
    import os

    import oracle
    if not os.path.exists(oracle.REF_SO):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    vals = _values(seed, 3000)
    sizes = np.array([v.size for v in vals], dtype=np.uint32)
    host = np.concatenate(vals)
    off = np.zeros(len(vals), np.uint64)
    off[1:] = np.cumsum(sizes[:-1].astype(np.uint64))
    assert tuple(oracle.Oracle().frames_digest(host, off, sizes)) == tuple(
        oracle.Reference().frames_digest(host, off, sizes))

