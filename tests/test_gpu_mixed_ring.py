"""The mixed decode launch when every value fits byU16 (lz4_decompress.hip:
launch_mixed<F, 4096u>): the ring decoder with its 4 KiB input ring, refilled
2 KiB at a time, and the ring pass claiming from the 32 work queues.  Batches
of more values than the launch has waves, so the claims go through the queues
(a batch no larger than the grid is a direct launch), and no value above
65 546 bytes, so the 8 KiB ring is not the one taken.  GPU only.

* block mode: mutated, truncated and undersized blocks -- the return codes and
  outputs must equal the oracle's (oracle/lz4_oracle.c, pinned to the
  reference by tests/golden/malformed.npz), whichever ring refill a sequence's
  bytes straddle;
* frame mode: a mixed batch (100 B / 4 KiB / 8 KiB - 64 KiB values) whose
  frames must equal the oracle's byte for byte and round-trip.
"""
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def test_mutants_byu16_ring_vs_oracle(gpu, orc):
    rng = random.Random(2024)
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, 4096, 6) + oracle.g1_values(pool, 100, 6) + oracle.g1_values(pool, 65536, 3)
    for _ in range(20):
        n = rng.choice([300, 4096, 9000, 20000, 40000, 65000])
        p = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 90)))
        vals.append((p * (n // len(p) + 1))[:n])
    blocks, sizes = [], []
    for v in vals:
        b = orc.compress(v)
        for _ in range(10):
            m = bytearray(b)
            for _ in range(rng.randrange(1, 4)):
                m[rng.randrange(len(m))] = rng.randrange(256)
            blocks.append(bytes(m))
            sizes.append(len(v))
        blocks += [b[:rng.randrange(1, len(b))], b, b, b]
        sizes += [len(v), max(len(v) - rng.randrange(1, 20), 0), min(len(v) + 7, 65546), max(len(v) - 1, 0)]
    # more blocks than the launch has waves (a work-queue launch), in a shuffled order
    order = list(range(len(blocks))) * 14
    rng.shuffle(order)
    blocks = [blocks[i] for i in order]
    sizes = [sizes[i] for i in order]
    assert len(blocks) > 5000 and max(sizes) <= 65546 and max(sizes) > 8192
    got = gpu.decompress_blocks(blocks, sizes)
    import kingdb_amd as K
    assert K.last_kernels() == ["lz4_decompress_mixed_kernel<false>"]
    memo = {}
    for i, ((r, out), b, s) in enumerate(zip(got, blocks, sizes)):
        if (b, s) not in memo:
            memo[(b, s)] = orc.decompress(b, s)
        er, eout = memo[(b, s)]
        assert r == er, (i, r, er)
        if r > 0:
            assert out == eout, i


def test_mixed_frames_byu16_ring_vs_oracle(orc):
    import kingdb_amd as K
    from kingdb_amd import _lib
    from kingdb_amd.lz4 import DeviceBatch, DeviceBuffer, lib
    K.set_device(0)
    rng = np.random.default_rng(5)
    pool = oracle.g1_pool(orc)
    sizes = np.array([100] * 5400 + [4096] * 540 + [int(x) for x in rng.integers(8193, 65547, 60)], dtype=np.uint32)
    rng.shuffle(sizes)
    starts = rng.integers(0, pool.size - 65546, sizes.size)
    vals = [pool[s:s + z] for s, z in zip(starts, sizes)]
    host = np.concatenate(vals)
    off = np.zeros(sizes.size, np.uint64)
    off[1:] = np.cumsum(sizes[:-1].astype(np.uint64))
    src = DeviceBuffer(host.nbytes + 64)
    src.upload(host)
    b = DeviceBatch._layout(sizes, src, None)
    st = K.Stream()
    b.compress(st)
    b.decompress(st)
    st.sync()
    assert "lz4_decompress_mixed_kernel<true>" in K.last_kernels()
    cst, dst = b.status()
    assert (cst == 0).all() and (dst == 0).all()
    dense, doff, tot = DeviceBuffer(b.frames.nbytes), DeviceBuffer(8 * b.n), DeviceBuffer(8)
    _lib.check(lib().kdb_lz4_pack_frames(None, b.frames.ptr, b._p(2), b._p(3), b.n, dense.ptr, doff.ptr, tot.ptr),
               "pack")
    total = int(tot.download(8).view(np.uint64)[0])
    got = (total, orc.crc32c_array(dense.download(total)))
    assert got == tuple(orc.frames_digest(host, off, sizes))
    assert b.roundtrip_ok()
    for x in (dense, doff, tot):
        x.free()
    b.free()


def _edge_value(rng, n, dists):
    """Random bytes with 40-byte copies from `dists` back every ~120 bytes, and
    periodic runs (offsets 1..63, longer than the offset): the oracle's parse
    turns them into fast-path sequences whose matches start at those offsets."""
    x = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    p, k = max(dists) + 64, 0
    while p + 300 < n:
        if k % 5 == 4:
            o = int(rng.integers(1, 64))
            ln = int(rng.integers(o + 1, o + 140))
            for i in range(ln):
                x[p + i] = x[p + i - o]
            p += ln
        else:
            d = dists[k % len(dists)]
            x[p:p + 40] = x[p - d:p - d + 40]
            p += 40
        p += int(rng.integers(20, 61))
        k += 1
    return bytes(x)


def test_ring_edge_offsets_vs_oracle(gpu, orc):
    """The ring decoder's fast path (lz4_decompress.hip decode_ring): the 8 KiB
    input ring's launch (a batch with a 1 MiB part) stores whole 64-lane steps
    into the 4 KiB output ring, so a match from 4 032 bytes back or more is read
    from the wave's own output in HBM; the 4 KiB input ring's launch (values of
    at most 64 KiB) keeps exact stores.  Matches from just inside to just past
    both edges (4 032 / 4 096 back), and periodic ones, decode to the input;
    the frames equal the oracle's."""
    rng = np.random.default_rng(4032)
    dists = [4000, 4031, 4032, 4033, 4063, 4064, 4065, 4095, 4096, 4097, 5000]
    big = [_edge_value(rng, 1 << 20, dists), _edge_value(rng, 300000, dists[::-1])]
    small = [_edge_value(rng, n, dists) for n in (9000, 20000, 65536)]
    for vals in (big + small, small):
        want = [orc.frame(v) for v in vals]
        frames = gpu.compress_frames(vals)
        assert frames == want
        back = gpu.decompress_frames(frames, [len(v) for v in vals])
        assert all(st == 0 and out == v for (st, out), v in zip(back, vals))
        blocks = [orc.compress(v) for v in vals]
        dec = gpu.decompress_blocks(blocks, [len(v) for v in vals])
        assert all(r == len(v) and out == v for (r, out), v in zip(dec, vals))


def test_ring_partial_decode_vs_oracle(gpu, orc):
    """LZ4_decompress_safe_partial with a target below the output size through the
    ring decoder (outputs above the LDS decoder's 8 KiB: decode_ring's oexit =
    min(target, oend - 12), lz4.cc:908-910): the decode stops after the sequence
    that reaches the target, on both ring launches; return codes and bytes equal
    the oracle's, whose partial decode malformed.npz pins to the reference."""
    rng = np.random.default_rng(908)
    pool = oracle.g1_pool(orc)
    big = [bytes(pool[:1 << 20]), bytes(pool[1 << 20:(1 << 20) + 300000])]
    small = [bytes(pool[o:o + n]) for o, n in ((5000, 9000), (70000, 30000), (200000, 65536))]
    for vals in (big + small, small):
        blocks, sizes, targets = [], [], []
        for v in vals:
            b = orc.compress(v)
            for t in (1, 64, 4031, 4097, len(v) // 3, len(v) - 13, len(v) - 1,
                      int(rng.integers(1, len(v)))):
                blocks.append(b)
                sizes.append(len(v))
                targets.append(int(t))
        got = gpu.decompress_blocks(blocks, sizes, targets)
        for i, ((r, out), b, s, t) in enumerate(zip(got, blocks, sizes, targets)):
            er, eout = orc.decompress(b, s, t)
            assert r == er, (i, s, t, r, er)
            assert out == eout, (i, s, t)
