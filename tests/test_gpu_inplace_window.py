"""The in-place compressor's per-sequence window (lz4_compress.hip,
KDB_LZ4_SEQ_WINDOW): a sequence's count, literals and next input words come
out of a 256-byte window loaded at its start when they lie in it, and out of
global memory when they do not.  These values put matches and literal runs on
both sides of that window's edges -- sources 40..400 bytes back, literal runs
of 0..600 bytes, matches of 4..600 bytes, values ending mid-window -- and the
frames must equal the oracle's (the reference's algorithm, oracle/lz4_oracle.c)
byte for byte.  GPU only."""
import numpy as np
import pytest


def _value(rng, size):
    """A value of pieces: random literals, then a copy of bytes `dist` back."""
    out = bytearray(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    while len(out) < size:
        lit = int(rng.choice([0, 1, 3, 15, 16, 50, 120, 190, 194, 200, 260, 600]))
        out += rng.integers(0, 256, lit, dtype=np.uint8).tobytes()
        dist = int(rng.integers(40, 400))
        ml = int(rng.choice([4, 5, 18, 46, 60, 64, 65, 130, 187, 188, 189, 300, 600]))
        start = max(0, len(out) - dist)
        for i in range(ml):                        # overlapping copies allowed (dist < ml)
            out.append(out[start + i])
    return np.frombuffer(bytes(out[:size]), np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_inplace_window_edges_vs_oracle(gpu, orc, seed):
    import kingdb_amd as K
    from kingdb_amd import _lib
    from kingdb_amd.lz4 import DeviceBatch, DeviceBuffer, lib
    K.set_device(0)
    rng = np.random.default_rng(seed)
    # in-place sizes (8 KiB .. 65 546 B) plus a few that end just past a sequence
    sizes = [65536, 65546, 8193, 12289, 40000] + [int(rng.integers(8193, 65547)) for _ in range(59)]
    vals = [_value(rng, s) for s in sizes]
    sizes = np.array([v.size for v in vals], dtype=np.uint32)
    host = np.concatenate(vals)
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
