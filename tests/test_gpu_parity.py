"""GPU: the gfx950 kernels (through the C ABI) against the reference-generated
golden fixtures and the oracle.  Bit-exact for every byte and return code."""
import random

import numpy as np
import pytest

import oracle
from conftest import load_golden, split

pytestmark = pytest.mark.gpu


def test_kat_blocks_frames(gpu):
    g = load_golden("kat_blocks.npz")
    inputs = split(g["inp"], g["inp_off"], g["inp_len"])
    blocks = split(g["blk"], g["blk_off"], g["blk_len"])
    frames = split(g["frm"], g["frm_off"], g["frm_len"])
    got = gpu.compress_blocks(inputs)
    for name, (r, b), exp in zip(g["names"], got, blocks):
        assert r == len(exp) and b == exp, name
    assert gpu.compress_frames(inputs) == frames
    dec = gpu.decompress_blocks(blocks, [len(x) for x in inputs])
    for name, (r, out), x in zip(g["names"], dec, inputs):
        assert r == len(x) and out == x, name
    fdec = gpu.decompress_frames(frames, [len(x) for x in inputs])
    for name, (st, out), x in zip(g["names"], fdec, inputs):
        assert st == 0 and out == x, name
    # launches whose values are all <= 4 KiB take the tagged-table kernel
    small = [i for i, x in enumerate(inputs) if len(x) <= 4096]
    sin = [inputs[i] for i in small]
    got = gpu.compress_blocks(sin)
    for i, (r, b) in zip(small, got):
        assert r == len(blocks[i]) and b == blocks[i], g["names"][i]
    assert gpu.compress_frames(sin) == [frames[i] for i in small]


def test_limited_output(gpu):
    g = load_golden("limited_output.npz")
    inputs = split(g["inp"], g["inp_off"], g["inp_len"])
    got = gpu.compress_blocks(inputs, caps=[int(c) for c in g["cap"]])
    for i, ((r, b), ret) in enumerate(zip(got, g["ret"])):
        assert r == int(ret), i
        if r:
            o = int(g["blk_off"][i])
            assert b == g["blk"][o:o + r].tobytes(), i


def test_malformed_return_codes(gpu):
    g = load_golden("malformed.npz")
    blocks = split(g["blk"], g["blk_off"], g["blk_len"])
    sizes = [int(s) for s in g["size"]]
    targets = [int(t) for t in g["target"]]
    got = gpu.decompress_blocks(blocks, sizes, targets)
    for i, (r, out) in enumerate(got):
        assert r == int(g["ret"][i]), (i, r, int(g["ret"][i]))
        if r > 0 and g["cmp"][i]:
            o = int(g["out_off"][i])
            assert out == g["out"][o:o + r].tobytes(), i


def test_decompress_mutants_vs_oracle(gpu, orc):
    """Return codes and outputs of mutated, truncated and undersized blocks equal
    the oracle's (pinned to the reference by malformed.npz): every error must be
    caught at the same input position whichever decoder path a sequence takes."""
    rng = random.Random(77)
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, 4096, 12) + oracle.g1_values(pool, 100, 12) + oracle.g1_values(pool, 65536, 4)
    for _ in range(24):
        n = rng.choice([20, 300, 2000, 4096, 8000, 30000, 70000])   # > 8 KiB: the ring decoder
        p = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 90)))
        vals.append((p * (n // len(p) + 1))[:n])
    blocks, sizes = [], []
    for v in vals:
        b = orc.compress(v)
        for k in range(8):
            m = bytearray(b)
            for _ in range(rng.randrange(1, 4)):
                m[rng.randrange(len(m))] = rng.randrange(256)
            blocks.append(bytes(m))
            sizes.append(len(v))
        blocks += [b[:rng.randrange(1, len(b))], b, b, b]
        sizes += [len(v), max(len(v) - rng.randrange(1, 20), 0), len(v) + 7, max(len(v) - 1, 0)]
    got = gpu.decompress_blocks(blocks, sizes)
    for i, ((r, out), b, s) in enumerate(zip(got, blocks, sizes)):
        er, eout = orc.decompress(b, s)
        assert r == er, (i, r, er)
        if r > 0:
            assert out == eout, i


def test_g1_db_bench_values(gpu, orc):
    """db_bench G1 values (SURVEY KATs T3-T5) compressed in one launch per size."""
    g = load_golden("g1_db_bench.npz")
    pool = oracle.g1_pool(orc)
    for size, count in ((100, 1000), (4096, 1000), (65536, 16)):
        vals = oracle.g1_values(pool, size, count)
        got = gpu.compress_blocks(vals)
        assert [r for r, _ in got] == list(g[f"s{size}_blk_len"])
        assert orc.crc32c(b"".join(b for _, b in got)) == int(g[f"s{size}_blk_crc"][0])
        frames = gpu.compress_frames(vals)
        assert [len(f) for f in frames] == list(g[f"s{size}_frm_len"])
        assert orc.crc32c(b"".join(frames)) == int(g[f"s{size}_frm_crc"][0])
        back = gpu.decompress_frames(frames, [size] * count)
        assert all(st == 0 and out == v for (st, out), v in zip(back, vals))


def test_test_db_generators(gpu):
    g = load_golden("test_db_generators.npz")
    for name in ("g2", "g3"):
        for size in (100, 4096):
            data = g[f"{name}_{size}_inp"]
            lens = g[f"{name}_{size}_frm_len"]
            off = np.concatenate([[0], np.cumsum(lens)[:-1]])
            frames = split(g[f"{name}_{size}_frm"], off, lens)
            vals = [data[i * size:(i + 1) * size].tobytes() for i in range(len(lens))]
            assert gpu.compress_frames(vals) == frames
            back = gpu.decompress_frames(frames, [size] * len(vals))
            assert all(st == 0 and out == v for (st, out), v in zip(back, vals))


def test_test_compression_shape(gpu):
    """unit-tests/test_compression.cc:43-125 on the GPU path."""
    g = load_golden("test_compression.npz")
    key = b"0x10c095000-0"
    value = (key * (442837 // len(key) + 1))[:442837]
    chunks = [value[i:i + 65536] for i in range(0, len(value), 65536)]
    frames = gpu.compress_frames(chunks)
    assert b"".join(frames) == g["frames"].tobytes()
    back = gpu.decompress_frames(frames, [len(c) for c in chunks])
    assert b"".join(out for _, out in back) == value


def test_scalar_mirrors(gpu, orc):
    rng = random.Random(5)
    for n in (0, 1, 12, 13, 100, 4096, 65546):
        x = bytes(rng.choice(b"abcd") for _ in range(n))
        bound = orc.compress_bound(n)
        r, b = gpu.compress_limited_output(x, bound)
        assert b == orc.compress(x)
        assert gpu.decompress_safe_partial(b, n, n) == (n, x) if n else True
        r2, _ = gpu.compress_limited_output(x, max(bound // 3, 0))
        exp = orc.compress(x, max(bound // 3, 0))
        assert r2 == (0 if exp is None else len(exp))


def test_random_vs_oracle(gpu, orc):
    rng = random.Random(2024)
    vals = []
    for _ in range(400):
        n = rng.choice([rng.randrange(0, 64), rng.randrange(64, 5000), rng.randrange(5000, 65547)])
        k = rng.randrange(4)
        if k == 0:
            v = bytes(rng.randrange(256) for _ in range(min(n, 3000))) * (n // 3000 + 1)
        elif k == 1:
            v = bytes(rng.choice(b"xy") for _ in range(n))
        elif k == 2:
            p = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 70)))
            v = p * (n // len(p) + 1)
        else:
            v = bytes(min(255, int(rng.expovariate(0.2))) for _ in range(n))
        vals.append(v[:n])
    got = gpu.compress_frames(vals)
    for v, f in zip(vals, got):
        assert f == orc.frame(v)


def test_device_g1_generator_matches_oracle(gpu, orc):
    from kingdb_amd.lz4 import DeviceBuffer, lib
    d = DeviceBuffer(1000 * 100)
    assert lib().kdb_lz4_gen_g1(d.ptr, 0, 1000, 301, None) == 0
    assert d.download(100000).tobytes() == orc.g1_pieces(1000).tobytes()
    assert lib().kdb_lz4_gen_g1(d.ptr, 123456, 10, 301, None) == 0
    assert d.download(1000).tobytes() == orc.g1_pieces(123466)[123456 * 100:].tobytes()


def test_device_batch_roundtrip_g1_long(gpu, orc):
    """64Ki x 4 KiB G1-long values resident in HBM: frames byte-identical to the
    oracle on a sample, full round trip bit-exact (size-independent property)."""
    n, size = 65536, 4096
    b = gpu.DeviceBatch.g1_long(n, size)
    b.compress()
    b.decompress()
    cst, dst = b.status()
    assert (cst == 0).all() and (dst == 0).all()
    assert (b.out_lens() == size).all()
    src = b.src.download(n * size)
    out = b.out.download(n * size)
    assert np.array_equal(src, out)
    flen = b.frame_lens()
    frames = b.frames.download(n * b.slot)
    for i in list(range(0, n, 997)) + [n - 1]:
        exp = orc.frame(src[i * size:(i + 1) * size].tobytes())
        got = frames[i * b.slot:i * b.slot + int(flen[i])].tobytes()
        assert got == exp, i
    b.free()


def test_device_batch_mixed_config4(gpu, orc):
    """SURVEY §8d config 4 shape (100 B / 4 KiB / 64 KiB parts) in one batch,
    plus the class edges (4096/4097, 8192/8193, 65546/65547): every size class
    launch of compress and decompress, frames byte-identical to the oracle on a
    sample, full round trip bit-exact."""
    from kingdb_amd.lz4 import mixed_sizes
    sizes = mixed_sizes(6000, mix=((100, 0.6), (4096, 0.25), (65536, 0.05), (4097, 0.02), (8192, 0.02),
                                   (8193, 0.02), (65546, 0.01), (65547, 0.01), (13, 0.01), (12, 0.01)))
    b = gpu.DeviceBatch.g1_long_sizes(sizes)
    b.compress()
    b.decompress()
    assert b.roundtrip_ok()
    src = b.src.download(b.raw_bytes)
    flen = b.frame_lens()
    frames = b.frames.download()
    for i in list(range(0, b.n, 37)) + [b.n - 1]:
        o, sz = int(b.src_off[i]), int(sizes[i])
        exp = orc.frame(src[o:o + sz].tobytes())
        fo = int(b.frame_off[i])
        assert frames[fo:fo + int(flen[i])].tobytes() == exp, (i, sz)
    b.free()


def test_device_scan_sizes(gpu):
    """launch_exclusive_scan (three-launch multi-block scan, pack.hip) at tile
    edges, and its single-workgroup fallback past 4 Mi elements, through
    kdb_lz4_pack_frames' offsets and total."""
    from kingdb_amd import _lib
    from kingdb_amd.lz4 import DeviceBuffer, lib
    rng = np.random.default_rng(4)
    for n in (1, 4095, 4096, 4097, 70001, (4 << 20) + 5):
        lens = rng.integers(0, 8, n).astype(np.uint32)
        src = DeviceBuffer(n * 8 + 64)
        src.upload(rng.integers(0, 256, n * 8, dtype=np.uint8))
        so = DeviceBuffer(8 * n)
        so.upload(np.arange(n, dtype=np.uint64) * 8)
        ln = DeviceBuffer(4 * n)
        ln.upload(lens)
        dst = DeviceBuffer(int(lens.sum()) + 64)
        doff = DeviceBuffer(8 * n)
        tot = DeviceBuffer(8)
        _lib.check(lib().kdb_lz4_pack_frames(None, src.ptr, so.ptr, ln.ptr, n, dst.ptr, doff.ptr, tot.ptr), "pack")
        exp = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))])
        assert np.array_equal(doff.download(8 * n).view(np.uint64), exp[:-1]), n
        assert int(tot.download(8).view(np.uint64)[0]) == int(exp[-1]), n
        for b in (src, so, ln, dst, doff, tot):
            b.free()


def test_pack_frames(gpu):
    """kdb_lz4_pack_frames: ragged lengths, unaligned source and destination."""
    from kingdb_amd import lz4 as L
    rng = np.random.default_rng(3)
    n = 5000
    lens = rng.integers(0, 700, n).astype(np.uint32)
    lens[::97] = 0
    gaps = rng.integers(0, 40, n).astype(np.uint64)
    src_off = np.zeros(n, np.uint64)
    src_off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    src = rng.integers(0, 256, int(src_off[-1]) + int(lens[-1]) + 64).astype(np.uint8)
    d_src = L.DeviceBuffer(src.nbytes)
    d_src.upload(src)
    meta = L.DeviceBuffer(n * 20 + 8)
    meta.upload(np.concatenate([src_off.view(np.uint8), lens.view(np.uint8)]))
    total = int(lens.sum())
    d_dst = L.DeviceBuffer(total + 64 + 3)
    d_dst.memset(0xAB)
    from kingdb_amd import _lib
    _lib.check(L.lib().kdb_lz4_pack_frames(None, d_src.ptr, meta.ptr, meta.ptr + 8 * n, n, d_dst.ptr + 3,
                                           meta.ptr + 12 * n, meta.ptr + 20 * n), "pack")
    got = d_dst.download()
    off = meta.download(8 * n + 8, 12 * n).view(np.uint64)
    exp = b"".join(src[int(o):int(o) + int(l)].tobytes() for o, l in zip(src_off, lens))
    assert int(off[n]) == total
    assert np.array_equal(off[:n], np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]))
    assert got[:3].tobytes() == b"\xab" * 3 and got[3 + total:3 + total + 8].tobytes() == b"\xab" * 8
    assert got[3:3 + total].tobytes() == exp


def test_host_pipeline(gpu, orc):
    """Pinned host -> device -> host pipeline (the host-inclusive path): packed
    frames identical to the reference's frame stream, round trip bit-exact."""
    from kingdb_amd.hostpipe import HostPipeline
    pool = oracle.g1_pool(orc)
    n, size = 3000, 4096
    vals = oracle.g1_values(pool, size, n - 2) + [bytes(size), bytes(np.random.default_rng(1).integers(0, 256, size, dtype=np.uint8))]
    hp = HostPipeline(n, size, chunk=512, nstreams=3)
    hp.h_raw.np[:] = np.frombuffer(b"".join(vals), np.uint8)
    hp.compress()
    cst, _ = hp.status()
    assert (cst == 0).all()
    assert hp.frames() == b"".join(orc.frame(v) for v in vals)
    hp.decompress()
    _, dst = hp.status()
    assert (dst == 0).all()
    assert np.array_equal(hp.h_out.np, hp.h_raw.np)
    hp.free()


def test_big_values_byu32(gpu, orc):
    """>= 65 547 B values (byU32 kernel + ring decoder), alone and mixed with
    small ones in the same launch (one launch per size class)."""
    from conftest import apply_recipe, big_value_inputs
    g = load_golden("big_values.npz")
    inputs = big_value_inputs(g, oracle.g1_pool(orc).tobytes())
    frames = gpu.compress_frames(inputs)
    blocks = gpu.compress_blocks(inputs)
    for name, x, f, (r, b), fl, fc, bl, bc in zip(g["names"], inputs, frames, blocks, g["frm_len"], g["frm_crc"],
                                                   g["blk_len"], g["blk_crc"]):
        assert len(f) == int(fl) and orc.crc32c(f) == int(fc), name
        assert r == int(bl) and orc.crc32c(b) == int(bc), name
    back = gpu.decompress_frames(frames, [len(x) for x in inputs])
    for name, (st, out), x in zip(g["names"], back, inputs):
        assert st == 0 and out == x, name
    dec = gpu.decompress_blocks([b for _, b in blocks], [len(x) for x in inputs])
    for name, (r, out), x in zip(g["names"], dec, inputs):
        assert r == len(x) and out == x, name
    # malformed 1 MiB blocks: exact return codes
    base = dict(zip([str(n) for n in g["names"]], [b for _, b in blocks]))["g1_1048576"]
    mal = [apply_recipe(base, int(k), int(p), int(v)) for k, p, v in g["mal_recipe"]]
    got = gpu.decompress_blocks(mal, [1 << 20] * len(mal))
    for (r, _), ret in zip(got, g["mal_ret"]):
        assert r == int(ret)
    # one mixed launch: 100 B .. 1 MiB
    pool = oracle.g1_pool(orc)
    mixed = []
    for i, x in enumerate(inputs):
        mixed += oracle.g1_values(pool, 100, 3) + [x] + oracle.g1_values(pool, 4096, 2) + [x[: 5000 + i]]
    mf = gpu.compress_frames(mixed)
    assert mf == [orc.frame(x) for x in mixed]
    mb = gpu.decompress_frames(mf, [len(x) for x in mixed])
    assert all(st == 0 and out == x for (st, out), x in zip(mb, mixed))


def test_byu32_tagged_table_edges(gpu, orc):
    """The tagged byU32 table (lz4_compress.hip Table32T, values <= 1 MiB): its empty
    entries stand for position 0, whose word may match later (a value whose only
    repeats are of its first 4 bytes); values just under and over the 1 MiB tag limit,
    matches just inside and outside the 64 KiB window, and a value repeated whole from
    past the window.  Frames equal the oracle's."""
    rng = np.random.default_rng(2024)
    vals = []
    for n in (65547, 100000, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, (1 << 20) + 70000):
        x = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        w0 = bytes(x[:4])
        for at in rng.integers(5, n - 8, 40):   # position 0's word, scattered
            x[int(at):int(at) + 4] = w0
        vals.append(bytes(x))
    # a repeat just inside / just outside the window (65 535 / 65 536 back)
    base = bytearray(rng.integers(0, 256, 200000, dtype=np.uint8).tobytes())
    for d in (65535, 65536, 65537):
        y = bytearray(base)
        y[150000:150032] = y[150000 - d:150000 - d + 32]
        vals.append(bytes(y))
    # a value repeated whole, 150 000 bytes back (past the window)
    z = bytearray(rng.integers(0, 256, 300000, dtype=np.uint8).tobytes())
    vals.append(bytes(z[:150000]) * 2)
    want = [orc.frame(v) for v in vals]
    frames = gpu.compress_frames(vals)
    assert frames == want
    back = gpu.decompress_frames(frames, [len(v) for v in vals])
    assert all(st == 0 and out == v for (st, out), v in zip(back, vals))
    # the same values of at most 1 MiB alone: a launch whose max_len is within the
    # tag limit takes the compact kernel (Table24T: 4-bit tags, position bits 16-19
    # in the byte plane, the 2 KiB ring)
    le = [i for i, v in enumerate(vals) if len(v) <= 1 << 20]
    assert gpu.compress_frames([vals[i] for i in le]) == [want[i] for i in le]


def test_compress_max_len_unbounded(gpu, orc):
    """max_len is a bound, not the exact largest length: 0xFFFFFFFF (a caller that
    does not know its lengths) gives the same frames for every size class.  Host
    code once took HIP's host min(), which is signed on uint32_t, and failed the
    4-8 KiB class's launch for bounds of 2^31 and more."""
    pool = oracle.g1_pool(orc)
    vals = (oracle.g1_values(pool, 100, 3) + oracle.g1_values(pool, 6000, 2) + oracle.g1_values(pool, 30000, 2)
            + oracle.g1_values(pool, 200000, 1))
    want = [orc.frame(v) for v in vals]
    for bound in (0xFFFFFFFF, 1 << 31, (1 << 20) + 1):
        assert gpu.compress_frames(vals, max_len=bound) == want, bound


def test_big_scalar_mirrors(gpu, orc):
    pool = oracle.g1_pool(orc).tobytes()
    x = pool[:300000]
    r, b = gpu.compress_limited_output(x, gpu.compress_bound(len(x)))
    assert b == orc.compress(x)
    r2, out = gpu.decompress_safe_partial(b, len(x), len(x))
    assert r2 == len(x) and out == x
