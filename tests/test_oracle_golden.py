"""CPU: the oracle (plain-C restatement) against the reference-generated goldens.

Pins the oracle: every expected byte here came from the reference's own
algorithm/lz4.cc + compressor.cc (tests/golden/make_golden.py)."""
import os

import numpy as np

import oracle
from conftest import GOLDEN, load_golden, split


def test_kat_blocks_and_frames(orc):
    g = load_golden("kat_blocks.npz")
    inputs = split(g["inp"], g["inp_off"], g["inp_len"])
    blocks = split(g["blk"], g["blk_off"], g["blk_len"])
    frames = split(g["frm"], g["frm_off"], g["frm_len"])
    for name, x, b, f in zip(g["names"], inputs, blocks, frames):
        assert orc.compress(x) == b, name
        assert orc.frame(x) == f, name
        r, out = orc.decompress(b, len(x))
        assert r == len(x) and out == x, name


def test_limited_output_return_values(orc):
    g = load_golden("limited_output.npz")
    inputs = split(g["inp"], g["inp_off"], g["inp_len"])
    for x, cap, ret, off in zip(inputs, g["cap"], g["ret"], g["blk_off"]):
        b = orc.compress(x, int(cap))
        assert (0 if b is None else len(b)) == int(ret)
        if ret:
            assert b == g["blk"][int(off):int(off) + int(ret)].tobytes()


def test_malformed_decode_codes(orc):
    g = load_golden("malformed.npz")
    blocks = split(g["blk"], g["blk_off"], g["blk_len"])
    src_pad = 64
    for i, b in enumerate(blocks):
        size, tgt, ret = int(g["size"][i]), int(g["target"][i]), int(g["ret"][i])
        src = np.zeros(len(b) + src_pad, np.uint8)
        src[: len(b)] = np.frombuffer(b, np.uint8)
        dst = np.zeros(max(size, 0) + 64, np.uint8)
        r = orc.lib.orc_decompress_safe_partial(oracle._ptr(src), oracle._ptr(dst), len(b), tgt, size)
        assert r == ret, i
        if r > 0 and g["cmp"][i]:
            o = int(g["out_off"][i])
            assert dst[:r].tobytes() == g["out"][o:o + r].tobytes(), i


def test_g1_db_bench_digests(orc):
    """SURVEY KATs T2-T5 (db_bench G1 values at 100 B / 4 KiB / 64 KiB)."""
    g = load_golden("g1_db_bench.npz")
    pool = oracle.g1_pool(orc)
    assert orc.crc32c(pool.tobytes()) == 0x9E7B9EF6
    for size, count in ((100, 1000), (4096, 1000), (65536, 16)):
        vals = oracle.g1_values(pool, size, count)
        blks = [orc.compress(v) for v in vals]
        assert [len(b) for b in blks] == list(g[f"s{size}_blk_len"])
        assert orc.crc32c(b"".join(blks)) == int(g[f"s{size}_blk_crc"][0])
    assert list(g["s4096_blk_len"][:5]) == [2261, 2263, 2269, 2272, 2277]
    assert int(g["s4096_blk_len"].sum()) == 2279907


def test_test_db_generator_frames(orc):
    g = load_golden("test_db_generators.npz")
    for name in ("g2", "g3"):
        for size in (100, 4096):
            data = g[f"{name}_{size}_inp"]
            lens = g[f"{name}_{size}_frm_len"]
            off = np.concatenate([[0], np.cumsum(lens)[:-1]])
            frames = split(g[f"{name}_{size}_frm"], off, lens)
            for i, f in enumerate(frames):
                assert orc.frame(data[i * size:(i + 1) * size].tobytes()) == f


def test_test_compression_kat(orc):
    """unit-tests/test_compression.cc: 7 frames, 287 x 6 + 225 = 1947 bytes (KAT T1)."""
    g = load_golden("test_compression.npz")
    key = b"0x10c095000-0"
    value = (key * (442837 // len(key) + 1))[:442837]
    frames = b"".join(orc.frame(value[i:i + 65536]) for i in range(0, len(value), 65536))
    assert frames == g["frames"].tobytes()
    assert list(g["frame_len"]) == [287] * 6 + [225]


def test_g1_generator_jump_ahead_matches_sequential(orc):
    """The piece-parallel G1 generator (datagen.hip) relies on jump-ahead; check
    the algebra on the CPU: piece j == sequential stream at draw 50 j."""
    M, A = 2147483647, 16807
    seq = orc.g1_pieces(40)
    for j in (0, 1, 7, 39):
        s = 301 * pow(A, 50 * j, M) % M
        raw = []
        for _ in range(50):
            s = s * A % M
            raw.append(32 + s % 95)
        assert bytes(raw * 2) == seq[j * 100:(j + 1) * 100].tobytes()


def test_big_values_byu32(orc):
    """Values past the byU16 range (>= 65 547 B: byU32 encoder) and the
    malformed-block codes on a 1 MiB block, against the reference's digests."""
    from conftest import apply_recipe, big_value_inputs
    g = load_golden("big_values.npz")
    inputs = big_value_inputs(g, oracle.g1_pool(orc).tobytes())
    blocks = {}
    for name, x, fl, fc, bl, bc in zip(g["names"], inputs, g["frm_len"], g["frm_crc"], g["blk_len"], g["blk_crc"]):
        f = orc.frame(x)
        b = orc.compress(x)
        assert len(f) == int(fl) and orc.crc32c(f) == int(fc), name
        assert len(b) == int(bl) and orc.crc32c(b) == int(bc), name
        r, out = orc.decompress(b, len(x))
        assert r == len(x) and out == x, name
        blocks[str(name)] = b
    base = blocks["g1_1048576"]
    for (kind, pos, val), ret in zip(g["mal_recipe"], g["mal_ret"]):
        r, _ = orc.decompress(apply_recipe(base, int(kind), int(pos), int(val)), 1 << 20)
        assert r == int(ret), (kind, pos, val)


def test_oracle_matches_reference_digests_prefix(orc):
    """tests/golden/digests.json (the reference's frames at BASELINE size,
    make_digests.py): the oracle's frames of each batch's first 65 536 values
    have the same byte count and CRC32C."""
    import json
    from kingdb_amd.lz4 import mixed_sizes
    d = json.load(open(os.path.join(GOLDEN, "digests.json")))
    for name, sizes in (("g1_long_4k", np.full(1 << 20, 4096, np.uint32)), ("mixed_1m", mixed_sizes(1 << 20))):
        g = d[name]
        assert g["n"] == len(sizes) and g["raw_bytes"] == int(sizes.astype(np.int64).sum())
        k = g["prefix_n"]
        lens = sizes[:k]
        off = np.zeros(k, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        src = orc.g1_pieces((int(lens.astype(np.int64).sum()) + 99) // 100)
        tot, crc = orc.frames_digest(src, off, lens)
        assert (tot, f"0x{crc:08x}") == (g["prefix_frame_bytes"], g["prefix_frames_crc32c"]), name
