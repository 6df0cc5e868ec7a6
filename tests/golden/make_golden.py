"""Generates the committed golden fixtures from the REFERENCE codec.

Run in the container that holds /root/reference (the GPU box does not):

    make -C oracle ref && python tests/golden/make_golden.py

Every expected output here comes from oracle/_ref/libkdbref.so, i.e. the
reference's own algorithm/lz4.cc + algorithm/compressor.cc compiled in place.
Inputs are synthetic (generators G1/G2/G3 of SURVEY.md §8d and edge patterns);
the reference holds no codec fixtures of its own.  Files are
numpy .npz (load with allow_pickle=False).
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def cat(chunks: list[bytes]) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    lens = np.array([len(c) for c in chunks], dtype=np.int64)
    off = np.zeros(len(chunks), dtype=np.int64)
    if len(chunks) > 1:
        off[1:] = np.cumsum(lens[:-1])
    data = np.frombuffer(b"".join(chunks), dtype=np.uint8) if chunks else np.zeros(0, np.uint8)
    return data.copy(), off, lens


def edge_inputs(ref: oracle.Reference, pool: np.ndarray) -> list[tuple[str, bytes]]:
    rng = random.Random(20141015)
    sizes = [0, 1, 2, 3, 4, 5, 8, 11, 12, 13, 14, 15, 16, 17, 19, 20, 24, 31, 32, 33, 63, 64, 65, 100,
             127, 128, 255, 256, 257, 270, 271, 510, 511, 1000, 1024, 4095, 4096, 4097, 8192,
             16384, 32768, 65535, 65536, 65546]
    g2 = ref.g2(65546, 1).tobytes()
    g3 = ref.g3(65546, 1).tobytes()
    out = []
    for n in sizes:
        out.append((f"zero{n}", bytes(n)))
        out.append((f"a{n}", b"a" * n))
        out.append((f"g1_{n}", pool[1234:1234 + n].tobytes()))
        out.append((f"g2_{n}", g2[:n]))
        out.append((f"g3_{n}", g3[:n]))
        per = rng.randrange(1, 40)
        base = bytes(rng.randrange(256) for _ in range(per))
        out.append((f"period{per}_{n}", (base * (n // per + 1))[:n]))
        out.append((f"ab{n}", bytes(rng.choice(b"ab") for _ in range(n))))
    # long runs to exercise the 255-continuation paths (lit >= 270, match >= 510)
    for n in (300, 600, 1200, 5000, 20000):
        out.append((f"litrun{n}", g3[:n] + b"z" * n + g3[n:2 * n]))
    # many hash collisions / periodic text
    for n in (3000, 9000):
        out.append((f"text{n}", ((b"the quick brown fox jumps over the lazy dog " * 400)[:n])))
    return out


def main() -> None:
    ref = oracle.Reference()
    orc = oracle.Oracle()
    pool = oracle.g1_pool(orc)
    assert orc.crc32c(pool.tobytes()) == 0x9E7B9EF6  # SURVEY KAT T2

    # ---- 1. block + frame KATs over edge inputs
    items = edge_inputs(ref, pool)
    names = [k for k, _ in items]
    inputs = [v for _, v in items]
    blocks = [ref.compress(v) for v in inputs]
    frames = [ref.frame(v) for v in inputs]
    assert all(b is not None for b in blocks)
    i_d, i_o, i_l = cat(inputs)
    b_d, b_o, b_l = cat(blocks)
    f_d, f_o, f_l = cat(frames)
    np.savez_compressed(os.path.join(OUT, "kat_blocks.npz"), names=np.array(names), inp=i_d, inp_off=i_o,
                        inp_len=i_l, blk=b_d, blk_off=b_o, blk_len=b_l, frm=f_d, frm_off=f_o, frm_len=f_l)

    # ---- 2. limitedOutput with caps below the bound (return value parity)
    rng = random.Random(7)
    lim_in, lim_cap, lim_ret, lim_blk = [], [], [], []
    for _ in range(600):
        n = rng.choice([rng.randrange(0, 200), rng.randrange(200, 3000)])
        kind = rng.randrange(3)
        if kind == 0:
            d = bytes(rng.choice(b"ab") for _ in range(n))
        elif kind == 1:
            d = pool[rng.randrange(0, 500000):][:n].tobytes()
        else:
            d = bytes(rng.randrange(256) for _ in range(n))
        bound = ref.compress_bound(n)
        cap = rng.choice([rng.randrange(0, bound + 1), max(0, bound - rng.randrange(0, 40)), n // 2, n])
        b = ref.compress(d, cap)
        lim_in.append(d)
        lim_cap.append(cap)
        lim_ret.append(0 if b is None else len(b))
        lim_blk.append(b or b"")
    i_d, i_o, i_l = cat(lim_in)
    b_d, b_o, b_l = cat(lim_blk)
    np.savez_compressed(os.path.join(OUT, "limited_output.npz"), inp=i_d, inp_off=i_o, inp_len=i_l,
                        cap=np.array(lim_cap, np.int64), ret=np.array(lim_ret, np.int64), blk=b_d,
                        blk_off=b_o)

    # ---- 3. malformed / truncated / random blocks: exact decode return codes
    rng = random.Random(99)
    m_blk, m_size, m_tgt, m_ret, m_out, m_cmp = [], [], [], [], [], []
    for it in range(4000):
        n = rng.randrange(0, 600)
        if rng.random() < 0.6:
            d = bytes(rng.choice(b"abc") for _ in range(n)) if rng.random() < 0.5 else pool[it * 37:it * 37 + n].tobytes()
            blk = bytearray(ref.compress(d))
            for _ in range(rng.randrange(1, 4)):
                if not blk:
                    break
                op = rng.randrange(4)
                if op == 0:
                    blk[rng.randrange(len(blk))] = rng.randrange(256)
                elif op == 1:
                    blk = blk[: rng.randrange(len(blk) + 1)]
                elif op == 2:
                    blk.insert(rng.randrange(len(blk) + 1), rng.randrange(256))
                else:
                    blk[rng.randrange(len(blk))] ^= 1 << rng.randrange(8)
            blk = bytes(blk)
        else:
            blk = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 48)))
        size = rng.choice([n, n, rng.randrange(0, 700), 0, 1, 12, 13, 17])
        tgt = size if rng.random() < 0.8 else rng.randrange(-2, size + 30)
        r, out = ref_decode(ref, blk, size, tgt)
        ro, oo = orc_decode(orc, blk, size, tgt)
        _, oo_ff = orc_decode(orc, blk, size, tgt, fill=0xFF)
        assert ro == r, (blk.hex(), size, tgt, ro, r)
        m_blk.append(blk)
        m_size.append(size)
        m_tgt.append(tgt)
        m_ret.append(r)
        m_out.append(out)
        # output bytes are specified unless the block used offset 0 (the
        # reference then copies destination bytes it never wrote, so the
        # result depends on the buffer's prior contents): detected by decoding
        # into a 0x00- and a 0xFF-filled buffer.
        m_cmp.append(1 if (r <= 0 or (oo == out and oo == oo_ff)) else 0)
    b_d, b_o, b_l = cat(m_blk)
    o_d, o_o, o_l = cat(m_out)
    np.savez_compressed(os.path.join(OUT, "malformed.npz"), blk=b_d, blk_off=b_o, blk_len=b_l,
                        size=np.array(m_size, np.int64), target=np.array(m_tgt, np.int64),
                        ret=np.array(m_ret, np.int64), out=o_d, out_off=o_o, cmp=np.array(m_cmp, np.int8))
    print("malformed: decodes", len(m_ret), "errors", sum(1 for r in m_ret if r < 0),
          "unspecified-output", m_cmp.count(0))

    # ---- 4. G1 (db_bench) values at 100 B / 4 KiB / 64 KiB: sizes + digests
    g1 = {}
    for size, count, keep in ((100, 1000, 1000), (4096, 1000, 64), (65536, 16, 2)):
        vals = oracle.g1_values(pool, size, count)
        blks = [ref.compress(v) for v in vals]
        frms = [ref.frame(v) for v in vals]
        g1[f"s{size}_blk_len"] = np.array([len(b) for b in blks], np.int64)
        g1[f"s{size}_frm_len"] = np.array([len(f) for f in frms], np.int64)
        g1[f"s{size}_blk_crc"] = np.array([ref.crc32c(b"".join(blks))], np.int64)
        g1[f"s{size}_frm_crc"] = np.array([ref.crc32c(b"".join(frms))], np.int64)
        g1[f"s{size}_blk_keep"] = np.frombuffer(b"".join(blks[:keep]), np.uint8).copy()
    np.savez_compressed(os.path.join(OUT, "g1_db_bench.npz"), **g1)

    # ---- 5. G2 / G3 (test_db generators) frames at 100 B and 4 KiB
    g = {}
    for name, gen in (("g2", ref.g2), ("g3", ref.g3)):
        for size, count in ((100, 500), (4096, 64)):
            data = gen(size, count)
            frms = [ref.frame(data[i * size:(i + 1) * size].tobytes()) for i in range(count)]
            f_d, f_o, f_l = cat(frms)
            g[f"{name}_{size}_inp"] = data
            g[f"{name}_{size}_frm"] = f_d
            g[f"{name}_{size}_frm_len"] = f_l
    np.savez_compressed(os.path.join(OUT, "test_db_generators.npz"), **g)

    # ---- 6. unit-tests/test_compression.cc (KAT T1): 442 837 B of the key
    #         "0x10c095000-0" repeated, compressed in 64 KiB chunks.
    key = b"0x10c095000-0"
    value = (key * (442837 // len(key) + 1))[:442837]
    chunks = [value[i:i + 65536] for i in range(0, len(value), 65536)]
    frms = [ref.frame(c) for c in chunks]
    stream = b"".join(frms)
    nfr, back = ref.frames_uncompress(stream, len(value))
    assert nfr == 7 and back == value and len(stream) == 1947
    np.savez_compressed(os.path.join(OUT, "test_compression.npz"),
                        frames=np.frombuffer(stream, np.uint8).copy(),
                        frame_len=np.array([len(f) for f in frms], np.int64))
    # ---- 7. values past the byU16 range (byU32 encoder, ring decoder):
    #         KingDB's default part size is 1 MB (util/options.h:171).
    big = big_inputs(ref, pool)
    b_names = [k for k, _ in big]
    b_frames = [ref.frame(v) for _, v in big]
    b_blocks = [ref.compress(v) for _, v in big]
    keep_inp = {k: np.frombuffer(v, np.uint8).copy() for k, v in big if not k.startswith(("g1_", "a_"))}
    arrs = {f"inp_{k}": v for k, v in keep_inp.items()}
    arrs["names"] = np.array(b_names)
    arrs["sizes"] = np.array([len(v) for _, v in big], np.int64)
    arrs["frm_len"] = np.array([len(f) for f in b_frames], np.int64)
    arrs["frm_crc"] = np.array([ref.crc32c(f) for f in b_frames], np.int64)
    arrs["blk_len"] = np.array([len(b) for b in b_blocks], np.int64)
    arrs["blk_crc"] = np.array([ref.crc32c(b) for b in b_blocks], np.int64)
    # malformed big blocks: truncations / byte edits of the 1 MiB G1 block,
    # kept as recipes (kind, position, value) applied by the test to the block
    # the GPU produced (itself pinned by length + crc above)
    rng = random.Random(5)
    base_blk = b_blocks[b_names.index("g1_1048576")]
    recipes, m_ret = [], []
    for it in range(12):
        kind = it % 3
        pos = rng.randrange(1, len(base_blk)) if kind == 0 else rng.randrange(len(base_blk))
        val = rng.randrange(8) if kind == 1 else 0xFF
        blk = apply_recipe(base_blk, kind, pos, val)
        r, _ = ref_decode(ref, blk, 1 << 20, 1 << 20)
        recipes.append((kind, pos, val))
        m_ret.append(r)
    arrs["mal_recipe"] = np.array(recipes, np.int64)
    arrs["mal_ret"] = np.array(m_ret, np.int64)
    np.savez_compressed(os.path.join(OUT, "big_values.npz"), **arrs)
    print("big values:", list(zip(b_names, arrs["frm_len"].tolist())), "malformed rets", m_ret)
    print("fixtures written to", OUT)


def apply_recipe(blk: bytes, kind: int, pos: int, val: int) -> bytes:
    """kind 0: truncate to pos bytes; 1: flip bit val at pos; 2: set pos to val."""
    b = bytearray(blk)
    if kind == 0:
        return bytes(b[:pos])
    if kind == 1:
        b[pos] ^= 1 << val
    else:
        b[pos] = val
    return bytes(b)


def big_inputs(ref: oracle.Reference, pool: np.ndarray) -> list[tuple[str, bytes]]:
    """Inputs >= 65 547 bytes.  g1_* and a_* are regenerated by the tests
    (G1 pool slices, 'a' runs); the others are stored in the fixture."""
    g1 = pool.tobytes()
    g2 = ref.g2(300000, 1).tobytes()
    g3 = ref.g3(200000, 1).tobytes()
    text = (b"the quick brown fox jumps over the lazy dog 0123456789 " * 10000)[:500000]
    return [
        ("g1_65547", g1[:65547]),
        ("g1_100000", g1[7:100007]),
        ("g1_262144", g1[:262144]),
        ("g1_1048576", g1[:1048576]),
        ("a_1048576", b"a" * 1048576),
        ("g2_300000", g2),
        ("g3_200000", g3),
        ("text_500000", text),
    ]


def ref_decode(ref: oracle.Reference, blk: bytes, size: int, tgt: int):
    src = np.zeros(len(blk) + 64, np.uint8)
    src[: len(blk)] = np.frombuffer(blk, np.uint8)
    dst = np.zeros(max(size, 0) + 64, np.uint8)
    r = ref.lib.ref_decompress_partial(oracle._ptr(src), len(blk), oracle._ptr(dst), tgt, size)
    return r, (dst[:r].tobytes() if r > 0 else b"")


def orc_decode(orc: oracle.Oracle, blk: bytes, size: int, tgt: int, fill: int = 0):
    src = np.zeros(len(blk) + 64, np.uint8)
    src[: len(blk)] = np.frombuffer(blk, np.uint8)
    dst = np.full(max(size, 0) + 64, fill, np.uint8)
    r = orc.lib.orc_decompress_safe_partial(oracle._ptr(src), oracle._ptr(dst), len(blk), tgt, size)
    return r, (dst[:r].tobytes() if r > 0 else b"")


if __name__ == "__main__":
    main()
