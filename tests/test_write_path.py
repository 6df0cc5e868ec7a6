"""The write path around the codec.

Pinned by tests/golden/hstable_streams.npz: put streams and the HSTable files
the reference's own Database -> WriteBuffer -> HSTableManager wrote for them
(tests/golden/make_golden_put.py, oracle/_ref/ref_db).

CPU: the oracle restatement (oracle/hstable.py + lz4_oracle.c orc_put_value)
reproduces every reference file byte for byte; the product's host-side HSTable
writer (csrc/hstable.cc) does too when fed the oracle's entries; the key hashes
and CRC-8 match independent implementations.
GPU: kdb_put_entries_batch (csrc/put.hip) produces the oracle's entry bytes,
key hashes and CRC32Cs, and the GPU path end to end writes the reference's files.
"""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_golden_put import decode_stream  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "hstable_streams.npz")


def golden():
    z = np.load(GOLD)
    out = {}
    for name in z["names"]:
        name = str(name)
        hs, ht, mps = (int(x) for x in z[f"{name}__opts"])
        files = {str(f): z[f"{name}__file_{f}"].tobytes() for f in z[f"{name}__files"]}
        out[name] = (decode_stream(z[f"{name}__stream"].tobytes()), hs, ht, files)
    return out


GOLDEN = golden()


def oracle_writer(orc, puts, hs, ht, batch=None):
    from oracle import hstable
    w = hstable.Writer(orc, hs, ht)
    step = batch or max(len(puts), 1)
    for i in range(0, len(puts), step):
        for k, v, ch in puts[i:i + step]:
            w.put(k, v, ch)
        w._flush(0, 0)          # end of a write-buffer flush (WriteOrdersAndFlushFile's last line)
    files = w.close()
    return w, files


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_oracle_per_call_matches_reference_hstables(orc, name):
    """orc_put_part (one PutPartValidSize call over carried thread state, the
    checker of the flush hook's batch) writes the reference's files too."""
    import oracle
    from oracle import hstable
    puts, hs, ht, files = GOLDEN[name]
    w = hstable.Writer(orc, hs, ht)
    st = oracle.PutState()
    for k, v, ch in puts:
        w.put_calls(st, k, v, ch)
    w._flush(0, 0)
    got = w.close()
    assert got == files


def test_oracle_per_call_matches_put_value(orc):
    """Random values and chunkings (incompressible tails disable compression mid-value):
    orc_put_part call by call equals orc_put_value for the whole value."""
    import oracle
    rng = np.random.default_rng(11)
    pool = orc.g1_pieces(30000).tobytes()
    st = oracle.PutState()
    for t in range(300):
        n = int(rng.integers(0, 200000))
        a = int(rng.integers(0, len(pool) - n)) if n < len(pool) else 0
        v = bytearray(pool[a:a + n])
        if n and t % 3 == 0:                      # an incompressible stretch
            b = int(rng.integers(0, n))
            v[b:] = rng.integers(0, 256, n - b, dtype=np.uint8).tobytes()
        v = bytes(v)
        cuts = sorted(set(int(x) for x in rng.integers(0, n + 1, int(rng.integers(0, 6))))) if n else []
        ch = [b - a for a, b in zip([0] + cuts, cuts + [n])] if n else [0]
        want = orc.put_value(b"k%d" % t, v, ch)
        off = 0
        for i, c in enumerate(ch):
            r = oracle.put_part(orc, st, b"k%d" % t, v[off:off + c], off, n)
            assert r["rc"] == 0
            assert (r["occ"], r["chunk_final"]) == want["parts"][i]
            last = i == len(ch) - 1
            assert r["svc"] == (want["svc"] if last and c else 0) or not last
            off += c
        if ch and ch[-1]:
            assert r["svc"] == want["svc"]
        assert r["crc"] == want["crc"]


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_oracle_matches_reference_hstables(orc, name):
    puts, hs, ht, files = GOLDEN[name]
    _, got = oracle_writer(orc, puts, hs, ht)
    assert list(got) == list(files)
    for f in files:
        assert got[f] == files[f], f


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_host_hstable_writer_matches_reference(orc, name):
    """csrc/hstable.cc (product, host side) fed the oracle's entries."""
    from kingdb_amd.put import HSTableWriter, PutBatchResult
    puts, hs, ht, files = GOLDEN[name]
    w, _ = oracle_writer(orc, puts, hs, ht)
    dense = w.dense()
    lens = np.array([len(e) for e, _, _ in dense], np.uint32)
    off = np.zeros(len(dense), np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    r = PutBatchResult(entries=np.frombuffer(b"".join(e for e, _, _ in dense), np.uint8).copy(), entry_off=off,
                       entry_len=lens, hashed=np.array([h for _, h, _ in dense], np.uint64),
                       crc=np.zeros(len(dense), np.uint32), kind=np.array([k for _, _, k in dense], np.uint32),
                       status=np.zeros(len(dense), np.int32))
    hw = HSTableWriter(hs, ht)
    hw.append(r)
    hw.close()
    got = hw.files()
    assert list(got) == list(files)
    for f in files:
        assert got[f] == files[f], f


@pytest.mark.parametrize("hs,batch", [(96 << 10, 6000), (32 << 20, 20000), (1 << 20, 4096)])
def test_host_hstable_writer_parallel_batches(orc, hs, batch):
    """Batches of >= 4096 plain entries take the writer's parallel path (file
    cuts by binary search over the dense offsets, rows encoded by the worker
    pool); the files must equal the oracle's for the same write-buffer flushes,
    with files cut inside and across batches.  A batch with a failed put falls
    back to the entry-by-entry path."""
    import oracle
    from oracle import hstable
    from kingdb_amd.put import HSTableWriter, PutBatchResult
    n = 20000
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, 100, n)
    puts = [(b"%016d" % i, v, None) for i, v in enumerate(vals)]
    w = hstable.Writer(orc, hs, 1)
    for lo in range(0, n, batch):
        for k, v, ch in puts[lo:lo + batch]:
            w.put(k, v, ch)
        w._flush(0, 0)
    files = w.close()
    dense = w.dense()
    assert len(dense) == n
    hw = HSTableWriter(hs, 1)
    for lo in range(0, n, batch):
        d = dense[lo:lo + batch]
        lens = np.array([len(e) for e, _, _ in d], np.uint32)
        off = np.zeros(len(d), np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        st = np.zeros(len(d), np.int32)
        ents = b"".join(e for e, _, _ in d)
        if lo == 0 and batch == 4096:
            # a failed put (IOError: no order, no bytes in the stream) -> the serial path
            st = np.append(st, -1).astype(np.int32)
            lens = np.append(lens, 0).astype(np.uint32)
            off = np.append(off, off[-1] + lens[-2]).astype(np.uint64)
        hashes = [h for _, h, _ in d] + ([0] * (len(st) - len(d)))
        kinds = [k for _, _, k in d] + ([0] * (len(st) - len(d)))
        r = PutBatchResult(entries=np.frombuffer(ents, np.uint8).copy(), entry_off=off, entry_len=lens,
                           hashed=np.array(hashes, np.uint64), crc=np.zeros(len(st), np.uint32),
                           kind=np.array(kinds, np.uint32), status=st)
        hw.append(r)
    hw.close()
    got = hw.files()
    assert list(got) == list(files)
    for f in files:
        assert got[f] == files[f], f


def test_db_options_bytes(orc):
    from kingdb_amd.put import db_options
    from oracle import hstable
    for hs, ht in ((32 << 20, 1), (64 << 10, 0)):
        assert db_options(hs, ht) == hstable.db_options_bytes(orc, hs, ht)


def test_key_hashes_and_crc8(orc):
    import xxhash
    rng = np.random.default_rng(2)
    for n in list(range(0, 70)) + [255, 1000]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert orc.xxh64(d) == xxhash.xxh64_intdigest(d)
    # MurmurHash3_x64_128 published vectors (seed 0): first 64-bit word
    assert orc.murmur3_64(b"") == 0
    assert orc.murmur3_64(b"hello") == 0xCBD8A7B341BD9B02
    # crc8 table of crc32c.cc:439-461: entries 1, 2, 128, 255
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0xB2 if c & 1 else c >> 1
        t.append(c)
    assert (t[1], t[2], t[128], t[255]) == (0x3E, 0x7C, 0xB2, 0x15)
    for b in range(256):
        assert orc.crc8(bytes([b])) == t[0xFF ^ b] ^ 0xFF


def test_policy_disable_cases(orc):
    """database.cc:196-209: raw-fallback frames are always disabled for one-part
    values; a frame with C + 8 > size is disabled; C + 8 <= size stays."""
    inc = bytes(np.random.default_rng(1).integers(0, 256, 1000, dtype=np.uint8))
    pv = orc.put_value(b"k", inc)
    assert pv["parts"][0][1][:8] == bytes(8) and pv["parts"][0][1][8:] == inc and pv["svc"] == 1008
    pv = orc.put_value(b"k", b"a" * 1000)
    assert pv["parts"][0][1][:4] != bytes(4) and pv["svc"] == len(pv["parts"][0][1])
    pv = orc.put_value(b"k", b"")
    assert pv["parts"] == [(0, b"")] and pv["svc"] == 0 and pv["crc"] == orc.crc32c(b"k")


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_gpu_put_entries_match_oracle(gpu, orc, name):
    from kingdb_amd.put import put_entries
    puts, hs, ht, files = GOLDEN[name]
    w, _ = oracle_writer(orc, puts, hs, ht)
    dense = w.dense()
    r = put_entries(puts, ht)
    assert (r.status == 0).all()
    assert len(dense) == len(puts)
    for i, (e, h, k) in enumerate(dense):
        assert int(r.hashed[i]) == h, i
        assert int(r.kind[i]) == k, i
        assert r.entry(i) == e, i
        k_, v, ch = puts[i]
        assert int(r.crc[i]) == orc.put_value(k_, v, ch)["crc"], i


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_gpu_write_path_matches_reference_files(gpu, name):
    from kingdb_amd.put import write_hstables
    puts, hs, ht, files = GOLDEN[name]
    got = write_hstables(puts, hs, ht)
    assert list(got) == list(files)
    for f in files:
        assert got[f] == files[f], f


@pytest.mark.gpu
def test_gpu_write_path_batches_match_oracle(gpu, orc):
    """Several write-buffer flushes: the same files as the oracle with the same batches."""
    from kingdb_amd.put import write_hstables
    puts, hs, ht, _ = GOLDEN["rollover"]
    for batch in (1, 7, 64):
        _, exp = oracle_writer(orc, puts, hs, ht, batch)
        assert write_hstables(puts, hs, ht, batch) == exp, batch


@pytest.mark.gpu
def test_gpu_crc_and_hash_random(gpu, orc):
    """CRC32C over key || value (64-lane chunked, GF(2) tree) and both key hashes
    on random keys/values of every small length and a few large ones."""
    import xxhash
    from kingdb_amd.put import put_entries
    rng = np.random.default_rng(9)
    puts = []
    for i in range(400):
        kl = int(rng.integers(1, 90))
        vl = int(rng.choice([0, 1, 3, 7, 59, 60, 61, 200, 5000, 70000]))
        puts.append((rng.integers(0, 256, kl, dtype=np.uint8).tobytes(),
                     rng.integers(0, 4, vl, dtype=np.uint8).tobytes()))
    for ht in (1, 0):
        r = put_entries(puts, ht)
        for i, (k, v) in enumerate(puts):
            pv = orc.put_value(k, v)
            assert int(r.crc[i]) == pv["crc"], i
            assert int(r.hashed[i]) == (xxhash.xxh64_intdigest(k) if ht else orc.murmur3_64(k)), i


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [True, False])
def test_gpu_put_pipeline_matches_oracle(gpu, orc, direct):
    """The bench's pipeline (kingdb_amd/putpipe.py: chunks over 4 streams, entry
    bytes DMA'd from HBM straight into pinned file buffers when direct) writes
    the oracle's files; small HSTables so files roll over inside and across
    chunks, and twice through one writer (reset + buffer reuse)."""
    import oracle
    from oracle import hstable
    from kingdb_amd.putpipe import PutPipeline
    n, ks, vs, hs = 6000, 16, 100, 96 << 10
    pool = oracle.g1_pool(orc)
    vals = oracle.g1_values(pool, vs, n)
    keys = [b"%016d" % i for i in range(n)]
    w = hstable.Writer(orc, hs, 1)
    chunk = 1024
    for lo in range(0, n, chunk):                 # one write-buffer flush per pipeline chunk
        for k, v in zip(keys[lo:lo + chunk], vals[lo:lo + chunk]):
            w.put(k, v, None)
        w._flush(0, 0)
    exp = w.close()
    pp = PutPipeline(n, ks, vs, chunk=chunk, nstreams=4, hstable_size=hs, hash_type=1, direct=direct)
    try:
        pp.h_keys.np[:] = np.frombuffer(b"".join(keys), np.uint8)
        pp.h_vals.np[:] = np.frombuffer(b"".join(vals), np.uint8)
        for _ in range(2):
            pp.run()
            got = pp.writer.files()
            assert list(got) == list(exp)
            for f in exp:
                assert got[f] == exp[f], f
    finally:
        pp.free()
