"""GPU: the write-buffer flush batch (include/kdb_flush.h, csrc/flush.hip,
SURVEY.md §8 row f3) against the per-call oracle.

Every PutPartValidSize call (/root/reference/interface/database.cc:128-276) of
a random stream -- several client threads interleaved, single-part values,
multipart values sent in parts of every size (64 KiB network parts, 1 MiB
Put splits, ragged ones), incompressible tails that fire the disable rule
mid-value, empty chunks, values whose first chunk is empty (the compressor's
running total then leaks from the thread's previous value), parts that
overrun the value's room (a stretch sent twice: IOError at :261-266) -- cut into batches at random
points, so values straddle batches and each thread's state is carried across
them.  oracle.put_part (lz4_oracle.c orc_put_part, itself pinned to the
reference's HSTable files by tests/test_write_path.py) runs the same calls one
by one: chunk_final, offset_chunk_compressed, size_value_compressed, crc32 and
the IOError verdict must match call for call.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _stream(orc, rng, nthreads, nvalues):
    pool = orc.g1_pieces(60000).tobytes()
    todo = []
    for t in range(nthreads):
        vals = []
        for j in range(nvalues):
            kind = rng.integers(0, 10)
            if kind < 5:
                n = int(rng.integers(0, 400))
            elif kind < 8:
                n = int(rng.integers(1000, 70000))
            else:
                n = int(rng.integers(65536, 300000))
            a = int(rng.integers(0, len(pool) - n))
            v = bytearray(pool[a:a + n])
            if n and rng.integers(0, 4) == 0:                       # incompressible tail
                b = int(rng.integers(0, n))
                v[b:] = rng.integers(0, 256, n - b, dtype=np.uint8).tobytes()
            v = bytes(v)
            key = b"t%d-v%d" % (t, j) + bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
            style = rng.integers(0, 6)
            if style == 0 or n == 0:
                chunks = [n]
            elif style == 1:
                chunks = [min(65536, n - o) for o in range(0, n, 65536)]
            elif style == 2:
                chunks = [min(1 << 20, n - o) for o in range(0, n, 1 << 20)]
            elif style == 3:
                cuts = sorted(set(int(x) for x in rng.integers(0, n + 1, int(rng.integers(1, 6)))))
                chunks = [b - a for a, b in zip([0] + cuts, cuts + [n])]
            elif style == 4:                                         # empty first chunk
                chunks = [0] + [min(50000, n - o) for o in range(0, n, 50000)]
            else:                                                    # a middle stretch sent twice
                h, q = n // 2, n // 4
                vals.append([(t, key, v[0:h], 0, n), (t, key, v[q:q + h], q, n), (t, key, v[h:], h, n)])
                continue
            calls, off = [], 0
            for c in chunks:
                calls.append((t, key, v[off:off + c], off, n))
                off += c
            vals.append(calls)
        todo.append([c for v in vals for c in v])
    # interleave the threads' call sequences at random, each thread in order
    out, idx = [], [0] * nthreads
    while any(idx[t] < len(todo[t]) for t in range(nthreads)):
        t = int(rng.integers(0, nthreads))
        if idx[t] < len(todo[t]):
            out.append(todo[t][idx[t]])
            idx[t] += 1
    return out


@pytest.mark.parametrize("seed,nthreads", [(1, 1), (2, 3), (3, 8)])
def test_flush_batches_match_per_call_oracle(gpu, orc, seed, nthreads):
    import oracle
    from kingdb_amd.flush import flush_parts
    rng = np.random.default_rng(seed)
    calls = _stream(orc, rng, nthreads, 40)
    # the oracle, call by call, each thread with its own ThreadStorage state
    ost = {}
    want = []
    for (tid, key, chunk, off, size) in calls:
        st = ost.setdefault(tid, oracle.PutState())
        want.append(oracle.put_part(orc, st, key, chunk, off, size))
    # the GPU, in random batches with the states carried
    states, got, i = {}, [], 0
    while i < len(calls):
        n = int(rng.integers(1, 60))
        res, states = flush_parts(calls[i:i + n], states)
        got += res
        i += n
    assert len(got) == len(want)
    for j, (g, w) in enumerate(zip(got, want)):
        if w["mode"] == 3:
            assert g["rc"] == -1 and g["mode"] == 3, j
            continue
        assert g["rc"] == w["rc"], (j, g["rc"], w["rc"])
        # a rejected call's order is never queued: its frame is not packed, the rest must match
        for f in ("mode", "occ", "svc", "crc") + (("chunk_final",) if w["rc"] == 0 else ()):
            assert g[f] == w[f], (j, f, calls[j][3], len(calls[j][2]), calls[j][4])
    for tid, st in ost.items():
        s = states[tid]
        assert (s.ts_offset, s.comp_total, s.enabled, s.crc) == (st.ts_offset, st.comp_total, st.enabled, st.crc)


def test_flush_single_part_values_one_batch(gpu, orc):
    """db_bench's shape (16 B keys / 100 B G1 values, one thread): one batch,
    every value a segment and a run of its own (the identity layout)."""
    import oracle
    from kingdb_amd.flush import flush_parts
    pool = orc.g1_pieces(5000).tobytes()
    calls = [(0, b"%016d" % i, pool[i * 37:i * 37 + 100], 0, 100) for i in range(4000)]
    res, states = flush_parts(calls)
    st = oracle.PutState()
    for c, r in zip(calls, res):
        w = oracle.put_part(orc, st, c[1], c[2], 0, 100)
        assert r == w
