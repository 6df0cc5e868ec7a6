"""The read path around the codec (read side):
CompressorLZ4::UncompressByteArray over stored values.

Pinned by tests/golden/get_values.npz (make_golden_get.py): the value regions
of the reference's own HSTable files plus mutated copies, with the status and
output of the reference's UncompressByteArray, with and without checksum
verification.  "undefined" rows are those where the reference would read or
write outside the value: only an error is required there.

CPU: the oracle restatement (orc_get_value) matches the reference on every
defined row.  GPU: kdb_get_values_batch (csrc/get.hip) matches it on every
row, and write path -> HSTable files -> read path returns every value.
"""
import os

import numpy as np
import pytest

from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden", "get_values.npz")
UNDEF = 99
# reference status (0 OK, 1 "Invalid checksum.", 2 other IOError) -> ours
MAP = {0: 0, 1: -2, 2: -1}


def golden():
    z = np.load(GOLD)
    lens = z["stored_len"].astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens)])
    st = z["stored"]
    items = [(st[off[i]:off[i + 1]].tobytes(), int(z["svc"][i]), int(z["size"][i]), int(z["checksum"][i]),
              int(z["checksum_initial"][i])) for i in range(len(lens))]
    exp = {v: (z[f"status_v{v}"], z[f"out_crc_v{v}"], z[f"out_len_v{v}"]) for v in (0, 1)}
    return items, exp


ITEMS, EXP = golden()


@pytest.mark.parametrize("verify", [0, 1])
def test_oracle_get_matches_reference(orc, verify):
    sts, crcs, lens = EXP[verify]
    n_def = 0
    for i, it in enumerate(ITEMS):
        st, out = orc.get_value(*it, verify=verify)
        if sts[i] == UNDEF:
            assert st != 0, i
            continue
        n_def += 1
        assert st == MAP[int(sts[i])], i
        if st == 0:
            assert len(out) == lens[i] and orc.crc32c(out) == crcs[i], i
    assert n_def > 1500


def test_reference_double_stream_bug_is_in_the_fixture():
    """with verification the reference rejects values stored as frames."""
    sts = EXP[1][0]
    assert (sts == 1).sum() > 1000


def test_oracle_corrected_verify_accepts_good_values(orc):
    bad = 0
    for i, it in enumerate(ITEMS[:1652]):      # the unmutated reference entries
        st, _ = orc.get_value(*it, verify=2)
        bad += st != 0
    assert bad == 0


@pytest.mark.gpu
@pytest.mark.parametrize("verify", [0, 1])
def test_gpu_get_matches_reference(gpu, orc, verify):
    from kingdb_amd.get import get_values
    sts, crcs, lens = EXP[verify]
    res = get_values(ITEMS, verify)
    for i, (st, out) in enumerate(res):
        if sts[i] == UNDEF:
            assert st != 0, i
            continue
        assert st == MAP[int(sts[i])], (i, st, int(sts[i]))
        if st == 0:
            assert len(out) == lens[i] and orc.crc32c(out) == crcs[i], i


@pytest.mark.gpu
def test_gpu_get_corrected_verify(gpu, orc):
    from kingdb_amd.get import get_values
    res = get_values(ITEMS, 2)
    for i, (st, out) in enumerate(res):
        ost, oout = orc.get_value(*ITEMS[i], verify=2)
        if ost == -3:
            assert st != 0, i
        else:
            assert st == ost, i
            if st == 0:
                assert out == oout, i


@pytest.mark.gpu
def test_gpu_write_then_read_round_trip(gpu, orc):
    """Write path -> the reference's HSTable format -> read path: every value back,
    and the corrected checksum verifies (kind 2 entries excepted: svc 0 there)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden_put import decode_stream
    from kingdb_amd.get import entry_items, get_values, read_hstable
    from kingdb_amd.put import write_hstables
    z = np.load(os.path.join(ROOT, "tests", "golden", "hstable_streams.npz"))
    for name in ("small", "edge", "rollover", "murmur"):
        puts = decode_stream(z[f"{name}__stream"].tobytes())
        hs, ht, _ = (int(x) for x in z[f"{name}__opts"])
        files = write_hstables(puts, hs, ht)
        items = []
        for f in files.values():
            items += entry_items(f, read_hstable(f), orc.crc32c)
        assert len(items) == len(puts)
        for (st, out), (k, v, _) in zip(get_values(items, 2), puts):
            assert st == 0 and out == v, name
