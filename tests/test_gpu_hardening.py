"""GPU: caller streams, capacity limits and undefined bytes.

* get_values / put_entries with an explicit (non-blocking) Stream return the
  same results as without one (the copies back ride the caller's stream).
* a stored value whose frames do not fit the launch's frame capacity reports
  KDB_LZ4_VALUE_UNSUPPORTED (the bytes may be fine), not IOError.
* a match with offset 0 (lz4.cc:959-960 lets ref == op through; the reference
  then copies bytes it never wrote, undefined) decodes to zeros -- never to
  bytes another value left in the decoder's LDS window.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

UNSUPPORTED = -(1 << 31)


def _stored(orc, key, value, chunks):
    pv = orc.put_value(key, value, chunks)
    return pv["stored"], pv["svc"], len(value)


def test_get_values_explicit_stream(gpu, orc):
    from kingdb_amd.get import get_values
    from kingdb_amd.lz4 import Stream
    pool = orc.g1_pieces(4000).tobytes()
    items = [_stored(orc, b"k%d" % i, pool[i * 97:i * 97 + 100 + 37 * i], None) for i in range(64)]
    a = get_values(items, 0)
    st = Stream()
    b = get_values(items, 0, stream=st)
    assert a == b
    assert all(s == 0 for s, _ in a)
    assert [o for _, o in a] == [pool[i * 97:i * 97 + 100 + 37 * i] for i in range(64)]


def test_put_entries_explicit_stream(gpu):
    from kingdb_amd.lz4 import Stream
    from kingdb_amd.put import put_entries
    rng = np.random.default_rng(5)
    puts = [(b"%016d" % i, bytes(rng.integers(97, 100, 100 + 13 * i, dtype=np.uint8))) for i in range(200)]
    a = put_entries(puts)
    b = put_entries(puts, stream=Stream())
    assert a.entries.tobytes() == b.entries.tobytes()
    for f in ("entry_off", "entry_len", "hashed", "crc", "kind", "status"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_get_frame_capacity_unsupported(gpu, orc):
    from kingdb_amd.get import get_values
    pool = orc.g1_pieces(10000).tobytes()
    val = pool[:5 * 65536 - 1000]                       # 5 parts of <= 64 KiB: 5 frames
    items = [_stored(orc, b"key%d" % i, val, [65536] * 4 + [len(val) - 4 * 65536]) for i in range(3)]
    ok = get_values(items, 0)
    assert all(s == 0 and o == val for s, o in ok)
    res = get_values(items, 0, frame_cap=7)             # room for value 0's 5 frames only
    assert res[0] == (0, val)
    assert res[1][0] == UNSUPPORTED and res[2][0] == UNSUPPORTED


def test_offset0_match_decodes_to_zeros(gpu):
    from kingdb_amd.lz4 import decompress_blocks
    # token: 8 literals, match length 4 (nibble 0); offset 0; last token: 16 literals
    blk = bytes([0x80]) + b"abcdefgh" + b"\x00\x00" + bytes([0xF0, 0x01]) + b"ijklmnopqrstuvwx"
    filler = [bytes([0x4f]) + b"\xaa" * 4 + b"\x01\x00" + bytes([200]) + bytes([0x50]) + b"\xaa" * 5]
    # ^ a block that decodes to 0xAA bytes (4 literals, an overlapping run, 5 literals), so
    #   the decoders' LDS windows hold 0xAA when the offset-0 blocks come
    fsize = 4 + (15 + 200 + 4) + 5
    blocks = filler * 3000 + [blk] * 3000
    sizes = [fsize] * 3000 + [28] * 3000
    res = decompress_blocks(blocks, sizes)
    for r, out in res[:3000]:
        assert r == fsize and out == b"\xaa" * fsize
    for r, out in res[3000:]:
        assert r == 28
        assert out == b"abcdefgh" + b"\x00" * 4 + b"ijklmnopqrstuvwx"
