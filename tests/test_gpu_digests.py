"""GPU: byte identity at the BASELINE sizes.

The full batches bench.py measures are compressed on the device, the frames
are packed into one dense stream on the device (kdb_lz4_pack_frames, the bytes
KingDB appends back to back), and the stream's length and CRC32C must equal
the REFERENCE's (tests/golden/digests.json, written by
tests/golden/make_digests.py from the reference's own CompressorLZ4::Compress
over the same values).  The round trip is then checked bit-exact over every
byte of every value.

  * g1_long_4k: configs[1]/[2], 1 048 576 x 4 096 B G1-long values;
  * mixed_1m:   configs[3] on one GPU, the 1 048 576-value mixed batch
                (90 % 100 B / 9 % 4 KiB / 1 % 64 KiB by count).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _packed_digest(gpu, b, orc):
    from kingdb_amd import _lib
    from kingdb_amd.lz4 import DeviceBuffer, lib
    dense = DeviceBuffer(int(b.frames.nbytes))
    doff = DeviceBuffer(8 * b.n)
    tot = DeviceBuffer(8)
    _lib.check(lib().kdb_lz4_pack_frames(None, b.frames.ptr, b._p(2), b._p(3), b.n, dense.ptr, doff.ptr, tot.ptr),
               "pack_frames")
    total = int(tot.download(8).view(np.uint64)[0])
    stream = dense.download(total)
    crc = orc.crc32c_array(stream)
    for x in (dense, doff, tot):
        x.free()
    return total, crc


@pytest.mark.parametrize("name", ["g1_long_4k", "mixed_1m"])
def test_full_size_frames_match_reference_digest(gpu, orc, name):
    from kingdb_amd.lz4 import mixed_sizes
    g = json.load(open(os.path.join(GOLDEN, "digests.json")))[name]
    sizes = np.full(1 << 20, 4096, np.uint32) if name == "g1_long_4k" else mixed_sizes(1 << 20)
    assert g["n"] == len(sizes) and g["raw_bytes"] == int(sizes.astype(np.int64).sum())
    b = gpu.DeviceBatch.g1_long_sizes(sizes)
    b.compress()
    cst, _ = b.status()
    assert (cst == 0).all()
    assert int(b.frame_lens().astype(np.int64).sum()) == g["frame_bytes"]
    total, crc = _packed_digest(gpu, b, orc)
    assert (total, f"0x{crc:08x}") == (g["frame_bytes"], g["frames_crc32c"])
    b.decompress()
    assert b.roundtrip_ok()
    b.free()
