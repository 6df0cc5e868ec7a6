"""Byte identity at the BASELINE sizes, without committing gigabytes.

Runs the REFERENCE's CompressorLZ4::Compress (oracle/_ref/libkdbref.so, built
from /root/reference by `make -C oracle ref`; container only) over the two
full-size batches bench.py measures, and commits for each
(generator, seed, n, sizes, sum of raw bytes, sum of frame bytes, CRC32C of the
frames concatenated) to tests/golden/digests.json:

  g1_long_4k   configs[2]/[1]: 1 048 576 x 4 096 B G1-long values (bench.py's
               headline batch: DeviceBatch.g1_long(n, 4096), first piece 0)
  mixed_1m     configs[3] on one GPU: the 1 048 576-value mixed batch of
               `bench.py --workload mixed` (kingdb_amd.lz4.mixed_sizes(1 << 20),
               consecutive G1-long slices from piece 0)

plus the same digest over each batch's first 65 536 values, which the CPU
suite checks against the oracle restatement in seconds.  The GPU suite
(tests/test_gpu_digests.py) compresses the full batches on the device and
compares the CRC32C of the packed frame stream with these numbers.

    python tests/golden/make_digests.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from kingdb_amd.lz4 import mixed_sizes  # noqa: E402  (pure numpy: the bench's size mix)

PREFIX = 65536


def batch(sizes: np.ndarray, orc: oracle.Oracle):
    sizes = np.asarray(sizes, np.uint32)
    off = np.zeros(len(sizes), np.uint64)
    off[1:] = np.cumsum(sizes[:-1].astype(np.uint64))
    total = int(sizes.astype(np.int64).sum())
    src = orc.g1_pieces((total + 99) // 100)
    return src, off, sizes


def main() -> None:
    orc = oracle.Oracle()
    ref = oracle.Reference()
    out = {}
    for name, sizes in (("g1_long_4k", np.full(1 << 20, 4096, np.uint32)),
                        ("mixed_1m", mixed_sizes(1 << 20))):
        t0 = time.time()
        src, off, lens = batch(sizes, orc)
        tot, crc = ref.frames_digest(src, off, lens)
        ptot, pcrc = ref.frames_digest(src, off[:PREFIX], lens[:PREFIX])
        out[name] = {
            "generator": "G1-long (db_bench CompressibleString 0.5, LevelDB Random(301)), pieces from 0",
            "seed": 301, "n": int(len(lens)),
            "sizes": "4096" if name == "g1_long_4k" else "kingdb_amd.lz4.mixed_sizes(1 << 20) (seed 4)",
            "size_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(lens, return_counts=True))},
            "raw_bytes": int(lens.astype(np.int64).sum()),
            "frame_bytes": tot, "frames_crc32c": f"0x{crc:08x}",
            "prefix_n": PREFIX, "prefix_frame_bytes": ptot, "prefix_frames_crc32c": f"0x{pcrc:08x}",
            "source": "oracle/_ref/libkdbref.so ref_frames_digest: the reference's algorithm/compressor.cc "
                      "CompressorLZ4::Compress + algorithm/crc32c.cc Extend",
        }
        print(name, out[name]["frame_bytes"], out[name]["frames_crc32c"], f"{time.time() - t0:.1f}s", flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "digests.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
