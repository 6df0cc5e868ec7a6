"""A/B timing of library builds on the headline batch, with a correctness gate.

    python tools/ab.py <lib.so> [--mixed] [--reps 5]

Loads the given libkdb_lz4 build (e.g. kingdb_amd/var/var_<name>.so from
tools/build_variants.sh, or the in-tree library), compresses and decompresses
the 1 Mi x 4 KiB G1-long batch (and with --mixed the 1 Mi mixed batch), times
each kernel pass with HIP events (min and median of --reps), and checks the
frame stream against tests/golden/digests.json (length + CRC32C of the packed
frames) and the round trip: a build whose output differs prints FAIL.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("so")
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--uniform", action="append", default=[],
                    help="SIZE:N extra uniform batch (round-trip gate only, no digest)")
    ap.add_argument("--no-headline", action="store_true")
    ap.add_argument("--exact-max-in", action="store_true",
                    help="decompress told the batch's largest frame (not the slot bound)")
    a = ap.parse_args()
    from kingdb_amd import _lib
    _lib.load(os.path.abspath(a.so))
    import kingdb_amd as K
    from kingdb_amd.lz4 import DeviceBuffer, lib, mixed_sizes
    import oracle
    orc = oracle.Oracle()
    K.set_device(0)
    dig = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    work = [] if a.no_headline else [("g1_long_4k", np.full(1 << 20, 4096, np.uint32))]
    if a.mixed:
        work.append(("mixed_1m", mixed_sizes(1 << 20)))
    for u in a.uniform:
        sz, cnt = (int(x) for x in u.split(":"))
        work.append((f"u{sz}x{cnt}", np.full(cnt, sz, np.uint32)))
    for name, sizes in work:
        b = K.DeviceBatch.g1_long_sizes(sizes)
        st = K.Stream()
        b.exact_max_in = a.exact_max_in
        b.compress(st)
        b.decompress(st)
        st.sync()
        e = [K.Event() for _ in range(3)]
        cs, ds = [], []
        for _ in range(a.reps):
            e[0].record(st)
            b.compress(st)
            e[1].record(st)
            b.decompress(st)
            e[2].record(st)
            cs.append(e[0].elapsed_ms(e[1]))
            ds.append(e[1].elapsed_ms(e[2]))
        dense, doff, tot = DeviceBuffer(b.frames.nbytes), DeviceBuffer(8 * b.n), DeviceBuffer(8)
        _lib.check(lib().kdb_lz4_pack_frames(None, b.frames.ptr, b._p(2), b._p(3), b.n, dense.ptr, doff.ptr,
                                             tot.ptr), "pack")
        total = int(tot.download(8).view(np.uint64)[0])
        crc = orc.crc32c_array(dense.download(total))
        g = dig.get(name)
        ok = (g is None or (total == g["frame_bytes"] and f"0x{crc:08x}" == g["frames_crc32c"])) and b.roundtrip_ok()
        rt = b.raw_bytes / 2**30 / ((np.median(cs) + np.median(ds)) / 1e3)
        print(f"{os.path.basename(a.so):24s} {name:10s} compress min {min(cs):7.3f} med {np.median(cs):7.3f} ms  "
              f"decompress min {min(ds):6.3f} med {np.median(ds):6.3f} ms  round trip {rt:6.1f} GiB/s  "
              f"{'OK' if ok else 'FAIL'}", flush=True)
        b.free()


if __name__ == "__main__":
    main()
