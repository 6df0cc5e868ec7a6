"""Where the host-inclusive timings disagree: the bench
line's decompress_ms (median of timed runs) against stall_profile's traced
run.  Prints every timed run in order, the traced profile, then timed runs
again, and decompress runs back to back, so a difference that comes from the
order of the runs (not from the pipeline) shows.

    python tools/hostpipe_probe.py [--values N] [--size S]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--values", type=int, default=1 << 20)
    ap.add_argument("--size", type=int, default=4096)
    a = ap.parse_args()
    import kingdb_amd as K
    from kingdb_amd.hostpipe import HostPipeline
    K.set_device(0)
    b = K.DeviceBatch.g1_long_sizes(np.full(a.values, a.size, np.uint32))
    hp = HostPipeline(a.values, a.size)
    hp.h_raw.np[:] = b.src.download(a.values * a.size)
    out = {"alternating": [], "after_profile": [], "decompress_only": [], "compress_only": []}
    for _ in range(4):
        out["alternating"].append((round(hp.compress() * 1e3, 2), round(hp.decompress() * 1e3, 2)))
    t0 = time.perf_counter()
    prof = hp.profile()
    out["profile_s"] = round(time.perf_counter() - t0, 2)
    out["profile"] = {k: prof[k].get("wall_ms") for k in ("compress", "decompress")}
    for _ in range(3):
        out["after_profile"].append((round(hp.compress() * 1e3, 2), round(hp.decompress() * 1e3, 2)))
    for _ in range(3):
        out["decompress_only"].append(round(hp.decompress() * 1e3, 2))
    for _ in range(3):
        out["compress_only"].append(round(hp.compress() * 1e3, 2))
    out["ok"] = bool(np.array_equal(hp.h_out.np, hp.h_raw.np))
    hp.h_out.np[:] = 0
    out["serial_alternating"] = []
    for _ in range(3):
        out["serial_alternating"].append((round(hp.compress() * 1e3, 2), round(hp.decompress(serial=True) * 1e3, 2)))
    out["serial_decompress_only"] = [round(hp.decompress(serial=True) * 1e3, 2) for _ in range(3)]
    out["serial_ok"] = bool(np.array_equal(hp.h_out.np, hp.h_raw.np))
    hp.dserial = True
    prof = hp.profile()
    out["serial_profile"] = prof["decompress"]
    hp.cserial = True
    out["both_serial_alternating"] = []
    for _ in range(4):
        out["both_serial_alternating"].append((round(hp.compress() * 1e3, 2), round(hp.decompress() * 1e3, 2)))
    out["both_serial_ok"] = bool(np.array_equal(hp.h_out.np, hp.h_raw.np))
    prof = hp.profile()
    out["both_serial_profile"] = {k: prof[k] for k in ("compress", "decompress")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
