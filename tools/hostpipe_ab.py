"""Host-inclusive pipeline configurations side by side (kingdb_amd/hostpipe.py):
chunk size, compute streams and device-to-host drain streams per direction.

    python tools/hostpipe_ab.py [--values N] [--size S] CHUNK:STREAMS:CDRAIN:DDRAIN ...

Median of 3 (after one warm-up) compress and decompress wall times over the
1 Mi x 4 KiB G1-long batch, and the round trip; every configuration checks the
round trip byte for byte."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--values", type=int, default=1 << 20)
    ap.add_argument("--size", type=int, default=4096)
    a = ap.parse_args()
    import kingdb_amd as K
    from kingdb_amd.hostpipe import HostPipeline
    K.set_device(0)
    b = K.DeviceBatch.g1_long_sizes(np.full(a.values, a.size, np.uint32))
    raw = b.src.download(a.values * a.size)
    for cfg in a.configs:
        chunk, ns, cd, dd = (int(x) for x in cfg.split(":"))
        hp = HostPipeline(a.values, a.size, chunk=chunk, nstreams=ns, cdrain=cd, ddrain=dd)
        hp.h_raw.np[:] = raw
        hp.compress()
        hp.decompress()
        tc, td = [], []
        for _ in range(3):
            tc.append(hp.compress())
            td.append(hp.decompress())
        ok = np.array_equal(hp.h_out.np, hp.h_raw.np)
        gib = a.values * a.size / 2**30
        c, d = float(np.median(tc)), float(np.median(td))
        print(f"{cfg:16s} compress {c*1e3:7.1f} ms ({gib/c:5.1f} GiB/s)  decompress {d*1e3:7.1f} ms ({gib/d:5.1f} GiB/s)"
              f"  round trip {gib/(c+d):5.1f} GiB/s  {'OK' if ok else 'FAIL'}", flush=True)
        hp.free()
    b.free()


if __name__ == "__main__":
    main()
