"""Probe: is the in-place compress class (64 KiB values, read from HBM/L2)
bound by HBM misses on the value's bytes?  Times the same 64 KiB batch with
every value at its own offset (cold: each byte is fetched from HBM once) and
with the values' offsets folded onto the first K values (hot: the working set
is K x 64 KiB, resident in L2/MALL).  Output frames are not checked (the hot
batch compresses K distinct values many times).

    python tools/probe/inplace_hot.py [--n 10486] [--size 65536] [--k 1,16,64]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10486)
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--k", default="1,16,64,256")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import kingdb_amd as K
    K.set_device(0)
    b = K.DeviceBatch.g1_long(a.n, a.size)
    st = K.Stream()
    e = [K.Event(), K.Event()]

    def timed():
        b.compress(st)
        st.sync()
        ts = []
        for _ in range(a.reps):
            e[0].record(st)
            b.compress(st)
            e[1].record(st)
            st.sync()
            ts.append(e[0].elapsed_ms(e[1]))
        return min(ts), float(np.median(ts))

    print(f"cold (own offsets): min {timed()[0]:.3f} ms", flush=True)
    for k in (int(x) for x in a.k.split(",")):
        off = b.src_off[np.arange(a.n) % k].copy()
        b.meta.upload(off.view(np.uint8))          # src_off is the first field of meta
        mn, md = timed()
        print(f"hot  (K={k:4d} distinct values, {k * a.size / 2**20:.1f} MiB): min {mn:.3f} med {md:.3f} ms",
              flush=True)
    b.meta.upload(b.src_off.view(np.uint8))
    print(f"cold again: min {timed()[0]:.3f} ms", flush=True)
    b.free()


if __name__ == "__main__":
    main()
