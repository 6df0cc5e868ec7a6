"""Diagnostic: time the compress/decompress kernels of one or more library
builds (e.g. ablation variants under kingdb_amd/build/) on the same batch.
Timing only -- ablated builds produce wrong output by design."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    so = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    from kingdb_amd import _lib
    _lib.load(so)
    import kingdb_amd as K
    K.set_device(0)
    b = K.DeviceBatch.g1_long(n, size)
    st = K.Stream()
    b.compress(st)
    b.decompress(st)
    st.sync()
    e = [K.Event() for _ in range(3)]
    cs, ds = [], []
    for _ in range(3):
        e[0].record(st)
        b.compress(st)
        e[1].record(st)
        b.decompress(st)
        e[2].record(st)
        cs.append(e[0].elapsed_ms(e[1]))
        ds.append(e[1].elapsed_ms(e[2]))
    print(f"{os.path.basename(so):32s} n={n} size={size} compress {min(cs):8.3f} ms  decompress {min(ds):8.3f} ms")


if __name__ == "__main__":
    main()
