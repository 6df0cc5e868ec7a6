"""Diagnostic: per-phase shader-clock breakdown of the compress kernel.

Loads build/libkdb_lz4_stamps.so (make -C kingdb_amd stamps) in place of the
product library, runs one G1-long batch, and prints mean cycles per value for
each phase.  Never used for reported numbers (stamps perturb timing)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kingdb_amd import _lib  # noqa: E402

so = os.path.join(ROOT, "kingdb_amd", "build", "libkdb_lz4_stamps.so")
lib = _lib.load(so)
lib.kdb_lz4_stamps_read.argtypes = [ctypes.c_void_p]
import kingdb_amd as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
size = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
K.set_device(0)
b = K.DeviceBatch.g1_long(n, size)
b.compress()
lib.kdb_lz4_device_sync()
lib.kdb_lz4_stamps_reset()
ev0, ev1 = K.Event(), K.Event()
ev0.record()
b.compress()
ev1.record()
ms = ev0.elapsed_ms(ev1)
buf = (ctypes.c_ulonglong * 16)()
lib.kdb_lz4_stamps_read(ctypes.addressof(buf))
names = {0: "stage+zero", 1: "search", 2: "catchup", 3: "literals", 4: "match", 5: "nextpos", 6: "last-lit",
         7: "misc", 10: "epilogue"}
tot = sum(buf[i] for i in names)
print(f"n={n} size={size} kernel {ms:.3f} ms; cycles/value total {tot / n:.0f}")
for i, nm in names.items():
    print(f"  {nm:12s} {buf[i] / n:10.0f} cyc/value  {100 * buf[i] / max(tot, 1):5.1f}%")
print(f"  chunks/value {buf[8] / n:.2f}  sequences/value {buf[9] / n:.2f}")
