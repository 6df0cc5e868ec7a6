"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
of `bench.py --steps K --warmup 0 --no-cpu-baseline`, corrected as
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes: FETCH_SIZE on
gfx950 reports half the bytes of wide streaming reads -> doubled; WRITE_SIZE
taken as is.  rocprofv3's derived FETCH_SIZE / WRITE_SIZE are in KiB.

    python tools/pmc_traffic.py <pass_fetch_dir> <pass_write_dir> <values> <size|mixed> [out.json]

size "mixed" (bench.py --workload mixed): a step launches one kernel per size
class and kind; the step's traffic of a kind is the SUM over its kernels (each
launched once per step), matching the roofline's "all compress launches of the
step".  Otherwise the kind's dominant (largest) kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(root, counter, total=False):
    vals = defaultdict(list)
    names = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            full = row.get("Kernel_Name", "?")
            short = full.split("(")[0].replace("void ", "")
            key = ("decompress" if "lz4_decompress" in short else "compress" if "lz4_compress" in short
                   else "pack_copy" if "pack_copy" in short else "pack_scan" if "pack_scan" in short else None)
            if key is None:
                continue
            vals[(key, short)].append(float(row["Counter_Value"]))
    # several kernels of one kind per step (size-class launches, most of them
    # returning at once): the kind's dominant kernel is the one with the most bytes
    out = {}
    for (key, short), v in vals.items():
        m = sum(v) / len(v)
        if total:
            out[key] = out.get(key, 0.0) + m
            names[key] = (names[key] + " + " if key in names else "") + short
        elif key not in out or m > out[key]:
            out[key] = m
            names[key] = short
    return out, names


def main():
    fdir, wdir, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    size = sys.argv[4] if sys.argv[4] == "mixed" else int(sys.argv[4])
    mixed = size == "mixed"
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic_mixed.json" if mixed else "pmc_traffic.json")
    fetch, names = per_kernel(fdir, "FETCH_SIZE", mixed)
    write, names2 = per_kernel(wdir, "WRITE_SIZE", mixed)
    names.update(names2)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from kingdb_amd import lz4  # the build the passes ran (bench.py refuses the summary for any other)
    res = {"values": n, "size": size, "build_id": lz4.build_id(),
           "passes": [os.path.normpath(fdir), os.path.normpath(wdir)],
           "scope": "sum of the kind's launches in one step" if mixed else "the kind's dominant launch",
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KiB x 1024; "
                     "FETCH_SIZE doubled (gfx950 half-count of wide reads, MI355X_MICROARCH.md HBM section) -- "
                     "exact for wide streaming reads; each kernel's `correction` says whether that holds",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k)
        w = write.get(k)
        rd = None if f is None else 2.0 * f * 1024.0
        rd1 = None if f is None else f * 1024.0
        wr = None if w is None else w * 1024.0
        nm = names.get(k) or ""
        # The guide's x2 is calibrated for wide (16 B per lane) streaming reads only.
        # The LDS-staged kernels read their inputs that way (register prefetch /
        # staging of whole 16-byte chunks), so x2 applies.  The in-place compress
        # classes (big / mixed kernels) also gather 4-byte candidate words and the
        # ring decoder refills with dword loads: for them the true read bytes lie
        # between the raw count and twice it, and both are reported.
        narrow = any(t in nm for t in ("big_kernel", "big_compact_kernel", "mixed_kernel", "mixed24_kernel"))
        res["kernels"][k] = {
            "kernel": nm, "fetch_size_kib_raw": f, "write_size_kib_raw": w,
            "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
            "hbm_bytes_per_launch": None if rd is None or wr is None else rd + wr,
            "hbm_bytes_per_launch_undoubled": None if rd1 is None or wr is None else rd1 + wr,
            "correction": ("FETCH_SIZE x2 applies: every read is a 16 B-per-lane streaming load" if not narrow else
                           "bounds: the launch mixes 16 B-per-lane streaming loads with 4-byte gathers, for "
                           "which the guide's x2 is uncalibrated; the true HBM bytes lie between "
                           "hbm_bytes_per_launch_undoubled and hbm_bytes_per_launch"),
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
