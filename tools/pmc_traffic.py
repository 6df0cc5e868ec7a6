"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
of `bench.py --steps K --warmup 0 --no-cpu-baseline`, corrected as
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes: FETCH_SIZE on
gfx950 reports half the bytes of wide streaming reads -> doubled; WRITE_SIZE
taken as is.  rocprofv3's derived FETCH_SIZE / WRITE_SIZE are in KiB.

    python tools/pmc_traffic.py <pass_fetch_dir> <pass_write_dir> <values> <size> [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(root, counter):
    vals = defaultdict(list)
    names = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            full = row.get("Kernel_Name", "?")
            short = full.split("(")[0].replace("void ", "")
            key = ("decompress" if "decompress_kernel" in short else "compress" if "compress_kernel" in short
                   else "pack_copy" if "pack_copy" in short else "pack_scan" if "pack_scan" in short else None)
            if key is None:
                continue
            vals[(key, short)].append(float(row["Counter_Value"]))
    # several kernels of one kind per step (size-class launches, most of them
    # returning at once): the kind's dominant kernel is the one with the most bytes
    out = {}
    for (key, short), v in vals.items():
        m = sum(v) / len(v)
        if key not in out or m > out[key]:
            out[key] = m
            names[key] = short
    return out, names


def main():
    fdir, wdir, n, size = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    fetch, names = per_kernel(fdir, "FETCH_SIZE")
    write, names2 = per_kernel(wdir, "WRITE_SIZE")
    names.update(names2)
    res = {"values": n, "size": size,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KiB x 1024; "
                     "FETCH_SIZE doubled (gfx950 half-count of wide reads, MI355X_MICROARCH.md HBM section)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k)
        w = write.get(k)
        rd = None if f is None else 2.0 * f * 1024.0
        wr = None if w is None else w * 1024.0
        res["kernels"][k] = {"kernel": names.get(k), "fetch_size_kib_raw": f, "write_size_kib_raw": w,
                             "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                             "hbm_bytes_per_launch": None if rd is None or wr is None else rd + wr}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
