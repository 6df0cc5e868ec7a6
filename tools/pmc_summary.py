"""Summarise rocprofv3 --pmc CSV passes: per kernel, the mean of each counter
per dispatch (and per wave where SQ_WAVES is present)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        short = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    if "gen_g1" in k:
        continue
    print(k)
    waves = None
    if "SQ_WAVES" in cs:
        waves = sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"])
    for c in sorted(cs):
        v = sum(cs[c]) / len(cs[c])
        extra = f"   per-wave {v / waves:14.1f}" if waves else ""
        print(f"  {c:28s} {v:18.1f}{extra}")
