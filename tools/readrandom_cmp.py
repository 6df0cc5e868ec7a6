#!/usr/bin/env python3
"""db_bench's readrandom (/root/reference/doc/bench/db_bench_kingdb.cc:505-518)
through KingDB itself, in the builds of tools/write_path_cmp.py: the reference
codec (kingdb_ref), the per-call drop-in (kingdb_dropin) and the drop-in +
hooks (kingdb_hook).  Each build writes its own database of `%016d` keys and
G1 values (oracle/ref_db.cc, the same put stream for all), closes it, and then
`kdb_db --readrandom` times Database::Get of uniformly random keys from 1 and
from 16 client threads (Database::GetRaw -> CompressorLZ4::UncompressByteArray,
database.cc:9-75: one frame decode per Get -- on the GPU builds one request to
the resident decode service, kingdb_amd/csrc/service.h).

  python tools/readrandom_cmp.py --out gpurun_out/rr.json [--sizes 100,4096] [--keys N]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

from write_path_cmp import stream  # noqa: E402  (G1 values, %016d keys)

BUILDS = ["kingdb_ref", "kingdb_dropin", "kingdb_hook"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--sizes", default="100,4096")
    ap.add_argument("--keys", type=int, default=0, help="keys per size (default: 200k at 100 B, 50k at 4 KiB)")
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--dir", default=None, help="parent directory of the databases (default: a temp dir)")
    ap.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args()
    parent = tempfile.mkdtemp(prefix="kdb_rr_", dir=a.dir)
    out = {"workload": "db_bench readrandom (db_bench_kingdb.cc:505-518)", "rows": []}
    try:
        for vs in (int(x) for x in a.sizes.split(",")):
            n = a.keys or (200000 if vs <= 100 else 50000)
            s = stream(n, 16, vs)
            sp = os.path.join(parent, f"s{vs}.bin")
            s.tofile(sp)
            for b in BUILDS:
                exe = os.path.join(ROOT, "oracle", "_ref", b, "kdb_db")
                db = os.path.join(parent, f"{b}_{vs}")
                w = subprocess.run([exe, db, sp, str(1 << 20), str(32 << 20), "1"], capture_output=True, text=True,
                                   timeout=a.timeout)
                if w.returncode != 0:
                    raise SystemExit(f"{b} write failed: {w.stderr[-2000:]}")
                for t in (int(x) for x in a.threads.split(",")):
                    r = subprocess.run([exe, "--readrandom", db, str(n), str(n), str(t), str(1 << 20), str(32 << 20),
                                        "1"], capture_output=True, text=True, timeout=a.timeout,
                                       env=dict(os.environ, KDB_LZ4_READ_STATS="1"))
                    f = r.stdout.split()
                    row = {"build": b, "value_bytes": vs, "keys": n, "threads": t, "rc": r.returncode}
                    if r.returncode == 0 and f and f[0] == "readrandom":
                        row.update(reads=int(f[1]), seconds=float(f[5]), reads_per_s=float(f[7]),
                                   us_per_read_per_thread=float(f[5]) * 1e6 * t / int(f[1]))
                    else:
                        row["error"] = (r.stdout + r.stderr)[-500:]
                    out["rows"].append(row)
                    print(json.dumps(row), flush=True)
                shutil.rmtree(db, ignore_errors=True)
    finally:
        shutil.rmtree(parent, ignore_errors=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
