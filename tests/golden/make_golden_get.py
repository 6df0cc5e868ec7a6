#!/usr/bin/env python3
"""Golden fixtures for the read path: stored values and what the
REFERENCE's CompressorLZ4::UncompressByteArray makes of them.

Inputs are the value regions of every entry of the HSTable files the reference
wrote in tests/golden/hstable_streams.npz (make_golden_put.py), plus mutated
copies (flipped bytes, bent frame headers, short size_value_compressed).  The
expected status (with and without checksum verification) and output come from
oracle/_ref/libkdbref.so (ref_uncompress_value).  Mutations on which the
reference would read or write outside the value (undefined behaviour there;
the oracle says -3) are not run on the reference: they are kept with status
"undefined", and only an error is required of the GPU.

    python tests/golden/make_golden_get.py     -> tests/golden/get_values.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from kingdb_amd.get import entry_items, read_hstable  # noqa: E402  (host-side parser)

OUT = os.path.join(ROOT, "tests", "golden", "get_values.npz")
UNDEF = 99


def main() -> None:
    orc, ref = oracle.Oracle(), oracle.Reference()
    z = np.load(os.path.join(ROOT, "tests", "golden", "hstable_streams.npz"))
    items = []
    for name in z["names"]:
        for fn in z[f"{name}__files"]:
            f = z[f"{name}__file_{fn}"].tobytes()
            items += entry_items(f, read_hstable(f), orc.crc32c)
    rng = np.random.default_rng(11)
    base = list(items)
    framed = [it for it in base if it[1] > 0 and it[0][:8] != bytes(8)]
    for k in range(600):
        st, svc, size, ck, ci = framed[int(rng.integers(len(framed)))]
        b = bytearray(st)
        kind = k % 5
        if kind == 0:                                   # flip bytes in the frame payloads
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(8, max(9, svc)))
                b[p % len(b)] ^= int(rng.integers(1, 256))
        elif kind == 1:                                 # bend the stored size of the first frame
            d = int(rng.integers(-20, 21)) or 1
            v = int.from_bytes(b[0:4], "little") + d
            b[0:4] = (v & 0xFFFFFFFF).to_bytes(4, "little")
        elif kind == 2:                                 # bend the raw size of the first frame
            v = int.from_bytes(b[4:8], "little") + int(rng.integers(-40, 41))
            b[4:8] = (v & 0xFFFFFFFF).to_bytes(4, "little")
        elif kind == 3:                                 # size_value_compressed off by a little
            svc = max(1, svc + int(rng.integers(-9, 10)))
        else:                                           # zero a frame header (disable mid-value)
            b[0:8] = bytes(8)
        items.append((bytes(b), svc, size, ck, ci))
    st_all, svc_all, size_all, ck_all, ci_all = [], [], [], [], []
    exp = {0: [], 1: []}
    for st, svc, size, ck, ci in items:
        st_all.append(st)
        svc_all.append(svc)
        size_all.append(size)
        ck_all.append(ck)
        ci_all.append(ci)
        for verify in (0, 1):
            o_st, _ = orc.get_value(st, svc, size, ck, ci, verify)
            if o_st == -3:
                exp[verify].append((UNDEF, b""))
                continue
            r_st, out = ref.uncompress_value(st, svc, size, ck, ci, bool(verify))
            # the reference returns a size_value-byte buffer; bytes past what it
            # decoded or copied are uninitialised -- keep the prefix it wrote
            # (the oracle's defined length) and check the oracle agrees on it
            if r_st == 0:
                _, o_out = orc.get_value(st, svc, size, ck, ci, verify)
                assert len(out) == size and out[:len(o_out)] == o_out
                out = out[:len(o_out)]
            exp[verify].append((r_st, out if r_st == 0 else b""))
    lens = np.array([len(s) for s in st_all], np.uint64)
    arrs = dict(stored=np.frombuffer(b"".join(st_all), np.uint8), stored_len=lens,
                svc=np.array(svc_all, np.uint64), size=np.array(size_all, np.uint64),
                checksum=np.array(ck_all, np.uint32), checksum_initial=np.array(ci_all, np.uint32))
    for verify in (0, 1):
        arrs[f"status_v{verify}"] = np.array([e[0] for e in exp[verify]], np.int32)
        arrs[f"out_crc_v{verify}"] = np.array([orc.crc32c(e[1]) for e in exp[verify]], np.uint32)
        arrs[f"out_len_v{verify}"] = np.array([len(e[1]) for e in exp[verify]], np.uint64)
    np.savez_compressed(OUT, **arrs)
    s0 = arrs["status_v0"]
    s1 = arrs["status_v1"]
    print(f"{len(items)} values ({len(base)} from reference HSTables): verify=0 ok {int((s0 == 0).sum())} "
          f"err {int(((s0 != 0) & (s0 != UNDEF)).sum())} undef {int((s0 == UNDEF).sum())}; verify=1 ok "
          f"{int((s1 == 0).sum())} bad-crc {int((s1 == 1).sum())}; {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
