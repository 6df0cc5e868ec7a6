#!/usr/bin/env python3
"""bench.py -- LZ4 compress+decompress GiB/s (device-resident), batched 4 KiB values.

BASELINE.json metric on its single-GPU config: 1M x 4 KiB values ("configs"[2]:
round trip, frames byte-identical to the reference).  One *step* = one
CompressorLZ4 frame-compress launch over the whole batch followed by one
frame-decompress launch of the frames it produced (the kernels in
kingdb_amd/csrc); inputs are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W]

For N > 1 the driver starts one process per GPU with torch.distributed.run;
each rank owns its own shard of G1-long values (no collective on the data
path -- LZ4 blocks are independent); gloo carries only the
barrier and the max-over-ranks of the elapsed time.  `value` is the raw bytes
all ranks processed / max elapsed.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "LZ4 compress+decompress GiB/s (device-resident), batched 4 KiB values, 1/8 GPU"
# --workload big: the same round trip on KingDB's default part size (a side line, not the headline)
METRIC_BIG = "LZ4 compress+decompress GiB/s (device-resident), KingDB 1 MiB parts (byU32 blocks), 1/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--values", type=int, default=None, help="values per GPU (default 1 Mi; big: 2560)")
    p.add_argument("--size", type=int, default=None, help="bytes per value (default 4096; big: 1 MiB)")
    p.add_argument("--workload", choices=("uniform", "mixed", "put", "get", "big"), default="uniform",
                   help="uniform: --values x --size (configs[2], the headline); mixed: configs[3], "
                        "--values per GPU of 90%% 100 B / 9%% 4 KiB / 1%% 64 KiB parts, byte-balanced shards; "
                        "put: configs[4], --values puts per GPU of 16 B keys / 100 B values from pinned host "
                        "memory to HSTable file bytes in host memory; get: the read path (configs[1] shape), "
                        "UncompressByteArray over --values stored --size B values resident in HBM; big: KingDB's "
                        "default part size (util/options.h:171-172: 1 MB parts, byU32 blocks, lz4.cc:673-676), "
                        "--values x --size B as the uniform workload (default 2560 x 1 MiB: one part per wave "
                        "slot of the in-place kernels, 10 per CU)")
    p.add_argument("--put-host-copy", action="store_true",
                   help="put workload: land entry bytes in a pinned staging buffer and memcpy them into the "
                        "files (the default DMAs them from HBM straight into pinned file buffers)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target wall time of the CPU leg")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--host-inclusive", action="store_true",
                   help="(default for the uniform workload) also time pinned host -> device -> host "
                        "(H2D + kernels + D2H, overlapped)")
    p.add_argument("--no-host-inclusive", action="store_true", help="skip the host-inclusive leg")
    p.add_argument("--hi-chunk", type=int, default=1 << 16, help="values per pipeline chunk")
    p.add_argument("--hi-streams", type=int, default=4)
    p.add_argument("--put-chunk", type=int, default=1 << 17, help="put workload: puts per pipeline chunk")
    p.add_argument("--pmc", default=None,
                   help="HBM traffic summary written by tools/pmc_traffic.py (default: "
                        "profiles/pmc_traffic.json, profiles/pmc_traffic_mixed.json for --workload mixed, "
                        "profiles/pmc_traffic_big.json for --workload big)")
    a = p.parse_args()
    if a.values is None:
        a.values = 2560 if a.workload == "big" else 1 << 20
    if a.size is None:
        a.size = 1 << 20 if a.workload == "big" else 4096
    return a


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_threads() -> tuple:
    """Threads for a CPU leg and how they were chosen: every core the process
    affinity allows, capped by OMP_NUM_THREADS where that is set -- on the GPU
    box the harness sets it to the lease's CPU share (16 per GPU) while nproc and
    the affinity mask show the whole machine, and worker pools are to be sized to
    the share."""
    nproc = os.cpu_count() or 1
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    cap_env = os.environ.get("OMP_NUM_THREADS")
    cap = int(cap_env) if cap_env and cap_env.isdigit() and int(cap_env) > 0 else None
    threads = max(1, min(affinity, cap) if cap else affinity)
    return threads, {"nproc": nproc, "affinity": affinity, "cap": cap,
                     "cap_source": "OMP_NUM_THREADS (the lease's CPU share)" if cap else None, "threads": threads}


def cpu_baseline(sample: np.ndarray, size: int, seconds: float) -> dict:
    """Times the reference's algorithm/lz4.cc (oracle/_ref, kind "reference")
    or, where that build is absent, the oracle restatement (kind "port") on the
    host cores, on a bounded sample of the same G1-long values."""
    import oracle  # checker / baseline only
    ref_so = oracle.REF_SO
    if os.path.exists(ref_so):
        lib = ctypes.CDLL(ref_so)
        fn, kind = lib.ref_bench_roundtrip, "reference"
    else:
        lib = ctypes.CDLL(oracle.Oracle().lib._name)
        fn, kind = lib.orc_bench_roundtrip, "port"
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                   ctypes.POINTER(ctypes.c_uint64)]
    threads, host = host_threads()

    def run(n, th, passes):
        tc, td, cb = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        rc = fn(sample.ctypes.data, n, size, th, passes, ctypes.byref(tc), ctypes.byref(td), ctypes.byref(cb))
        if rc != 0:
            raise RuntimeError("CPU baseline round trip failed")
        return tc.value, td.value

    nall = len(sample) // size
    res = {}
    for label, th, n, budget in (("all", threads, nall, 0.7 * seconds), ("one", 1, max(nall // 16, 1024), 0.3 * seconds)):
        tc, td = run(n, th, 1)
        passes = int(min(50, max(1, math.ceil(budget / max(tc + td, 1e-3)))))
        tc, td = run(n, th, passes)
        raw = float(n) * size * passes
        res[label] = dict(rt=raw / (tc + td) / GIB, c=raw / tc / GIB, d=raw / td / GIB, n=n, passes=passes)
    a, o = res["all"], res["one"]
    return {
        "value": round(a["rt"], 3), "unit": "GiB/s", "cores": threads, "kind": kind, "host": host,
        "per_core_gibs": round(a["rt"] / threads, 3),
        "sample": (f"{a['n']} x {size} B G1-long values (the first values of the GPU batch), "
                   f"{a['passes']} timed round-trip passes after 1 warm-up, blocked partition over "
                   f"{threads} threads; CPU: {cpu_model()}"),
        "compress_gibs": round(a["c"], 3), "decompress_gibs": round(a["d"], 3),
        "one_thread": {"value": round(o["rt"], 3), "compress_gibs": round(o["c"], 3),
                       "decompress_gibs": round(o["d"], 3), "values": o["n"], "passes": o["passes"]},
        "source": ("algorithm/lz4.cc LZ4_compress_limitedOutput + LZ4_decompress_safe_partial, compiled "
                   "from the reference (oracle/_ref)" if kind == "reference" else
                   "oracle/lz4_oracle.c restatement (reference build absent)"),
    }


def cpu_baseline_mixed(sample: np.ndarray, off: np.ndarray, lens: np.ndarray, seconds: float) -> dict | None:
    """configs[3]'s CPU path: the reference's algorithm/lz4.cc round trip
    (oracle/_ref ref_bench_roundtrip_var) over a bounded prefix of the same
    mixed batch, every value one block as CompressorLZ4 makes it; None where the
    reference build is absent."""
    import oracle  # checker / baseline only
    if not os.path.exists(oracle.REF_SO):
        return None
    lib = ctypes.CDLL(oracle.REF_SO)
    fn = lib.ref_bench_roundtrip_var
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                   ctypes.POINTER(ctypes.c_uint64)]
    threads, host = host_threads()
    off = np.ascontiguousarray(off, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)

    def run(n, th, passes):
        tc, td, cb = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        if fn(sample.ctypes.data, off.ctypes.data, lens.ctypes.data, n, th, passes, ctypes.byref(tc),
              ctypes.byref(td), ctypes.byref(cb)) != 0:
            raise RuntimeError("CPU baseline round trip failed")
        return tc.value, td.value

    res = {}
    nall = len(lens)
    for label, th, n, budget in (("all", threads, nall, 0.7 * seconds), ("one", 1, max(nall // 16, 1024), 0.3 * seconds)):
        n = min(n, nall)
        tc, td = run(n, th, 1)
        passes = int(min(50, max(1, math.ceil(budget / max(tc + td, 1e-3)))))
        tc, td = run(n, th, passes)
        raw = float(lens[:n].astype(np.int64).sum()) * passes
        res[label] = dict(rt=raw / (tc + td) / GIB, c=raw / tc / GIB, d=raw / td / GIB, n=n, passes=passes)
    a, o = res["all"], res["one"]
    return {
        "value": round(a["rt"], 3), "unit": "GiB/s", "cores": threads, "kind": "reference", "host": host,
        "per_core_gibs": round(a["rt"] / threads, 3),
        "sample": (f"the first {a['n']} values of the mixed batch ({int(lens.astype(np.int64).sum())} B), "
                   f"{a['passes']} timed round-trip passes after 1 warm-up, byte-balanced over {threads} threads; "
                   f"CPU: {cpu_model()}"),
        "compress_gibs": round(a["c"], 3), "decompress_gibs": round(a["d"], 3),
        "one_thread": {"value": round(o["rt"], 3), "compress_gibs": round(o["c"], 3),
                       "decompress_gibs": round(o["d"], 3), "values": o["n"], "passes": o["passes"]},
        "source": "algorithm/lz4.cc LZ4_compress_limitedOutput + LZ4_decompress_safe_partial, compiled "
                  "from the reference (oracle/_ref)",
    }


def compressor_calls_100b() -> dict | None:
    """configs[0]: unit-tests/test_compression.cc's shape -- CompressorLZ4 on
    100-byte values, one thread -- timed with the reference's own class
    (oracle/_ref/kingdb_ref/bench_compressor, built from /root/reference) and
    with the drop-in class (oracle/_ref/kingdb_dropin/bench_compressor: one GPU
    call per value, the scalar zero-copy path); None where not built."""
    import subprocess
    out = {}
    for kind, d in (("reference", "kingdb_ref"), ("dropin", "kingdb_dropin")):
        exe = os.path.join(ROOT, "oracle", "_ref", d, "bench_compressor")
        if not os.path.exists(exe):
            return None
        r = subprocess.run([exe, "100", "20000" if kind == "reference" else "2000"], capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            out[kind] = {"error": f"rc={r.returncode}: {r.stderr.strip()[-200:]}"}
            continue
        j = json.loads(r.stdout.strip().splitlines()[-1])
        out[kind] = {"compress_us": j["compress_us"], "uncompress_us": j["uncompress_us"], "calls": j["calls"]}
    out["unit"] = "us per CompressorLZ4::Compress / Uncompress call, one thread, 100 B G1 values"
    return out


def host_inclusive(batch, n: int, size: int, args) -> dict:
    """Pinned host buffers -> H2D -> frame kernel -> pack -> D2H (ΣF bytes)
    and back, chunked and overlapped over several streams (kingdb_amd/hostpipe.py).
    Reported beside `value`, never as it."""
    from kingdb_amd.hostpipe import HostPipeline
    hp = HostPipeline(n, size, chunk=args.hi_chunk, nstreams=args.hi_streams)
    hp.h_raw.np[:] = batch.src.download(n * size)
    hp.compress()
    hp.decompress()
    tc, td = [], []
    for _ in range(3):
        tc.append(hp.compress())
        td.append(hp.decompress())
    cst, dst = hp.status()
    ok = bool((cst == 0).all() and (dst == 0).all() and hp.frame_bytes == int(batch.frame_lens().astype(np.int64).sum())
              and np.array_equal(hp.h_out.np, hp.h_raw.np))
    if not ok:
        raise SystemExit("bench: host-inclusive round trip is not bit-exact")
    raw = float(n) * size
    c, d = float(np.median(tc)), float(np.median(td))
    res = {
        "value": round(raw / (c + d) / GIB, 3), "unit": "GiB/s",
        "compress_gibs": round(raw / c / GIB, 3), "decompress_gibs": round(raw / d / GIB, 3),
        "compress_ms": round(c * 1e3, 3), "decompress_ms": round(d * 1e3, 3),
        "pcie_bytes": {"compress_h2d": int(raw) + 20 * n, "compress_d2h": hp.frame_bytes + 8 * n,
                       "decompress_h2d": hp.frame_bytes + 12 * n, "decompress_d2h": int(raw) + 8 * n},
        "chunk": hp.chunk, "streams": len(hp.streams),
        "copies": ("serial: each phase's H2D copies in chunk order on one stream, D2H on another, no copy stream "
                   "used for both directions" if hp.cserial and hp.dserial else "per-chunk streams"),
        "timing": "host wall clock, first enqueue to last byte in pinned host memory; median of 3 after 1 warm-up",
    }
    # where the wall time goes (traced runs after the timed ones; weak #9 of round 2)
    res["stall_profile"] = hp.profile()
    # the traced runs measure the same pipeline: their wall time against the timed median
    res["traced_over_timed"] = {ph: round(res["stall_profile"][ph]["wall_ms"] / res[ph + "_ms"], 3)
                                for ph in ("compress", "decompress")}
    hp.free()
    return res


def copy_bandwidth(batch, stream, reps: int = 5) -> float:
    """Achievable HBM copy rate on this device: hipMemcpyAsync
    device-to-device of the raw buffer, (read + write bytes) / time, HIP events
    on the bench stream.  Run after the round trip was verified (it overwrites
    the decoded output with the same bytes)."""
    import kingdb_amd as K
    from kingdb_amd import _lib
    from kingdb_amd import lz4 as L
    nb = int(batch.raw_bytes)

    def cp():
        _lib.check(L.lib().kdb_lz4_memcpy_d2d(batch.out.ptr, batch.src.ptr, nb, stream.ptr), "memcpy_d2d")
    cp()
    e0, e1 = K.Event(), K.Event()
    e0.record(stream)
    for _ in range(reps):
        cp()
    e1.record(stream)
    ms = e0.elapsed_ms(e1) / reps
    return 2.0 * nb / (ms * 1e-3) / 1e9


def ref_write_path(keys: np.ndarray, vals: np.ndarray) -> dict | None:
    """configs[4] CPU path: the reference's own Database::PutPart -> WriteBuffer ->
    HSTableManager (oracle/_ref/ref_db, built from /root/reference) on the same
    puts, writing its HSTables to a scratch directory; None where not built."""
    import shutil
    import struct
    import subprocess
    import tempfile
    import oracle  # checker / baseline only
    exe = os.path.join(os.path.dirname(oracle.REF_SO), "ref_db")
    if not os.path.exists(exe):
        return None
    n, ks = keys.shape
    vs = vals.shape[1]
    rec = np.zeros((n, 4 + ks + 8 + 4 + 4 + vs), np.uint8)
    rec[:, 0:4] = np.frombuffer(struct.pack("<I", ks), np.uint8)
    rec[:, 4:4 + ks] = keys
    rec[:, 4 + ks:12 + ks] = np.frombuffer(struct.pack("<Q", vs), np.uint8)
    rec[:, 12 + ks:16 + ks] = np.frombuffer(struct.pack("<I", 1), np.uint8)
    rec[:, 16 + ks:20 + ks] = np.frombuffer(struct.pack("<I", vs), np.uint8)
    rec[:, 20 + ks:] = vals
    d = tempfile.mkdtemp(prefix="kdbref")
    try:
        rec.tofile(os.path.join(d, "s.bin"))
        try:
            # the reference's own KingDB can stop making progress (tools/write_path_cmp.py):
            # bounded, so a stuck baseline cannot take the GPU line down with it
            r = subprocess.run([exe, os.path.join(d, "db"), os.path.join(d, "s.bin")], check=True,
                               capture_output=True, text=True, timeout=100)
        except subprocess.TimeoutExpired:
            return {"value": None, "unit": "puts/s", "cores": 1, "kind": "reference",
                    "note": "the reference's write path (oracle/_ref/ref_db) made no progress within 100 s and was "
                            "killed; no CPU number this run"}
        f = r.stdout.split()
        t_put, t_all = float(f[2]), float(f[5])
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"value": round(n / t_put, 1), "unit": "puts/s", "cores": 1, "kind": "reference",
            "sample": f"{n} puts ({ks} B keys, {vs} B G1 values), the GPU batch's own, one client thread "
                      f"(KingDB's write buffer and storage threads behind it), HSTables on local disk; "
                      f"CPU: {cpu_model()}",
            "with_close_puts_per_s": round(n / t_all, 1), "seconds_put": round(t_put, 4),
            "seconds_with_close": round(t_all, 4),
            "source": "interface/database.cc PutPart -> cache/write_buffer.cc -> storage/hstable_manager.h, "
                      "compiled from the reference (oracle/_ref/ref_db)"}


def ref_read_path(stored: np.ndarray, off: np.ndarray, lens: np.ndarray, size: int, seconds: float) -> dict | None:
    """configs[1] CPU path: the reference's CompressorLZ4::UncompressByteArray
    (oracle/_ref, compiled from /root/reference) over a bounded sample of the
    same stored values, on all host cores; None where not built."""
    import oracle  # checker / baseline only
    if not os.path.exists(oracle.REF_SO):
        return None
    lib = ctypes.CDLL(oracle.REF_SO)
    fn = lib.ref_bench_get
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                   ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    threads, host = host_threads()
    n = len(lens)
    off = np.ascontiguousarray(off, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint64)
    t = ctypes.c_double()
    if fn(stored.ctypes.data, off.ctypes.data, lens.ctypes.data, n, size, threads, 1, ctypes.byref(t)) != 0:
        raise RuntimeError("reference read path failed on the sample")
    passes = int(min(50, max(1, math.ceil(seconds / max(t.value, 1e-3)))))
    if fn(stored.ctypes.data, off.ctypes.data, lens.ctypes.data, n, size, threads, passes, ctypes.byref(t)) != 0:
        raise RuntimeError("reference read path failed on the sample")
    return {"value": round(float(n) * size * passes / t.value / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "reference", "host": host,
            "sample": f"{n} stored {size} B G1-long values (the first of the GPU batch), {passes} timed passes after "
                      f"1 warm-up, blocked over {threads} threads; CPU: {cpu_model()}",
            "source": "algorithm/compressor.cc CompressorLZ4::UncompressByteArray (verify off), compiled from the "
                      "reference (oracle/_ref)"}


def bench_get(args, world: int, rank: int, local: int, barrier, sync_all) -> None:
    """configs[1] as KingDB reads it: Database::GetRaw's UncompressByteArray over
    a batch of stored values (one frame each at 4 KiB) already in HBM -- the
    frame walk, the frame decode and the status/size pass of
    kdb_get_values_batch (csrc/get.hip), verify off (ReadOptions' default)."""
    import kingdb_amd as K
    from kingdb_amd import _lib
    from kingdb_amd import lz4 as L
    from kingdb_amd.lz4 import DeviceBuffer
    from kingdb_amd.shard import g1_first_piece, gather_ranks, max_over_ranks
    n, size = args.values, args.size
    stream = K.Stream()
    batch = K.DeviceBatch.g1_long(n, size, first_piece=g1_first_piece(rank, n, size), stream=stream)
    batch.compress(stream)            # the stored values: one CompressorLZ4 frame each
    stream.sync()
    cst, _ = batch.status()
    if not (cst == 0).all():
        raise SystemExit("bench: could not build the stored values")
    flen = batch.frame_lens().astype(np.uint64)
    sizes = batch.sizes.astype(np.uint64)
    zeros32 = np.zeros(n, np.uint32)
    # stored_off u64 | avail u64 | svc u64 | size u64 | out_off u64 | checksum u32 | checksum_initial u32 |
    # out_len u64 | status i32
    m = np.concatenate([batch.frame_off.astype(np.uint64).view(np.uint8), flen.view(np.uint8), flen.view(np.uint8),
                        sizes.view(np.uint8), batch.src_off.astype(np.uint64).view(np.uint8), zeros32.view(np.uint8),
                        zeros32.view(np.uint8), np.zeros(n, np.uint64).view(np.uint8), np.zeros(n, np.int32).view(np.uint8)])
    meta = DeviceBuffer(m.nbytes)
    meta.upload(m, stream=stream.ptr)
    lib = L.lib()
    frame_cap = n
    sb = int(lib.kdb_get_scratch_bytes(n, frame_cap))
    scratch = DeviceBuffer(sb)
    b = meta.ptr
    max_in = int(flen.max())

    def step():
        _lib.check(lib.kdb_get_values_batch(stream.ptr, batch.frames.ptr, b, b + 8 * n, b + 16 * n, b + 24 * n, n,
                                            batch.out.ptr, b + 32 * n, 0, b + 40 * n, b + 44 * n, frame_cap, max_in,
                                            size, scratch.ptr, sb, b + 48 * n, b + 56 * n), "kdb_get_values_batch")
    for _ in range(args.warmup):
        step()
    stream.sync()
    evs = [(K.Event(), K.Event()) for _ in range(args.steps)]
    barrier()
    sync_all()
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        step()
        evs[k][1].record(stream)
    stream.sync()
    sync_all()
    barrier()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine)
    g_ms = float(np.mean([e0.elapsed_ms(e1) for e0, e1 in evs]))
    res = meta.download(12 * n, 48 * n)
    olen, stat = res[:8 * n].view(np.uint64), res[8 * n:].view(np.int32)
    ok = bool((stat == 0).all() and np.array_equal(olen, sizes))
    if ok and not args.no_verify:
        t = batch.raw_bytes
        ok = bool(np.array_equal(batch.src.download(t), batch.out.download(t)))
    if not ok:
        raise SystemExit("bench: read path output is not bit-exact -- refusing to report a number")
    raw = float(batch.raw_bytes)
    frames = float(flen.sum())
    alg = raw + frames
    achieved = alg / (g_ms * 1e-3) / 1e9
    total_raw = max_over_ranks(raw, op="sum") * args.steps
    per_gpu = gather_ranks(raw * args.steps / mine / GIB)
    line = {
        "metric": "KingDB read path GiB/s (UncompressByteArray over stored values, device-resident)",
        "value": round(total_raw / elapsed / GIB, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: G1-long (db_bench CompressibleString 0.5, LevelDB Random(301)), stored as CompressorLZ4 "
                "frames by the GPU write path's compressor",
        "config": {"workload": f"configs[1] as a read: {n} x {size} B stored values per GPU -> values "
                               f"(frame walk + frame decode + status pass, verify off)",
                   "values_per_gpu": n, "value_bytes": size, "raw_bytes_per_gpu": int(raw),
                   "parallelism": f"dp{world} (independent shards, no collective)", "ratio": round(frames / raw, 4)},
        "roofline": {"bound": "hbm", "kernel": "kdb_get_values_batch (walk, scan, decode and finish launches)",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "alg_bytes_per_launch": int(alg), "avg_launch_ms": round(g_ms, 4)},
        "per_gpu_gibs": [round(x, 3) for x in per_gpu],
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ns = min(n, 65536)
        fo = batch.frame_off[:ns].astype(np.uint64)
        span = int(fo[-1] + flen[ns - 1])
        stored = batch.frames.download(span)
        line["cpu_baseline"] = ref_read_path(stored, fo, flen[:ns], size, args.cpu_seconds)
    for x in (meta, scratch):
        x.free()
    batch.free()
    if rank == 0:
        print(json.dumps(line), flush=True)


def bench_put(args, world: int, rank: int, local: int, barrier, sync_all) -> None:
    """configs[4]: the write path, host memory to HSTable bytes, PCIe included."""
    from kingdb_amd.lz4 import DeviceBuffer
    from kingdb_amd.putpipe import PutPipeline
    from kingdb_amd.shard import gather_ranks, max_over_ranks
    n, ks, vs = args.values, 16, 100
    pp = PutPipeline(n, ks, vs, chunk=args.put_chunk, nstreams=args.hi_streams, direct=not args.put_host_copy)
    base = rank * n                                   # this rank's slice of one global put sequence
    keys = np.frombuffer(b"".join(b"%016d" % (base + i) for i in range(n)), np.uint8).reshape(n, ks)
    pp.h_keys.np[:] = keys.reshape(-1)
    g = DeviceBuffer(n * vs + 64)
    from kingdb_amd import _lib
    from kingdb_amd import lz4 as L
    _lib.check(L.lib().kdb_lz4_gen_g1(g.ptr, base, n, 301, None), "gen_g1")   # 100-byte G1 pieces = values
    pp.h_vals.np[:] = g.download(n * vs)
    g.free()
    for _ in range(args.warmup):
        pp.run()
    times = []
    barrier()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        times.append(pp.run())
    sync_all()
    barrier()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine)
    per_gpu = gather_ranks(n * args.steps / mine)
    # what was timed: every put accepted, entries framed in order (spot-check the
    # first entries' keys and sizes; byte parity is tests/test_write_path.py's job)
    files = pp.writer.files()
    first = files[min(files)]
    pos, ok = 8192, True
    for i in range(min(n, 1000)):
        h = first[pos:pos + 64]
        # EntryHeader: crc8, fixed32, varint flags, varint size_key, varint size_value, fixed64 svc, varint pad, fixed64
        ok &= h[5] == 8 and h[6] == ks and h[7] == vs
        svc = int.from_bytes(h[8:16], "little")
        ok &= first[pos + 25:pos + 25 + ks] == keys[i].tobytes()
        pos += 25 + ks + (svc if svc else vs)
    if not ok:
        raise SystemExit("bench: write-path output malformed -- refusing to report a number")
    total = max_over_ranks(float(n), op="sum") * args.steps
    file_bytes = pp.writer.file_bytes()
    line = {
        "metric": "KingDB write path puts/s (16 B keys / 100 B values, pinned host memory -> HSTable bytes, PCIe "
                  "included)",
        "value": round(total / elapsed, 1), "unit": "puts/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: %016d keys, 100-byte G1 values (db_bench CompressibleString 0.5)",
        "config": {"workload": f"configs[4]: {n} puts per GPU through Database::PutPart semantics (frame policy, "
                               f"LZ4, CRC32C, xxHash-64, EntryHeader) into HSTable files, one writer per GPU",
                   "puts_per_gpu": n, "key_bytes": ks, "value_bytes": vs, "chunk": pp.chunk,
                   "streams": len(pp.streams), "entry_landing": "host copy" if args.put_host_copy else "direct DMA",
                   "parallelism": f"dp{world} (independent shards, no collective)"},
        "per_gpu_puts_per_s": [round(x, 1) for x in per_gpu],
        "mb_per_s_in": round(total * (ks + vs) / elapsed / 1e6, 1),
        "mb_per_s_out": round(file_bytes * max_over_ranks(1.0, op="sum") * args.steps / elapsed / 1e6, 1),
        "hstable_bytes_per_gpu": file_bytes, "files_per_gpu": len(files),
        "step_seconds": [round(t, 4) for t in times],
        "last_step_host_seconds": {k: round(v, 4) for k, v in pp.stats.items()},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = ref_write_path(keys, pp.h_vals.np.reshape(n, vs))
    pp.free()
    if rank == 0:
        print(json.dumps(line), flush=True)


def main() -> None:
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)

    # torch first (plumbing: gloo barrier / max-over-ranks, torch.cuda.synchronize):
    # loading it before libkdb_lz4.so keeps ONE HIP runtime in the process.
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    import kingdb_amd as K
    from kingdb_amd import lz4 as L
    from kingdb_amd.shard import g1_first_piece, gather_ranks, max_over_ranks

    # One rank per GPU.  More ranks than GPUs (a rehearsal of the N > 1 path on
    # a 1-GPU box) share devices round-robin; on a full node this is identity.
    n_dev = torch.cuda.device_count()
    if n_dev > 0 and local >= n_dev:
        print(f"warning: LOCAL_RANK={local} >= {n_dev} visible GPU(s): rank shares GPU "
              f"{local % n_dev} (rehearsal only)", file=sys.stderr)
        local = local % n_dev
    K.set_device(local)
    torch_sync = torch.cuda.is_available()
    if torch_sync:
        torch.cuda.set_device(local)

    def sync_all():
        L.lib().kdb_lz4_device_sync()
        if torch_sync:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    if args.workload in ("put", "get"):
        (bench_put if args.workload == "put" else bench_get)(args, world, rank, local, barrier, sync_all)
        if world > 1:
            dist.destroy_process_group()
        return

    n, size = args.values, args.size
    stream = K.Stream()
    if args.workload == "mixed":
        # configs[3]: one global mixed batch of n*world values, byte-balanced
        # contiguous shards; each rank generates its own slice.
        from kingdb_amd.shard import byte_balanced_ranges
        gsizes = L.mixed_sizes(n * world)
        lo, hi = byte_balanced_ranges(gsizes, world)[rank]
        before = int(gsizes[:lo].astype(np.int64).sum())
        batch = K.DeviceBatch.g1_long_sizes(gsizes[lo:hi], first_piece=(before + 99) // 100, stream=stream)
        n = batch.n
    else:
        first_piece = g1_first_piece(rank, n, size)  # rank's slice of one G1-long stream
        batch = K.DeviceBatch.g1_long(n, size, first_piece=first_piece, stream=stream)
    stream.sync()
    # the decoder is told the batch's largest frame (kdb_lz4_max_u32 on the
    # device + a 4-byte read back, inside every timed step), not the slot bound
    batch.exact_max_in = True

    for _ in range(args.warmup):
        batch.compress(stream)
        batch.decompress(stream)
    # every output of the passes poisoned after the warm-ups (outside the timed
    # region): the check after the loop then proves the timed steps wrote them
    batch.poison(stream)
    stream.sync()

    evs = [[K.Event() for _ in range(3)] for _ in range(args.steps)]
    barrier()
    sync_all()
    t0 = time.perf_counter()
    names = {}
    for k in range(args.steps):
        evs[k][0].record(stream)
        batch.compress(stream)
        if k == 0:
            names["compress"] = L.last_kernels()    # host-side record of what was queued, no HIP call
        evs[k][1].record(stream)
        batch.decompress(stream)
        if k == 0:
            names["decompress"] = L.last_kernels()
        evs[k][2].record(stream)
    stream.sync()
    sync_all()
    barrier()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine)

    c_ms = float(np.mean([evs[k][0].elapsed_ms(evs[k][1]) for k in range(args.steps)]))
    d_ms = float(np.mean([evs[k][1].elapsed_ms(evs[k][2]) for k in range(args.steps)]))

    # correctness of what was timed (outside the timed region)
    cst, dst = batch.status()
    flen = batch.frame_lens().astype(np.int64)
    ok = bool((cst == 0).all() and (dst == 0).all() and np.array_equal(batch.out_lens(), batch.sizes))
    if ok and not args.no_verify:
        ok = batch.roundtrip_ok()
    if not ok:
        raise SystemExit("bench: round trip is not bit-exact -- refusing to report a number")

    raw = float(batch.raw_bytes)
    frames = float(flen.sum())
    alg_bytes = raw + frames  # per launch, compress and decompress alike
    # the kernels the step's launches actually queued (kdb_lz4_last_kernels): a
    # mixed step has one launch per size class, covered by the roofline together
    kc = " + ".join(names["compress"])
    kd = " + ".join(names["decompress"])
    if c_ms >= d_ms:
        dom_key, dom_name, dom_ms = "compress", kc, c_ms
    else:
        dom_key, dom_name, dom_ms = "decompress", kd, d_ms
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    # HBM bytes of the same launch(es) from committed PMC passes of this exact
    # workload (tools/pmc_traffic.py); used only when the passes were taken with
    # this very build (kdb_lz4_build_id) and name the kernels this run queued
    traffic, traffic_source, traffic_refused = None, None, None
    pmc = args.pmc or os.path.join(ROOT, "profiles", {"mixed": "pmc_traffic_mixed.json",
                                                      "big": "pmc_traffic_big.json"}.get(args.workload,
                                                                                         "pmc_traffic.json"))
    try:
        pm = json.load(open(pmc))
        want = (args.values, "mixed") if args.workload == "mixed" else (n, size)
        got = pm["kernels"][dom_key]
        got_names = set(k.replace("kdb_lz4::", "") for k in (got.get("kernel") or "").split(" + "))
        if (pm.get("values"), pm.get("size")) != want or not (world == 1 or args.workload in ("uniform", "big")):
            traffic_refused = "no PMC passes of this workload"
        elif pm.get("build_id") != L.build_id():
            traffic_refused = (f"PMC passes taken with build {pm.get('build_id')}, this run uses {L.build_id()}")
        elif args.workload in ("uniform", "big") and not got_names <= set(names[dom_key]):
            traffic_refused = f"PMC kernel {sorted(got_names)} not among this run's {names[dom_key]}"
        elif args.workload == "mixed" and got_names != set(names[dom_key]):
            traffic_refused = f"PMC kernels {sorted(got_names)} differ from this run's {names[dom_key]}"
        else:
            traffic = got["hbm_bytes_per_launch"]
            traffic_source = {"file": os.path.relpath(pmc, ROOT), "passes": pm.get("passes"),
                              "build_id": pm.get("build_id"),
                              "scope": pm.get("scope", "the kind's dominant launch"),
                              "correction": got.get("correction"),
                              "traffic_undoubled": got.get("hbm_bytes_per_launch_undoubled")}
    except (OSError, ValueError, KeyError) as e:
        traffic_refused = f"no usable PMC summary ({type(e).__name__})"

    total_raw = max_over_ranks(raw, op="sum") * args.steps
    value = total_raw / elapsed / GIB
    per_gpu = gather_ranks(raw * args.steps / mine / GIB)
    copy_gbs = copy_bandwidth(batch, stream)
    line = {
        "metric": METRIC if args.workload != "big" else METRIC_BIG,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: G1-long (db_bench CompressibleString 0.5, LevelDB Random(301)), generated on device",
        "config": {
            "workload": (f"{n} x {size} B values per GPU: CompressorLZ4 frame compress + frame decompress (round trip)"
                         if args.workload == "uniform" else
                         f"KingDB's default part size (util/options.h:171-172): {n} x {size} B parts per GPU, "
                         f"byU32 blocks (lz4.cc:673-676): CompressorLZ4 frame compress + frame decompress (round trip)"
                         if args.workload == "big" else
                         f"configs[3] mixed batch, {n} values on rank 0 (by count 90% 100 B / 9% 4 KiB / 1% 64 KiB "
                         f"parts, {args.values * world} values byte-balanced over {world} GPU(s)): frame compress + "
                         f"frame decompress (round trip)"),
            "values_per_gpu": n, "value_bytes": size if args.workload in ("uniform", "big") else "mixed",
            "raw_bytes_per_gpu": int(raw),
            "parallelism": f"dp{world} (independent shards, no collective)",
            "ratio": round(frames / raw, 4),
            "decompress_max_in": "largest frame of the batch, reduced on the device inside each step",
        },
        "roofline": {
            "bound": "hbm", "kernel": dom_name,
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": traffic_source,
            "traffic_refused": traffic_refused, "build_id": L.build_id(),
            "alg_bytes_per_launch": int(alg_bytes), "avg_launch_ms": round(dom_ms, 4),
            "copy_gbs": round(copy_gbs, 1), "frac_of_copy": round(achieved / copy_gbs, 5),
        },
        "per_gpu_gibs": [round(x, 3) for x in per_gpu],
        "kernels_ms": {"compress": round(c_ms, 4), "decompress": round(d_ms, 4)},
        "compress_gibs": round(raw / (c_ms * 1e-3) / GIB, 2),
        "decompress_gibs": round(raw / (d_ms * 1e-3) / GIB, 2),
        "cpu_baseline": None,
    }
    line["verify"] = ("every decoded byte and status checked after the timed steps; frames, decoded bytes, "
                      "lengths and status words were poisoned before them" if not args.no_verify else
                      "statuses and lengths only (poisoned before the timed steps)")
    if not args.no_host_inclusive and args.workload == "uniform" and world == 1:
        line["host_inclusive"] = host_inclusive(batch, n, size, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload in ("uniform", "big"):
        ncpu = min(n, 131072, max(1, (1 << 30) // size))   # at most 1 GiB of the batch
        sample = batch.src.download(ncpu * size)
        line["cpu_baseline"] = cpu_baseline(sample, size, args.cpu_seconds)
        if args.workload == "uniform":
            line["configs0_compressor_100b"] = compressor_calls_100b()
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "mixed":
        # a prefix of the same batch, about 512 MiB of raw bytes
        lens = batch.sizes
        m = int(np.searchsorted(np.cumsum(lens.astype(np.int64)), 512 << 20)) + 1
        m = min(m, n)
        nbytes = int(batch.src_off[m - 1]) + int(lens[m - 1])
        sample = batch.src.download(nbytes)
        line["cpu_baseline"] = cpu_baseline_mixed(sample, batch.src_off[:m], lens[:m], args.cpu_seconds)
    batch.free()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
