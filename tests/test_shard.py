"""CPU: the multi-GPU sharding host logic -- byte-balanced
contiguous ranges, multipart groups kept on one rank, host stitching by prefix
sum, max-over-ranks timing -- including a world_size-2 gloo run in which each
rank encodes only its own shard (oracle as the stand-in codec: this test
covers the partitioning, not the kernels) and the stitched stream must equal
the single-rank stream."""
import os
import socket

import numpy as np
import pytest

from kingdb_amd.shard import byte_balanced_ranges, g1_first_piece, gather_ranks, max_over_ranks, stitch_offsets


def test_ranges_cover_and_balance():
    rng = np.random.default_rng(5)
    sizes = rng.choice([100, 4096, 65536], size=5000, p=[0.9, 0.09, 0.01])
    for world in (1, 2, 4, 8):
        r = byte_balanced_ranges(sizes, world)
        assert r[0][0] == 0 and r[-1][1] == len(sizes)
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        per = [int(sizes[lo:hi].sum()) for lo, hi in r]
        assert max(per) - min(per) <= 2 * 65536


def test_groups_stay_together():
    # values split into 64 KiB parts; a part group must never straddle ranks
    parts, groups = [], []
    rng = np.random.default_rng(9)
    for v in range(300):
        s = int(rng.integers(1, 300000))
        while s > 0:
            parts.append(min(s, 65536))
            groups.append(v)
            s -= 65536
    groups = np.array(groups)
    for world in (2, 3, 8):
        for lo, hi in byte_balanced_ranges(parts, world, groups):
            if lo < hi and lo > 0:
                assert groups[lo] != groups[lo - 1]
    with pytest.raises(ValueError):
        byte_balanced_ranges([1, 2, 3], 2, groups=[1, 0, 0])


def test_edge_cases():
    assert byte_balanced_ranges([], 3) == [(0, 0)] * 3
    assert byte_balanced_ranges([7], 2) in ([(0, 1), (1, 1)], [(0, 0), (0, 1)])
    assert list(stitch_offsets([10, 0, 5])) == [0, 10, 10]
    assert g1_first_piece(0, 1 << 20, 4096) == 0
    assert g1_first_piece(3, 1000, 4096) == 3 * 40960
    assert max_over_ranks(1.5) == 1.5  # no process group
    assert gather_ranks(2.5) == [2.5]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist

    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = oracle.Oracle()
    pool = oracle.g1_pool(orc)
    values = oracle.g1_values(pool, 100, 300) + oracle.g1_values(pool, 4096, 30) + [bytes(5000), b""]
    lo, hi = byte_balanced_ranges([len(v) for v in values], world)[rank]
    mine = b"".join(orc.frame(v) for v in values[lo:hi])
    # what the host does after the fact: per-device byte totals -> offsets
    totals = [None] * world
    dist.all_gather_object(totals, len(mine))
    off = int(stitch_offsets(totals)[rank])
    elapsed = max_over_ranks(0.25 * (rank + 1))
    assert gather_ranks(10.0 + rank) == [10.0 + r for r in range(world)]
    assert max_over_ranks(float(hi - lo), op="sum") == len(values)
    with open(os.path.join(out_dir, f"rank{rank}.bin"), "wb") as f:
        f.write(mine)
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{off} {elapsed} {lo} {hi}")
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_stitch(tmp_path, orc):
    import torch.multiprocessing as mp

    import oracle
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    pool = oracle.g1_pool(orc)
    values = oracle.g1_values(pool, 100, 300) + oracle.g1_values(pool, 4096, 30) + [bytes(5000), b""]
    whole = b"".join(orc.frame(v) for v in values)
    stitched = bytearray(len(whole))
    spans = []
    for r in range(world):
        off, elapsed, lo, hi = (tmp_path / f"rank{r}.txt").read_text().split()
        data = (tmp_path / f"rank{r}.bin").read_bytes()
        stitched[int(off):int(off) + len(data)] = data
        spans.append((int(lo), int(hi)))
        assert float(elapsed) == 0.25 * world  # max over ranks
    assert bytes(stitched) == whole
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == len(values)
    assert 0 < spans[0][1] < len(values)


# ------------------------------------------------------------------ GPU
def _gpu_worker(rank, world, port, out_dir):
    """One rank per device (round-robin onto the visible GPUs, as bench.py maps
    ranks): the rank's shard goes through the HIP codec."""
    import torch.distributed as dist

    import kingdb_amd as K
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    want = rank % K.device_count()
    K.set_device(want)
    bound = [K.get_device()]           # the device this rank asked for, as the library sees it
    orc = oracle.Oracle()
    pool = oracle.g1_pool(orc)
    values = oracle.g1_values(pool, 100, 3000) + oracle.g1_values(pool, 4096, 300) + \
        oracle.g1_values(pool, 65536, 8) + [bytes(5000), b"", bytes(range(256)) * 300]
    lo, hi = byte_balanced_ranges([len(v) for v in values], world)[rank]
    frames = K.compress_frames(values[lo:hi])
    back = K.decompress_frames(frames, [len(v) for v in values[lo:hi]])
    bound.append(K.get_device())       # and still bound after the batches
    ok = all(st == 0 and out == v for (st, out), v in zip(back, values[lo:hi]))
    mine = b"".join(frames)
    totals = [None] * world
    dist.all_gather_object(totals, len(mine))
    off = int(stitch_offsets(totals)[rank])
    with open(os.path.join(out_dir, f"rank{rank}.bin"), "wb") as f:
        f.write(mine)
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{off} {int(ok)} {lo} {hi} {want} {bound[0]} {bound[1]}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_world2_ranks_stitch_to_reference_stream(tmp_path, gpu, orc):
    """world_size 2, each rank compressing (and round-tripping) its byte-balanced
    shard on its own device: the stitched frame stream equals the oracle's
    stream of the whole batch."""
    import torch.multiprocessing as mp

    import oracle
    world = 2
    mp.spawn(_gpu_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    pool = oracle.g1_pool(orc)
    values = oracle.g1_values(pool, 100, 3000) + oracle.g1_values(pool, 4096, 300) + \
        oracle.g1_values(pool, 65536, 8) + [bytes(5000), b"", bytes(range(256)) * 300]
    whole = b"".join(orc.frame(v) for v in values)
    stitched = bytearray(len(whole))
    for r in range(world):
        off, ok, lo, hi, want, b0, b1 = (tmp_path / f"rank{r}.txt").read_text().split()
        assert ok == "1", f"rank {r} round trip"
        assert want == b0 == b1, f"rank {r} asked for device {want}, kdb_lz4_get_device said {b0} then {b1}"
        data = (tmp_path / f"rank{r}.bin").read_bytes()
        stitched[int(off):int(off) + len(data)] = data
    assert bytes(stitched) == whole


@pytest.mark.gpu
def test_gpu_host_threads_share_the_library(gpu, orc):
    """INTEGRATION.md's in-process model: one host thread per device (here 4
    threads round-robin on the visible devices), each with its own batches and
    scalar calls at once -- per-thread streams, staging and fork streams."""
    import threading

    import kingdb_amd as K
    import oracle
    pool = oracle.g1_pool(orc)
    errs = []

    def work(t):
        try:
            want = t % K.device_count()
            K.set_device(want)
            if K.get_device() != want:
                errs.append((t, "bound device", K.get_device(), want))
            vals = oracle.g1_values(pool, 100 + 997 * t, 400) + [bytes(range(256)) * (t + 1)]
            for _ in range(3):
                fr = K.compress_frames(vals)
                if fr != [orc.frame(v) for v in vals]:
                    errs.append((t, "frames"))
                back = K.decompress_frames(fr, [len(v) for v in vals])
                if any(st != 0 or out != v for (st, out), v in zip(back, vals)):
                    errs.append((t, "round trip"))
                for v in vals[:20]:
                    r, blk = K.compress_limited_output(v, K.compress_bound(len(v)))
                    if blk != orc.compress(v):
                        errs.append((t, "scalar"))
            if K.get_device() != want:
                errs.append((t, "device after calls", K.get_device(), want))
        except Exception as e:  # noqa: BLE001
            errs.append((t, repr(e)))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert errs == []
