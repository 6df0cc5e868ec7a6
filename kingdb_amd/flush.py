"""The write-buffer flush batch (include/kdb_flush.h).

Python face of kdb_flush_parts_batch, with the same batch layout the KingDB
hook builds (kingdb_amd/csrc/flush_hook.cc, Pipeline::gpu_batch):

  flush_parts(calls, states)   one GPU batch of PutPartValidSize calls
      calls   [(tid, key, chunk, offset_chunk, size_value)] in call order
      states  {tid: FlushState} carried in (missing: the ThreadStorage defaults)
  -> ([{"rc", "mode", "occ", "chunk_final", "svc", "crc"}], states after the batch)

The CPU side only lays the batch out (segments: one thread's consecutive
parts of one value; runs: segments whose policy state chains); every frame,
policy decision and CRC comes from the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .lz4 import DeviceBuffer

FRAME, DISABLED, RAW, FAILED = 0, 1, 2, 3
_last: dict = {}   # the last batch's raw outputs (diagnostics)


class FlushState(ctypes.Structure):
    """kdb_flush_state: one client thread's PutPartValidSize state."""
    _fields_ = [("ts_offset", ctypes.c_uint64), ("comp_total", ctypes.c_uint64), ("enabled", ctypes.c_uint32),
                ("crc", ctypes.c_uint32)]


class FlushPart(ctypes.Structure):
    """kdb_flush_part."""
    _fields_ = [("occ", ctypes.c_uint64), ("svc", ctypes.c_uint64), ("frame_at", ctypes.c_uint64),
                ("size", ctypes.c_uint32), ("crc", ctypes.c_uint32), ("mode", ctypes.c_uint32),
                ("status", ctypes.c_int32)]


def lib():
    return _lib.load()


def _a256(x: int) -> int:
    return (x + 255) & ~255


def layout(calls):
    """Segments and runs (flush_hook.cc's rules): (perm, seg_first, run_first,
    seg_head, run_tid, run_seen) -- perm[q] = the call at batch position q."""
    cur = {}
    part_seg, seg_run, seg_head, run_tid, run_seen = [], [], [], [], []
    for i, (tid, _k, chunk, off, _v) in enumerate(calls):
        fresh = off == 0
        if tid not in cur or (fresh and len(chunk) > 0):
            seen = tid in cur
            r = len(run_tid)
            run_tid.append(tid)
            run_seen.append(seen)
            s = len(seg_run)
            seg_run.append(r)
            seg_head.append(i)
            cur[tid] = [r, s]
            part_seg.append(s)
        elif fresh:
            s = len(seg_run)
            seg_run.append(cur[tid][0])
            seg_head.append(i)
            cur[tid][1] = s
            part_seg.append(s)
        else:
            part_seg.append(cur[tid][1])
    nseg, nruns = len(seg_run), len(run_tid)
    seg_order = sorted(range(nseg), key=lambda s: (seg_run[s], s))
    seg_pos = [0] * nseg
    for at, s in enumerate(seg_order):
        seg_pos[s] = at
    perm = sorted(range(len(calls)), key=lambda i: (seg_pos[part_seg[i]], i))
    seg_first = [0] * (nseg + 1)
    for i in range(len(calls)):
        seg_first[seg_pos[part_seg[i]] + 1] += 1
    run_first = [0] * (nruns + 1)
    for s in range(nseg):
        run_first[seg_run[s] + 1] += 1
    seg_first = np.cumsum(seg_first).astype(np.uint32)
    run_first = np.cumsum(run_first).astype(np.uint32)
    return perm, seg_first, run_first, [seg_head[s] for s in seg_order], run_tid, run_seen


def flush_parts(calls, states=None):
    states = dict(states or {})
    m = len(calls)
    if m == 0:
        return [], states
    perm, seg_first, run_first, heads, run_tid, run_seen = layout(calls)
    nseg, nruns = len(heads), len(run_tid)
    keys = [calls[h][1] for h in heads]
    chunks = [calls[i][2] for i in perm]
    key_len = np.array([len(k) for k in keys], np.uint32)
    key_off = np.zeros(nseg, np.uint64)
    key_off[1:] = np.cumsum(key_len[:-1].astype(np.uint64))
    chunk_len = np.array([len(c) for c in chunks], np.uint32)
    chunk_off = np.zeros(m, np.uint64)
    chunk_off[1:] = np.cumsum(chunk_len[:-1].astype(np.uint64))
    offset = np.array([calls[i][3] for i in perm], np.uint64)
    size = np.array([calls[i][4] for i in perm], np.uint64)
    carry = (FlushState * nruns)()
    for r, (tid, seen) in enumerate(zip(run_tid, run_seen)):
        if not seen and tid in states:
            carry[r] = states[tid]
    raw = int(chunk_len.sum())
    kb = b"".join(keys)
    cb = b"".join(chunks)
    # device inputs, one buffer: arrays then bytes
    parts_in = [key_off.view(np.uint8), key_len.view(np.uint8), chunk_off.view(np.uint8), chunk_len.view(np.uint8),
                offset.view(np.uint8), size.view(np.uint8), seg_first.view(np.uint8), run_first.view(np.uint8),
                np.frombuffer(bytes(carry), np.uint8), np.frombuffer(kb, np.uint8), np.frombuffer(cb, np.uint8)]
    offs, at = [], 0
    for a in parts_in:
        offs.append(at)
        at = _a256(at + a.nbytes + 64)
    host = np.zeros(at, np.uint8)
    for o, a in zip(offs, parts_in):
        host[o:o + a.nbytes] = a
    d_in = DeviceBuffer(at)
    d_in.upload(host)
    scratch = int(lib().kdb_flush_scratch_bytes(m, nseg, raw))
    d_scratch = DeviceBuffer(scratch)
    frame_cap = sum(((8 + len(c) + len(c) // 255 + 16) + 15) & ~15 for c in chunks) + 64
    o_parts, o_carry = 0, _a256(ctypes.sizeof(FlushPart) * m)
    o_total = o_carry + _a256(ctypes.sizeof(FlushState) * nruns)
    d_out = DeviceBuffer(o_total + 256)
    d_frames = DeviceBuffer(frame_cap)
    b = d_in.ptr
    _lib.check(lib().kdb_flush_parts_batch(
        None, b + offs[9], b + offs[0], b + offs[1], b + offs[10], b + offs[2], b + offs[3], b + offs[4],
        b + offs[5], b + offs[6], b + offs[7], b + offs[8], m, nseg, nruns, int(chunk_len.max()), d_scratch.ptr,
        scratch, raw, d_out.ptr + o_parts, d_out.ptr + o_carry, d_frames.ptr, d_out.ptr + o_total),
        "kdb_flush_parts_batch")
    out = d_out.download()
    frames = d_frames.download()
    parts = (FlushPart * m).from_buffer_copy(out[o_parts:o_parts + ctypes.sizeof(FlushPart) * m].tobytes())
    couts = (FlushState * nruns).from_buffer_copy(
        out[o_carry:o_carry + ctypes.sizeof(FlushState) * nruns].tobytes())
    total = int(out[o_total:o_total + 8].view(np.uint64)[0])
    _last.update(parts=parts, frames=frames, total=total, perm=perm, chunks=chunks)
    res = [None] * m
    for q, i in enumerate(perm):
        P = parts[q]
        if P.mode == FRAME:
            assert P.frame_at + P.size <= total
            fin = frames[P.frame_at:P.frame_at + P.size].tobytes()
        elif P.mode == DISABLED:
            fin = bytes(8) + chunks[q]
        elif P.mode == RAW:
            fin = chunks[q]
        else:
            fin = b""
        res[i] = {"rc": 0 if P.status == 0 else -1, "mode": int(P.mode), "occ": int(P.occ), "chunk_final": fin,
                  "svc": int(P.svc), "crc": int(P.crc)}
    for r, tid in enumerate(run_tid):
        s = FlushState()
        ctypes.memmove(ctypes.byref(s), ctypes.byref(couts[r]), ctypes.sizeof(FlushState))
        states[tid] = s
    return res, states
