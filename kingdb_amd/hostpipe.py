"""Host-inclusive pipeline: values in pinned host memory -> frames in pinned
host memory and back, with the H2D copy, the kernels and the D2H copy
overlapped over several HIP streams.

This is the shape the north star asks to be measured beside the
device-resident number: KingDB's path starts and ends in host memory -- the
write buffer (cache/write_buffer.cc:228-319) on the way in, the mmap'd HSTable
files (storage/hstable_manager.h:656-673) on the way back -- so a GPU codec
pays PCIe both ways.  Per chunk of values:

  compress:   H2D raw bytes + per-value metadata  ->  frame kernel into slots
              ->  pack kernel (dense frame stream, pack.hip)  ->  D2H of the
              chunk's frame total (8 B)  ...  D2H of exactly ΣF frame bytes
              + frame lengths/status, to the running host offset
  decompress: H2D packed frames + per-value (offset, length) -> frame
              decompress kernel -> D2H raw bytes

The D2H of a compressed chunk needs its byte count, so the host waits for
chunk c-depth's pack while chunks c-depth+1 .. c are already queued (depth =
number of streams); the copies of later chunks keep the link busy meanwhile.
Device-to-host copies run on streams of their own (behind an event of the
chunk's kernels), so they overlap the host-to-device copies of later chunks:
PCIe carries both directions at once (the link alone: ~57 GB/s one way, ~88
GB/s both ways), and on one stream per chunk a D2H held up the next chunk's
H2D queued behind it (round 2: the two directions' busy times added up).
All timing is host wall clock from the first enqueue to the last byte landing
in host memory.  Nothing here computes LZ4 on the CPU.
"""
from __future__ import annotations

import ctypes
import time

import numpy as np

from . import _lib
from .lz4 import DeviceBuffer, Event, Stream, frame_bound, lib


def _union(ivs) -> float:
    """Total length of the union of [a, b) intervals."""
    tot, end = 0.0, None
    for a, b in sorted(ivs):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


class PinnedBuffer:
    """hipHostMalloc'd bytes with a numpy view."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _lib.check(lib().kdb_lz4_host_alloc(ctypes.byref(p), max(self.nbytes, 1)), "host_alloc")
        self.ptr = p.value
        self.np = np.ctypeslib.as_array((ctypes.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))

    def free(self) -> None:
        if self.ptr:
            self.np = None
            lib().kdb_lz4_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostPipeline:
    """n equal-size values of `size` bytes, processed in chunks of `chunk`
    values over `nstreams` streams."""

    def __init__(self, n: int, size: int, chunk: int = 1 << 16, nstreams: int = 4, cdrain: int = 4,
                 ddrain: int = 4):
        self.n, self.size = int(n), int(size)
        self.chunk = max(1, min(int(chunk), self.n))
        self.nchunks = (self.n + self.chunk - 1) // self.chunk
        self.slot = (frame_bound(size) + 15) & ~15
        n = self.n
        self.streams = [Stream() for _ in range(max(1, nstreams))]
        # device-to-host copies: compress drains over `cdrain` streams, decompress
        # over `ddrain` (profiles/r03_n10_hostpipe.txt: 4 and 4 measured best,
        # 19.7 GiB/s round trip; 1 and 1: 17.4)
        self.dstreams = [Stream() for _ in range(max(1, nstreams, cdrain, ddrain))]
        self.cdrain, self.ddrain = max(1, cdrain), max(1, ddrain)
        # Serial copies (round 6, the default): each phase's host-to-device
        # copies in chunk order on a stream of their own, the decode's
        # device-to-host copies likewise, and no copy stream ever carries the
        # other direction.  Measured on MI355X (tools/hostpipe_probe.py,
        # profiles/r06/r06_e_hostprobe.json): compress 99-110 -> 88.6 ms,
        # decompress 108-121 -> 85.8 ms (its floor is 4.3 GB of D2H at
        # 57 GB/s, ~75 ms).  The per-chunk streams of round 3 left the 4 + 4
        # copy queues of each direction contending, and a decompress that
        # reused streams the compress had copied the other way on ran at
        # 124 ms.
        self.dserial = True
        self.cserial = True
        self.dup, self.ddown, self.cup = Stream(), Stream(), Stream()
        # host side (pinned): raw values, packed frames, decoded values, metadata
        self.h_raw = PinnedBuffer(n * size)
        self.h_frames = PinnedBuffer(n * self.slot)
        self.h_out = PinnedBuffer(n * size)
        self.h_cmeta = PinnedBuffer(n * 20)       # src_off u64 | len u32 | slot_off u64
        self.h_cres = PinnedBuffer(n * 8)         # frame_len u32 | status i32
        self.h_dmeta = PinnedBuffer(n * 12)       # frame_off u64 | avail u32
        self.h_dres = PinnedBuffer(n * 8)         # out_len u32 | status i32
        self.h_tot = PinnedBuffer(self.nchunks * 8)
        # device side
        self.d_raw = DeviceBuffer(n * size + 64)
        self.d_slots = DeviceBuffer(n * self.slot + 64)
        self.d_packed = DeviceBuffer(n * self.slot + 64)
        self.d_out = DeviceBuffer(n * size + 64)
        self.d_cmeta = DeviceBuffer(n * 20)
        self.d_cres = DeviceBuffer(n * 8)
        self.d_pack_off = DeviceBuffer(n * 8)
        self.d_tot = DeviceBuffer(self.nchunks * 8)
        self.d_dmeta = DeviceBuffer(n * 12)
        self.d_dconst = DeviceBuffer(n * 12)     # out_off u64 | out_cap u32 (caller's output layout)
        self.d_dres = DeviceBuffer(n * 8)
        idx = np.arange(n, dtype=np.uint64)
        cm = self.h_cmeta.np
        cm[: 8 * n] = (idx * np.uint64(size)).view(np.uint8)
        cm[8 * n: 12 * n] = np.full(n, size, np.uint32).view(np.uint8)
        cm[12 * n: 20 * n] = (idx * np.uint64(self.slot)).view(np.uint8)
        dc = np.concatenate([(idx * np.uint64(size)).view(np.uint8), np.full(n, size, np.uint32).view(np.uint8)])
        self.d_dconst.upload(dc)
        self.frame_bytes = 0
        self.frame_off = np.zeros(n + 1, np.uint64)
        self._trace = None        # [(kind, chunk, start Event, end Event)] while profile() runs
        self._pool = []           # events for the traced runs, made before them
        self._kinds = None        # the span kinds traced (None: all)
        self._base = None         # the traced run's time origin

    def _mark(self, st, kind: str = "") -> "Event | None":
        if self._trace is None or (kind and self._kinds is not None and kind not in self._kinds):
            return None
        # from a pool made before the traced run: creating events inside it
        # delayed the compress loop's enqueues behind its host waits (traced
        # compress 114 ms against 90 timed, profiles/r06/r06_g_bench.json)
        e = self._pool.pop() if self._pool else Event()
        e.record(st)
        return e

    def _span(self, kind: str, c: int, e0, st) -> None:
        if self._trace is not None and e0 is not None:
            self._trace.append((kind, c, e0, self._mark(st)))

    def _range(self, c: int) -> tuple[int, int]:
        lo = c * self.chunk
        return lo, min(lo + self.chunk, self.n)

    def compress(self) -> float:
        """Host raw values -> packed host frames.  Returns wall seconds."""
        L = lib()
        n, size = self.n, self.size
        S = len(self.streams)
        done = [Event() for _ in range(self.nchunks)]
        host_off = 0
        chunk_off = np.zeros(self.nchunks + 1, np.uint64)

        def drain(c: int) -> None:
            nonlocal host_off
            lo, hi = self._range(c)
            ds = self.dstreams[c % self.cdrain]
            _lib.check(L.kdb_lz4_event_sync(done[c].ptr), "event_sync")
            tot = int(self.h_tot.np[8 * c: 8 * c + 8].view(np.uint64)[0])
            e0 = None if serial else self._mark(ds, "d2h")
            _lib.check(L.kdb_lz4_memcpy_d2h(self.h_frames.ptr + host_off, self.d_packed.ptr + lo * self.slot,
                                            tot, ds.ptr), "d2h frames")
            self._span("d2h", c, e0, ds)
            if serial and tracing("d2h"):
                dend[c] = self._mark(ds)
            chunk_off[c] = host_off
            host_off += tot

        serial = self.cserial
        hdone = [Event() for _ in range(self.nchunks)] if serial else None
        dend = [None] * self.nchunks       # (serial, traced) each frames copy's end

        def tracing(kind: str) -> bool:
            return self._trace is not None and (self._kinds is None or kind in self._kinds)
        t0 = time.perf_counter()
        for c in range(self.nchunks):
            lo, hi = self._range(c)
            m = hi - lo
            st = self.streams[c % S].ptr
            cm, dm = self.h_cmeta.ptr, self.d_cmeta.ptr
            hs = self.cup if serial else self.streams[c % S]   # the stream of the chunk's host-to-device copies
            # (serial: traced by the hdone events the run records anyway -- event
            # records between these copies slowed the compress 88.6 -> 96.9 ms,
            # profiles/r06/r06_k_trace_ab.json)
            e0 = None if serial else self._mark(hs, "h2d")
            for base, w in ((0, 8), (8 * n, 4), (12 * n, 8)):
                _lib.check(L.kdb_lz4_memcpy_h2d(dm + base + w * lo, cm + base + w * lo, w * m, hs.ptr), "h2d meta")
            _lib.check(L.kdb_lz4_memcpy_h2d(self.d_raw.ptr + lo * size, self.h_raw.ptr + lo * size, m * size, hs.ptr),
                       "h2d raw")
            self._span("h2d", c, e0, hs)
            if serial:
                hdone[c].record(self.cup)
                _lib.check(L.kdb_lz4_stream_wait_event(st, hdone[c].ptr), "stream_wait_event")
            e0 = None if serial else self._mark(self.streams[c % S], "kernel")
            flen = self.d_cres.ptr + 4 * lo
            stat = self.d_cres.ptr + 4 * n + 4 * lo
            _lib.check(L.kdb_lz4_compress_frames_batch(
                st, self.d_raw.ptr, dm + 8 * lo, dm + 8 * n + 4 * lo, m, size, self.d_slots.ptr,
                dm + 12 * n + 8 * lo, flen, stat), "compress_frames_batch")
            _lib.check(L.kdb_lz4_pack_frames(
                st, self.d_slots.ptr, dm + 12 * n + 8 * lo, flen, m, self.d_packed.ptr + lo * self.slot,
                self.d_pack_off.ptr + 8 * lo, self.d_tot.ptr + 8 * c), "pack_frames")
            self._span("kernel", c, e0, self.streams[c % S])
            _lib.check(L.kdb_lz4_memcpy_d2h(self.h_tot.ptr + 8 * c, self.d_tot.ptr + 8 * c, 8, st), "d2h total")
            done[c].record(self.streams[c % S])
            ds = self.dstreams[c % self.cdrain].ptr
            _lib.check(L.kdb_lz4_stream_wait_event(ds, done[c].ptr), "stream_wait_event")
            for base in (4 * lo, 4 * n + 4 * lo):
                _lib.check(L.kdb_lz4_memcpy_d2h(self.h_cres.ptr + base, self.d_cres.ptr + base, 4 * m, ds),
                           "d2h results")
            if c >= S - 1:
                drain(c - (S - 1))
        for c in range(max(0, self.nchunks - (S - 1)), self.nchunks):
            drain(c)
        for s in self.streams + self.dstreams + [self.cup]:
            s.sync()
        if serial and self._trace is not None:
            # Serial mode is traced with the events the run records anyway, plus
            # one at the end of each frames copy: event records between the
            # copies slowed the compress (88.6 -> 96.9 ms with records around
            # every H2D span, profiles/r06/r06_k_trace_ab.json).  A span starts
            # at the latest event its stream had to wait for:
            #   h2d    (the one copy stream, back to back): the previous chunk's hdone;
            #   kernel (stream c % S): its chunk's hdone and that stream's previous chunk's done;
            #   d2h    (dstream c % cdrain): its chunk's done and that stream's previous frames copy.
            base = self._base
            for c in range(self.nchunks):
                if tracing("h2d"):
                    self._trace.append(("h2d", c, hdone[c - 1] if c else base, hdone[c]))
                if tracing("kernel"):
                    self._trace.append(("kernel", c, [hdone[c]] + ([done[c - S]] if c >= S else []), done[c]))
                if tracing("d2h") and dend[c] is not None:
                    prev = c - self.cdrain
                    self._trace.append(("d2h", c, [done[c]] + ([dend[prev]] if prev >= 0 else []), dend[c]))
        t = time.perf_counter() - t0
        self.frame_bytes = host_off
        flen = self.h_cres.np[: 4 * n].view(np.uint32).astype(np.uint64)
        self.frame_off[1:] = np.cumsum(flen)
        chunk_off[self.nchunks] = host_off
        if int(self.frame_off[-1]) != host_off:
            raise RuntimeError("pack totals disagree with frame lengths")
        return t

    def status(self) -> tuple[np.ndarray, np.ndarray]:
        n = self.n
        return (self.h_cres.np[4 * n: 8 * n].view(np.int32), self.h_dres.np[4 * n: 8 * n].view(np.int32))

    def frames(self) -> bytes:
        return self.h_frames.np[: self.frame_bytes].tobytes()

    def decompress(self, serial: bool | None = None) -> float:
        """Packed host frames (as produced by compress()) -> host raw values.

        serial (default: self.dserial): every chunk's host-to-device copies on
        one stream, in chunk order, and every device-to-host copy on another,
        each chunk's decode on a compute stream between them (events): the two
        directions then stream side by side, each in order, instead of 4 + 4
        copy queues contending in each direction."""
        if serial is None:
            serial = self.dserial
        if serial:
            return self._decompress_serial()
        L = lib()
        n, size = self.n, self.size
        S = len(self.streams)
        dm = self.h_dmeta.np
        dm[: 8 * n] = self.frame_off[:n].view(np.uint8)
        dm[8 * n: 12 * n] = np.diff(self.frame_off).astype(np.uint32).view(np.uint8)
        max_in = int(np.diff(self.frame_off).max()) if n else 0
        kdone = [Event() for _ in range(self.nchunks)]
        t0 = time.perf_counter()
        for c in range(self.nchunks):
            lo, hi = self._range(c)
            m = hi - lo
            st = self.streams[c % S].ptr
            f0, f1 = int(self.frame_off[lo]), int(self.frame_off[hi])
            e0 = self._mark(self.streams[c % S], "h2d")
            _lib.check(L.kdb_lz4_memcpy_h2d(self.d_packed.ptr + f0, self.h_frames.ptr + f0, f1 - f0, st), "h2d frames")
            for base, w in ((0, 8), (8 * n, 4)):
                _lib.check(L.kdb_lz4_memcpy_h2d(self.d_dmeta.ptr + base + w * lo, self.h_dmeta.ptr + base + w * lo,
                                                w * m, st), "h2d meta")
            self._span("h2d", c, e0, self.streams[c % S])
            e0 = self._mark(self.streams[c % S], "kernel")
            olen = self.d_dres.ptr + 4 * lo
            stat = self.d_dres.ptr + 4 * n + 4 * lo
            _lib.check(L.kdb_lz4_decompress_frames_batch(
                st, self.d_packed.ptr, self.d_dmeta.ptr + 8 * lo, self.d_dmeta.ptr + 8 * n + 4 * lo, m, max_in, size,
                self.d_out.ptr, self.d_dconst.ptr + 8 * lo, self.d_dconst.ptr + 8 * n + 4 * lo, olen, stat),
                "decompress_frames_batch")
            self._span("kernel", c, e0, self.streams[c % S])
            kdone[c].record(self.streams[c % S])
            ds = self.dstreams[c % self.ddrain]
            _lib.check(L.kdb_lz4_stream_wait_event(ds.ptr, kdone[c].ptr), "stream_wait_event")
            e0 = self._mark(ds, "d2h")
            _lib.check(L.kdb_lz4_memcpy_d2h(self.h_out.ptr + lo * size, self.d_out.ptr + lo * size, m * size,
                                            ds.ptr), "d2h out")
            self._span("d2h", c, e0, ds)
            for base in (4 * lo, 4 * n + 4 * lo):
                _lib.check(L.kdb_lz4_memcpy_d2h(self.h_dres.ptr + base, self.d_dres.ptr + base, 4 * m, ds.ptr),
                           "d2h results")
        for s in self.streams + self.dstreams:
            s.sync()
        return time.perf_counter() - t0

    def _decompress_serial(self) -> float:
        L = lib()
        n, size = self.n, self.size
        S = len(self.streams)
        dm = self.h_dmeta.np
        dm[: 8 * n] = self.frame_off[:n].view(np.uint8)
        dm[8 * n: 12 * n] = np.diff(self.frame_off).astype(np.uint32).view(np.uint8)
        max_in = int(np.diff(self.frame_off).max()) if n else 0
        up, down = self.dup, self.ddown
        hdone = [Event() for _ in range(self.nchunks)]
        kdone = [Event() for _ in range(self.nchunks)]
        t0 = time.perf_counter()
        for c in range(self.nchunks):
            lo, hi = self._range(c)
            m = hi - lo
            f0, f1 = int(self.frame_off[lo]), int(self.frame_off[hi])
            e0 = self._mark(up, "h2d")
            _lib.check(L.kdb_lz4_memcpy_h2d(self.d_packed.ptr + f0, self.h_frames.ptr + f0, f1 - f0, up.ptr), "h2d frames")
            for base, w in ((0, 8), (8 * n, 4)):
                _lib.check(L.kdb_lz4_memcpy_h2d(self.d_dmeta.ptr + base + w * lo, self.h_dmeta.ptr + base + w * lo,
                                                w * m, up.ptr), "h2d meta")
            self._span("h2d", c, e0, up)
            hdone[c].record(up)
            ks = self.streams[c % S]
            _lib.check(L.kdb_lz4_stream_wait_event(ks.ptr, hdone[c].ptr), "stream_wait_event")
            e0 = self._mark(ks, "kernel")
            _lib.check(L.kdb_lz4_decompress_frames_batch(
                ks.ptr, self.d_packed.ptr, self.d_dmeta.ptr + 8 * lo, self.d_dmeta.ptr + 8 * n + 4 * lo, m, max_in,
                size, self.d_out.ptr, self.d_dconst.ptr + 8 * lo, self.d_dconst.ptr + 8 * n + 4 * lo,
                self.d_dres.ptr + 4 * lo, self.d_dres.ptr + 4 * n + 4 * lo), "decompress_frames_batch")
            self._span("kernel", c, e0, ks)
            kdone[c].record(ks)
            _lib.check(L.kdb_lz4_stream_wait_event(down.ptr, kdone[c].ptr), "stream_wait_event")
            e0 = self._mark(down, "d2h")
            _lib.check(L.kdb_lz4_memcpy_d2h(self.h_out.ptr + lo * size, self.d_out.ptr + lo * size, m * size,
                                            down.ptr), "d2h out")
            self._span("d2h", c, e0, down)
            for base in (4 * lo, 4 * n + 4 * lo):
                _lib.check(L.kdb_lz4_memcpy_d2h(self.h_dres.ptr + base, self.d_dres.ptr + base, 4 * m, down.ptr),
                           "d2h results")
        for s in self.streams + self.dstreams + [self.dup, self.ddown]:
            s.sync()
        return time.perf_counter() - t0

    def _copies(self, h2d: bool, d2h: bool) -> float:
        """The link alone: n*size bytes in the pipeline's chunks over its
        streams, one or both directions at once.  Wall seconds."""
        L = lib()
        S = len(self.streams)
        t0 = time.perf_counter()
        for c in range(self.nchunks):
            lo, hi = self._range(c)
            nb = (hi - lo) * self.size
            if h2d:
                _lib.check(L.kdb_lz4_memcpy_h2d(self.d_raw.ptr + lo * self.size, self.h_raw.ptr + lo * self.size, nb,
                                                self.streams[c % S].ptr), "h2d")
            if d2h:
                _lib.check(L.kdb_lz4_memcpy_d2h(self.h_out.ptr + lo * self.size, self.d_out.ptr + lo * self.size, nb,
                                                self.streams[(c + S // 2) % S].ptr), "d2h")
        for s in self.streams:
            s.sync()
        return time.perf_counter() - t0

    def profile(self, kinds=None) -> dict:
        """Where the host-inclusive time goes: traced compress and decompress
        runs (HIP events around every chunk's H2D, kernels and D2H on its
        stream; the median of three per phase), each kind's busy time as the
        union of its intervals, against the wall time and against the link alone
        (the same bytes copied with no kernel, each direction and both at once)."""
        raw = float(self.n) * self.size
        link = {}
        for name, h, d in (("h2d", True, False), ("d2h", False, True), ("both", True, True)):
            self._copies(h, d)
            t = min(self._copies(h, d) for _ in range(3))
            link[name + "_gbs"] = round((raw * (h + d)) / t / 1e9, 2)
        out = {"link_alone": link}
        # one untraced round trip first: the first compress after other copy
        # traffic runs ~10 % slow (profiles/r06/r06_e_hostprobe.json), and the
        # traced runs are to show the pipeline the timed runs measure
        self.compress()
        self.decompress()
        self._kinds = set(kinds) if kinds else None

        def traced(phase):
            self._pool = [Event() for _ in range(8 * self.nchunks + 8)]
            self._trace = []
            base = Event()
            base.record(self.streams[0])
            self._base = base
            for ds in self.dstreams + [self.dup, self.ddown, self.cup]:   # every traced stream starts after the base event
                _lib.check(lib().kdb_lz4_stream_wait_event(ds.ptr, base.ptr), "stream_wait_event")
            wall = getattr(self, phase)()
            spans, self._trace = self._trace, None

            def at(e):   # an event's time, or the latest of several
                return max(base.elapsed_ms(x) for x in e) if isinstance(e, list) else base.elapsed_ms(e)
            return wall, [(kind, at(e0), at(e1)) for kind, _c, e0, e1 in spans]

        # three traced round trips, as the timed runs alternate the phases; each
        # phase's run of median wall time is reported (the statistic of the timed
        # median: a single traced run could land on either side of it)
        runs = {"compress": [], "decompress": []}
        for _ in range(3):
            for phase in ("compress", "decompress"):
                runs[phase].append(traced(phase))
        for phase in ("compress", "decompress"):
            wall, spans = sorted(runs[phase], key=lambda r: r[0])[1]
            iv = {}
            for kind, a, b in spans:
                iv.setdefault(kind, []).append((a, b))
            res = {"wall_ms": round(wall * 1e3, 3), "traced_runs_ms": [round(r[0] * 1e3, 3) for r in runs[phase]]}
            allcopy = []
            if not iv:
                out[phase] = res
                continue
            for kind, ivs in sorted(iv.items()):
                res[kind + "_busy_ms"] = round(_union(ivs), 3)
                res[kind + "_sum_ms"] = round(sum(b - a for a, b in ivs), 3)
                if kind != "kernel":
                    allcopy += ivs
            res["link_busy_ms"] = round(_union(allcopy), 3)
            first = min(a for ivs in iv.values() for a, _ in ivs)
            last = max(b for ivs in iv.values() for _, b in ivs)
            res["device_span_ms"] = round(last - first, 3)
            res["first_op_at_ms"] = round(first, 3)
            out[phase] = res
        by = {"compress": (raw, float(self.frame_bytes)), "decompress": (float(self.frame_bytes), raw)}
        for phase, (hb, db) in by.items():
            r = out[phase]
            if "h2d_busy_ms" in r:
                r["h2d_gbs_while_busy"] = round(hb / (r["h2d_busy_ms"] * 1e-3) / 1e9, 2)
            if "d2h_busy_ms" in r:
                r["d2h_gbs_while_busy"] = round(db / (r["d2h_busy_ms"] * 1e-3) / 1e9, 2)
        self._kinds = None
        return out

    def free(self) -> None:
        for b in (self.h_raw, self.h_frames, self.h_out, self.h_cmeta, self.h_cres, self.h_dmeta, self.h_dres,
                  self.h_tot, self.d_raw, self.d_slots, self.d_packed, self.d_out, self.d_cmeta, self.d_cres,
                  self.d_pack_off, self.d_tot, self.d_dmeta, self.d_dconst, self.d_dres):
            b.free()
