"""GPU: the compressor's batched emission (lz4_compress.hip flush_batch, round
5) against the oracle on values that stress it: runs of a small alphabet
(many short sequences: more than 64 per value, so batches flush mid-value),
incompressible tails (literal runs past 64 and past 270 bytes: multi-byte
length runs), long runs (match-length runs of several bytes), in the
<= 4 KiB class and the LDS-staged 4-8 KiB class, alone and mixed with short
values (the per-value choice of the mixed kernel).  Frames must be the
oracle's byte for byte (the oracle is pinned to the reference's lz4.cc)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mix(x):
    m = (1 << 64) - 1
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & m
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & m
    x ^= x >> 33
    return x


def _runs_value(seed, n, tail):
    """oracle/hook_mt.cc's value shape: runs of 1-30 letters of a 12-letter
    alphabet, optionally an incompressible tail."""
    rng = np.random.default_rng(seed)
    runs = rng.integers(1, 31, n)
    letters = rng.integers(0, 12, n).astype(np.uint8) + ord("a")
    v = np.repeat(letters, runs)[:n].tobytes()
    if tail:
        cut = int(rng.integers(0, n))
        v = v[:cut] + rng.integers(0, 256, n - cut, dtype=np.uint8).tobytes()
    return v


def _values():
    rng = np.random.default_rng(11)
    vals = []
    for k in range(400):
        n = int(rng.choice([int(rng.integers(1, 400)), int(rng.integers(2000, 4097)), int(rng.integers(4097, 8193)),
                            4096, 4097, 8192]))
        vals.append(_runs_value(k, n, k % 4 == 0))
    # long runs (match-length run bytes), long literal runs, mixed
    vals += [b"a" * n for n in (600, 4096, 5000, 8192)]
    vals += [rng.integers(0, 256, n, dtype=np.uint8).tobytes() + b"b" * 700 for n in (300, 2000, 5000)]
    vals += [(b"xyz" * 3000)[:n] for n in (4000, 7000)]
    return vals


@pytest.mark.parametrize("with_short", [False, True])
def test_batched_emission_frames_equal_oracle(gpu, orc, with_short):
    vals = _values()
    if with_short:
        vals = vals + [_runs_value(1000 + k, 100, False) for k in range(200)] + [b"q" * 20000]   # mixed kernel
    got = gpu.compress_frames(vals)
    bad = [i for i, (v, f) in enumerate(zip(vals, got)) if f != orc.frame(v)]
    assert not bad, [(i, len(vals[i])) for i in bad[:10]]
