"""Test configuration: registers the `gpu` marker and puts the repo root on sys.path.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, and
that libkdb_lz4.so loads and exports every symbol include/kdb_lz4.h declares.
`-m gpu` runs on an MI355X: HIP kernels vs the golden fixtures and the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def split(data, off, lens):
    return [data[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, lens)]


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle.Oracle()


@pytest.fixture(scope="session")
def gpu():
    """The product library, on a real device; fails (not skips) if the HIP
    extension is missing on a GPU box."""
    import kingdb_amd
    from kingdb_amd import _lib
    _lib.load()
    n = kingdb_amd.device_count()
    if n == 0:
        pytest.fail("no GPU visible to libkdb_lz4.so")
    kingdb_amd.set_device(0)
    return kingdb_amd


def big_value_inputs(g, pool_bytes):
    """Inputs of big_values.npz by name: G1 pool slices and 'a' runs are
    regenerated (tests/golden/make_golden.py:big_inputs), the rest stored."""
    out = []
    for name, size in zip(g["names"], g["sizes"]):
        name, size = str(name), int(size)
        if name.startswith("g1_"):
            start = 7 if size == 100000 else 0
            out.append(pool_bytes[start:start + size])
        elif name.startswith("a_"):
            out.append(b"a" * size)
        else:
            out.append(g["inp_" + name].tobytes())
        assert len(out[-1]) == size, name
    return out


def apply_recipe(blk, kind, pos, val):
    """kind 0: truncate to pos bytes; 1: flip bit val at pos; 2: set pos to val."""
    b = bytearray(blk)
    if kind == 0:
        return bytes(b[:pos])
    if kind == 1:
        b[pos] ^= 1 << val
    else:
        b[pos] = val
    return bytes(b)
