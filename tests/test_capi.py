"""CPU: libkdb_lz4.so loads and exports every symbol include/kdb_lz4.h declares;
host-side helpers behave; compute entry points refuse to run without a GPU
(they never fall back to a CPU codec)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def header_symbols():
    syms = set()
    for h in ("kdb_lz4.h", "kdb_put.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        syms |= set(re.findall(r"\b(kdb_(?:lz4|put|get|hstable)_\w+)\s*\(", text))
    return sorted(syms)


def test_library_exports_every_header_symbol():
    from kingdb_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 35
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} missing from the ctypes signature table"
    # link-time aliases with the reference's own lz4.h names (lz4.h:115,129,169)
    for s in ("LZ4_compressBound", "LZ4_compress_limitedOutput", "LZ4_decompress_safe_partial"):
        assert hasattr(lib, s)


def test_bound_helpers_match_reference_macro(orc):
    from kingdb_amd import _lib
    lib = _lib.load()
    for n in (0, 1, 12, 100, 254, 255, 4096, 65536, 0x7E000000, 0x7E000001, -1):
        assert lib.kdb_lz4_compressBound(n) == orc.compress_bound(n)
        assert lib.LZ4_compressBound(n) == orc.compress_bound(n)
    for n in (0, 100, 4096, 65536):
        assert lib.kdb_lz4_frame_bound(n) == 8 + orc.compress_bound(n)


def test_no_cpu_fallback_without_device():
    import kingdb_amd
    from kingdb_amd import _lib
    if kingdb_amd.device_count() > 0:
        pytest.skip("a GPU is visible; this checks the no-GPU behaviour")
    lib = _lib.load()
    dst = ctypes.create_string_buffer(64)
    # LZ4 conventions: 0 = compression failed, negative = decode failed.
    assert lib.kdb_lz4_compress_limitedOutput(b"a" * 40, ctypes.addressof(dst), 40, 64) == 0
    assert lib.kdb_lz4_decompress_safe_partial(b"\x10a", ctypes.addressof(dst), 2, 1, 1) < 0
    with pytest.raises(_lib.HipError):
        kingdb_amd.compress_frames([b"x" * 100])


def test_missing_library_fails_loudly(tmp_path):
    from kingdb_amd import _lib
    saved = _lib._lib
    try:
        _lib._lib = None
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved
