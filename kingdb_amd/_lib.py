"""ctypes binding of libkdb_lz4.so (the C ABI in include/kdb_lz4.h).

The library holds the gfx950 HIP kernels; there is no CPU codec behind it.
Loading fails loudly (ImportError-like RuntimeError) when the .so is missing.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# KDB_LZ4_LIB: another build of the same library (A/B variants under
# kingdb_amd/var/, tools/build_variants.sh); the default is the in-tree build
LIB_PATH = os.environ.get("KDB_LZ4_LIB") or os.path.join(HERE, "libkdb_lz4.so")

OK = 0
EINVAL = -1
EHIP = -2
ENODEV = -3
EUNSUPPORTED = -4
VALUE_UNSUPPORTED = -(2 ** 31)

_c = ctypes
_vp = _c.c_void_p
_u8p = _c.c_void_p   # device / host byte pointers are passed as integers
_i = _c.c_int
_u32 = _c.c_uint32
_u64 = _c.c_uint64

# name -> (restype, argtypes); mirrors include/kdb_lz4.h one for one.
SIGNATURES = {
    "kdb_lz4_version": (_i, []),
    "kdb_lz4_device_count": (_i, [_c.POINTER(_i)]),
    "kdb_lz4_set_device": (_i, [_i]),
    "kdb_lz4_get_device": (_i, [_c.POINTER(_i)]),
    "kdb_lz4_selftest": (_i, [_i, _c.POINTER(_i), _c.POINTER(_u32)]),
    "kdb_lz4_service_stats": (_i, [_i, _c.POINTER(_u32), _c.POINTER(_u32), _c.POINTER(_u32)]),
    "kdb_lz4_service_counters": (_i, [_i, _c.POINTER(_u32), _c.POINTER(_u32), _c.POINTER(_u32)]),
    "kdb_lz4_service_seed_requests": (_i, [_u32, _u32]),
    "kdb_lz4_last_kernels": (_i, [_c.c_char_p, _u64]),
    "kdb_lz4_build_id": (_i, [_c.c_char_p, _u64]),
    "kdb_lz4_max_u32": (_i, [_vp, _vp, _u32, _vp]),
    "kdb_lz4_warmup": (_i, []),
    "kdb_lz4_malloc": (_i, [_c.POINTER(_vp), _u64]),
    "kdb_lz4_free": (_i, [_vp]),
    "kdb_lz4_host_alloc": (_i, [_c.POINTER(_vp), _u64]),
    "kdb_lz4_host_free": (_i, [_vp]),
    "kdb_lz4_memcpy_h2d": (_i, [_vp, _vp, _u64, _vp]),
    "kdb_lz4_memcpy_d2h": (_i, [_vp, _vp, _u64, _vp]),
    "kdb_lz4_memcpy_d2d": (_i, [_vp, _vp, _u64, _vp]),
    "kdb_lz4_memset": (_i, [_vp, _i, _u64, _vp]),
    "kdb_lz4_stream_create": (_i, [_c.POINTER(_vp)]),
    "kdb_lz4_stream_destroy": (_i, [_vp]),
    "kdb_lz4_stream_sync": (_i, [_vp]),
    "kdb_lz4_device_sync": (_i, []),
    "kdb_lz4_event_create": (_i, [_c.POINTER(_vp)]),
    "kdb_lz4_event_destroy": (_i, [_vp]),
    "kdb_lz4_event_record": (_i, [_vp, _vp]),
    "kdb_lz4_event_sync": (_i, [_vp]),
    "kdb_lz4_stream_wait_event": (_i, [_vp, _vp]),
    "kdb_lz4_event_elapsed_ms": (_i, [_vp, _vp, _c.POINTER(_c.c_float)]),
    "kdb_lz4_compressBound": (_i, [_i]),
    "kdb_lz4_compress_limitedOutput": (_i, [_c.c_char_p, _vp, _i, _i]),
    "kdb_lz4_decompress_safe_partial": (_i, [_c.c_char_p, _vp, _i, _i, _i]),
    "kdb_lz4_frame_bound": (_u64, [_u32]),
    "kdb_lz4_compress_blocks_batch": (_i, [_vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp]),
    "kdb_lz4_decompress_blocks_batch": (_i, [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    "kdb_lz4_compress_frames_batch": (_i, [_vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp]),
    "kdb_lz4_decompress_frames_batch": (_i, [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    "kdb_lz4_pack_frames": (_i, [_vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    "kdb_lz4_gen_g1": (_i, [_vp, _u64, _u64, _u32, _vp]),
    # include/kdb_flush.h (the write-buffer flush batch)
    "kdb_flush_scratch_bytes": (_u64, [_u32, _u32, _u64]),
    "kdb_flush_parts_batch": (_i, [_vp] * 12 + [_u32, _u32, _u32, _u32, _vp, _u64, _u64, _vp, _vp, _vp, _vp]),
    # include/kdb_put.h (the write path around the codec)
    "kdb_put_scratch_bytes": (_u64, [_u32, _u32, _u64]),
    "kdb_put_entries_batch": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _vp, _u64,
                                   _u64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "kdb_get_scratch_bytes": (_u64, [_u32, _u64]),
    "kdb_get_values_batch": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _i, _vp, _vp, _u64, _u32, _u32, _vp,
                                  _u64, _vp, _vp]),
    "kdb_hstable_db_options": (_i, [_u64, _u32, _vp]),
    "kdb_hstable_writer_create": (_i, [_u64, _u32, _c.POINTER(_vp)]),
    "kdb_hstable_writer_create2": (_i, [_u64, _u32, _u32, _c.POINTER(_vp)]),
    "kdb_hstable_writer_append": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    "kdb_hstable_writer_append_device": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    "kdb_hstable_writer_close": (_i, [_vp]),
    "kdb_hstable_writer_file_count": (_i, [_vp, _c.POINTER(_u32)]),
    "kdb_hstable_writer_file": (_i, [_vp, _u32, _c.POINTER(_u32), _c.POINTER(_vp), _c.POINTER(_u64)]),
    "kdb_hstable_writer_save": (_i, [_vp, _c.c_char_p]),
    "kdb_hstable_writer_reset": (_i, [_vp]),
    "kdb_hstable_writer_destroy": (_i, [_vp]),
    # link-time aliases of the reference's lz4.h names
    "LZ4_compressBound": (_i, [_i]),
    "LZ4_compress_limitedOutput": (_i, [_c.c_char_p, _vp, _i, _i]),
    "LZ4_decompress_safe_partial": (_i, [_c.c_char_p, _vp, _i, _i, _i]),
}

_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libkdb_lz4.so (once).  Raises if the HIP library was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: the kingdb_amd HIP extension is not built "
            "(run `make -C kingdb_amd` or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class HipError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != OK:
        names = {EINVAL: "EINVAL", EHIP: "EHIP", ENODEV: "ENODEV", EUNSUPPORTED: "EUNSUPPORTED"}
        raise HipError(f"{what} failed: {names.get(rc, rc)}")
