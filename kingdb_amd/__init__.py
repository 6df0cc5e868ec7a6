"""kingdb_amd -- MI355X-native (gfx950) LZ4 block codec for KingDB values.

The product is ``libkdb_lz4.so``: hand-written HIP kernels behind the C ABI in
``include/kdb_lz4.h`` plus the C++ ``kdb::CompressorLZ4`` drop-in.  This
package is its Python face (ctypes), used by the tests and the benchmark.
"""
from . import _lib  # noqa: F401
from .lz4 import (  # noqa: F401
    DeviceBatch,
    DeviceBuffer,
    Event,
    Stream,
    compress_blocks,
    compress_bound,
    build_id,
    compress_frames,
    compress_limited_output,
    decompress_blocks,
    decompress_frames,
    decompress_safe_partial,
    device_count,
    frame_bound,
    get_device,
    last_kernels,
    selftest,
    set_device,
)

__all__ = [
    "DeviceBatch", "DeviceBuffer", "Event", "Stream", "build_id", "compress_blocks", "compress_bound",
    "compress_frames", "compress_limited_output", "decompress_blocks", "decompress_frames",
    "decompress_safe_partial", "device_count", "frame_bound", "get_device", "last_kernels", "selftest",
    "set_device",
]
