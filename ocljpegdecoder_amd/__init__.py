"""ocljpegdecoder_amd -- MI355X-native JPEG pixel back-end.

Drop-in replacement for the OpenCL IDCT/colour back-end of
xinfushe/oclJPEGDecoder (src/oclDCT8x8.cpp + src/idct8x8.cl behind src/idct.h).
The hot path is the fused HIP kernel in csrc/hjd_kernels.hpp, reached through
the C ABI in include/hjd.h (libhjd.so).  Importing this package loads the
native library and fails loudly if it is missing.
"""
from . import _lib

_lib.load()

from .backend import (  # noqa: E402
    IN_I32_NATURAL,
    IN_Q16_ZIGZAG,
    OTHER,
    KERNEL_AUTO,
    KERNEL_LATENCY,
    KERNEL_PERSISTENT,
    OUT_BGR24,
    OUT_BGRX,
    OUT_BYTES,
    GRAY,
    YUV411_H4V1,
    YUV420,
    YUV422,
    YUV440,
    YUV444,
    autotune_cache_clear,
    block_components,
    Context,
    cpu_share,
    FrameSpec,
    Plan,
    decode_frame,
    default_pitch,
    device_count,
    device_worker_cpus,
    frame_blocks,
    mcu_geometry,
    stream_worker_threads,
    worker_cpus,
)

from .jpeg import (GpuDecoder, GpuJpegStream, JpegInfo, JpegStream, bmp_bytes, bmp_header,  # noqa: E402
                   decode_coefs, decode_coefs_batch, decode_coefs_into, decode_jpeg, emulate_entropy, parse,
                   pinned_bytes)

__all__ = [
    "GpuDecoder", "GpuJpegStream", "JpegInfo", "JpegStream", "bmp_bytes", "bmp_header", "decode_coefs",
    "decode_coefs_batch", "decode_coefs_into", "decode_jpeg", "emulate_entropy",
    "parse", "pinned_bytes",
    "Context", "FrameSpec", "Plan", "autotune_cache_clear", "decode_frame", "device_count", "frame_blocks", "mcu_geometry", "worker_cpus", "cpu_share",
    "device_worker_cpus", "stream_worker_threads",
    "YUV444", "YUV420", "YUV422", "GRAY", "YUV411_H4V1", "YUV440", "OTHER", "block_components", "KERNEL_AUTO", "KERNEL_PERSISTENT", "KERNEL_LATENCY", "OUT_BGRX", "OUT_BGR24", "OUT_BYTES", "default_pitch", "IN_Q16_ZIGZAG", "IN_I32_NATURAL",
]
