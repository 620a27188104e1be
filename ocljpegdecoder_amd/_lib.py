"""ctypes binding of the native library (ocljpegdecoder_amd/lib/libhjd.so).

The library is the product: importing the package without it raises
immediately -- there is no Python or CPU fallback for the pixel path.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HJD_LIB") or os.path.join(_PKG, "lib", "libhjd.so")   # HJD_LIB: tuning builds only

c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u32p = ctypes.POINTER(ctypes.c_uint32)


class HjdFrame(ctypes.Structure):
    """struct hjd_frame (include/hjd.h)."""
    _fields_ = [
        ("coef_offset", ctypes.c_uint64),
        ("out_offset", ctypes.c_uint64),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("out_pitch", ctypes.c_int32),
        ("sampling", ctypes.c_int32),
        ("qt_index", ctypes.c_int32 * 3),
        ("out_format", ctypes.c_int32),
    ]


assert ctypes.sizeof(HjdFrame) == 48


class HjdLaunchShape(ctypes.Structure):
    """struct hjd_launch_shape (include/hjd.h)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("kernel", "tasks_per_wave", "max_tasks_per_wave", "grid", "variant",
                                              "autotune_launches", "autotune_cached")]


class HjdJpegInfo(ctypes.Structure):
    """struct hjd_jpeg_info (include/hjd_host.h)."""
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("sampling", ctypes.c_int32),
        ("restart_interval", ctypes.c_int32),
        ("mcu_w", ctypes.c_int32),
        ("mcu_h", ctypes.c_int32),
        ("nblocks", ctypes.c_int64),
        ("qt", (ctypes.c_int32 * 64) * 3),
        ("qt_precision", ctypes.c_int32 * 3),
        ("scan_offset", ctypes.c_int64),
        ("process", ctypes.c_int32),
        ("single_scan", ctypes.c_int32),
    ]


# (name, restype, argtypes) of every exported C symbol declared in include/*.h
SIGNATURES = {
    # include/hjd.h
    "hjd_abi_version": (ctypes.c_int, []),
    "hjd_last_error": (ctypes.c_char_p, []),
    "hjd_device_count": (ctypes.c_int, [c_i32p]),
    "hjd_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "hjd_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hjd_ctx_device": (ctypes.c_int, [ctypes.c_void_p]),
    "hjd_frame_blocks": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    "hjd_plan_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HjdFrame), ctypes.c_int, ctypes.c_int,
                                       c_i32p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "hjd_plan_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hjd_plan_set_variant": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hjd_plan_set_kernel": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hjd_plan_set_chunk": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hjd_plan_tasks": (ctypes.c_int64, [ctypes.c_void_p]),
    "hjd_plan_pixels": (ctypes.c_int64, [ctypes.c_void_p]),
    "hjd_plan_coef_bytes": (ctypes.c_int64, [ctypes.c_void_p]),
    "hjd_plan_launch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]),
    "hjd_plan_autotune": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int, c_i32p, c_i32p]),
    "hjd_autotune_cache_clear": (ctypes.c_int, []),
    "hjd_plan_launch_shape": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HjdLaunchShape)]),
    "hjd_idct_blocks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_void_p]),
    "hjd_debug_csc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    "hjd_debug_csc_exhaustive": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "hjd_debug_plan_launch_stages": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_int]),
    "hjd_debug_rw_mix": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "hjd_debug_d16_gather": (ctypes.c_int, [ctypes.c_int, c_i32p, c_i32p]),
    "hjd_debug_clock_probe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_void_p]),
}

_lib = None


class HjdError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what} failed with status {code}: {error_string()}")
        self.code = code


def load():
    """Load libhjd.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"native library missing: {LIB_PATH} -- run `python tools/build_native.py` "
                          "(or __graft_entry__.build()); the HIP path has no fallback")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so
    # (SONAME libamdhip64.so.7) and NEEDs it unversioned, so if libhjd.so pulled
    # /opt/rocm's copy in first, torch would load a second runtime beside it.
    # Loading torch first makes libhjd.so's NEEDED libamdhip64.so.7 resolve to
    # the runtime torch already mapped.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        # a tuning build named by HJD_LIB (e.g. an older tree for an A/B) may
        # lack newer entry points; the product library must export them all
        fn = getattr(lib, name, None) if os.environ.get("HJD_LIB") else getattr(lib, name)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _bind_host(lib)
    _lib = lib
    return lib


def _bind_host(lib):
    """Host JPEG front end symbols (include/hjd_host.h), when compiled in."""
    u8p = ctypes.POINTER(ctypes.c_uint8)
    sigs = {
        "hjd_jpeg_parse": (ctypes.c_int, [u8p, ctypes.c_size_t, ctypes.POINTER(HjdJpegInfo)]),
        "hjd_jpeg_decode_coefs": (ctypes.c_int, [u8p, ctypes.c_size_t, ctypes.POINTER(HjdJpegInfo),
                                                 ctypes.POINTER(ctypes.c_int16), ctypes.c_int64]),
        "hjd_jpeg_decode_batch": (ctypes.c_int, [ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                                 ctypes.POINTER(ctypes.POINTER(ctypes.c_int16)), ctypes.c_int64,
                                                 ctypes.c_int, c_i32p]),
    }
    vp = ctypes.c_void_p
    sigs.update({
        "hjd_stream_create": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
        "hjd_stream_destroy": (ctypes.c_int, [vp]),
        "hjd_stream_submit": (ctypes.c_int, [vp, u8p, ctypes.c_size_t, vp, ctypes.c_int32]),
        "hjd_stream_sync": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64)]),
        "hjd_stream_busy": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
        "hjd_debug_worker_cpus": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                                 ctypes.c_int, ctypes.c_int, c_i32p, ctypes.c_int, c_i32p]),
        "hjd_gdec_create": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                           ctypes.POINTER(vp)]),
        "hjd_gdec_destroy": (ctypes.c_int, [vp]),
        "hjd_gdec_decode": (ctypes.c_int, [vp, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                           ctypes.POINTER(vp), c_i32p, vp]),
        "hjd_gdec_decode_coefs": (ctypes.c_int, [vp, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                                 ctypes.c_int, vp, ctypes.POINTER(ctypes.c_int64), vp]),
        "hjd_gdec_sync": (ctypes.c_int, [vp, c_i32p]),
        "hjd_gdec_set_output_format": (ctypes.c_int, [vp, ctypes.c_int]),
        "hjd_gdec_last_bytes": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
        "hjd_gstream_create": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                              ctypes.c_int, ctypes.POINTER(vp)]),
        "hjd_gstream_destroy": (ctypes.c_int, [vp]),
        "hjd_gstream_submit": (ctypes.c_int, [vp, u8p, ctypes.c_size_t, vp, ctypes.c_int32]),
        "hjd_gstream_submit_host": (ctypes.c_int, [vp, u8p, ctypes.c_size_t, vp, ctypes.c_int32]),
        "hjd_bmp_header": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, u8p]),
        "hjd_bmp_header_bgr24": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, u8p]),
        "hjd_gstream_set_output_format": (ctypes.c_int, [vp, ctypes.c_int]),
        "hjd_gstream_host_bytes": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64)]),
        "hjd_host_register": (ctypes.c_int, [vp, ctypes.c_size_t]),
        "hjd_host_unregister": (ctypes.c_int, [vp]),
        "hjd_debug_host_prep": (ctypes.c_int, [ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                               ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
        "hjd_debug_host_reader": (ctypes.c_int, [ctypes.c_int]),
        "hjd_host_cpu_share": (ctypes.c_int, []),
        "hjd_debug_cpu_share": (ctypes.c_int, [ctypes.c_char_p]),
        "hjd_device_worker_cpus": (ctypes.c_int, [ctypes.c_int, c_i32p, ctypes.c_int, c_i32p]),
        "hjd_debug_destuff_host": (ctypes.c_int, [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                                  ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64)]),
        "hjd_debug_destuff_gpu": (ctypes.c_int, [vp, u8p, ctypes.c_size_t, ctypes.c_int, u8p, ctypes.c_size_t,
                                                 ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int64),
                                                 ctypes.POINTER(ctypes.c_uint32)]),
        "hjd_stream_set_output_format": (ctypes.c_int, [vp, ctypes.c_int]),
        "hjd_gstream_sync": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64)]),
        "hjd_debug_entropy_emulate": (ctypes.c_int, [u8p, ctypes.c_size_t, ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_int16), ctypes.c_int64, c_i32p]),
        "hjd_debug_entropy_sync_check": (ctypes.c_int, [u8p, ctypes.c_size_t, ctypes.c_int,
                                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    })
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
            SIGNATURES.setdefault(name, (res, args))


def error_string() -> str:
    lib = load()
    s = lib.hjd_last_error()
    return s.decode() if s else ""


def check(code, what):
    if code != 0:
        raise HjdError(code, what)
    return code
