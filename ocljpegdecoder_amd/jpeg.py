"""Host JPEG front end + streaming decode (include/hjd_host.h).

    info = parse(data)                        # headers only
    coefs, info = decode_coefs(data)          # host Huffman -> int16 zigzag coefficients
    pixels = decode_jpeg(ctx, data)           # host Huffman + fused HIP kernel, BGRX on the device
    with JpegStream(ctx, max_blocks) as st:   # Huffman workers || H2D || kernel
        st.submit(data, out_tensor); st.sync()
    gd = GpuDecoder(ctx, max_frames, max_scan_bytes, max_blocks)   # Huffman decode ON the GPU
        gd.decode([data, ...], [out_tensor, ...]); gd.sync()
    with GpuJpegStream(ctx, 32, 32 << 22, 32 * 194400) as st:      # destuff workers || H2D || GPU Huffman + pixels
        st.submit(data, out_tensor); st.sync()
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import HjdJpegInfo, check

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i16p = ctypes.POINTER(ctypes.c_int16)


@dataclass
class JpegInfo:
    width: int
    height: int
    sampling: int
    restart_interval: int
    mcu_w: int
    mcu_h: int
    nblocks: int
    qt: np.ndarray            # [3][64] file (zigzag) order, per component
    qt_precision: tuple
    scan_offset: int
    process: int = 0          # 0 baseline, 1 extended sequential, 2 progressive
    single_scan: bool = True  # one interleaved sequential scan (GPU entropy decodable)

    @classmethod
    def from_c(cls, c: HjdJpegInfo) -> "JpegInfo":
        return cls(c.width, c.height, c.sampling, c.restart_interval, c.mcu_w, c.mcu_h, c.nblocks,
                   np.array(c.qt, dtype=np.int32), tuple(c.qt_precision), c.scan_offset,
                   c.process, bool(c.single_scan))


def _src(data):
    """(uint8 pointer, size, object to keep alive) of JPEG bytes, without a copy:
    bytes / bytearray / memoryview / uint8 numpy array / ctypes array.  (A copy
    per call cost a 1 MB FHD JPEG ~0.1 ms of allocation, page faults and memcpy
    on the latency path.)  The library only reads the bytes (const uint8_t*)."""
    if isinstance(data, bytes):   # the object's own buffer (c_char_p does not copy): ~1 us
        return ctypes.cast(ctypes.c_char_p(data), _u8p), len(data), data
    if isinstance(data, ctypes.Array):
        return ctypes.cast(data, _u8p), len(data), data
    a = data if isinstance(data, np.ndarray) else np.frombuffer(data, np.uint8)
    if a.dtype != np.uint8 or not a.flags.c_contiguous:
        raise ValueError("JPEG bytes must be contiguous uint8")
    return a.ctypes.data_as(_u8p), a.nbytes, a


def _buf(data):
    """The bytes' address as a uint8 pointer that keeps them alive (_src)."""
    return _src(data)[0]


def parse(data: bytes) -> JpegInfo:
    lib = _lib.load()
    info = HjdJpegInfo()
    check(lib.hjd_jpeg_parse(_buf(data), len(data), ctypes.byref(info)), "hjd_jpeg_parse")
    return JpegInfo.from_c(info)


def decode_coefs(data: bytes):
    """Host Huffman decode -> (int16 [nblocks][64] zigzag coefficients, JpegInfo)."""
    lib = _lib.load()
    buf = _buf(data)
    info = HjdJpegInfo()
    check(lib.hjd_jpeg_parse(buf, len(data), ctypes.byref(info)), "hjd_jpeg_parse")
    coefs = np.empty((info.nblocks, 64), np.int16)
    check(lib.hjd_jpeg_decode_coefs(buf, len(data), ctypes.byref(info), coefs.ctypes.data_as(_i16p), info.nblocks),
          "hjd_jpeg_decode_coefs")
    return coefs, JpegInfo.from_c(info)


def decode_coefs_into(data: bytes, out: np.ndarray) -> JpegInfo:
    """Host Huffman decode into a caller-provided int16 [>= nblocks][64] array
    (e.g. a pinned host tensor's numpy view, for an H2D copy straight after)."""
    lib = _lib.load()
    buf = _buf(data)
    info = HjdJpegInfo()
    check(lib.hjd_jpeg_parse(buf, len(data), ctypes.byref(info)), "hjd_jpeg_parse")
    if out.dtype != np.int16 or out.ndim != 2 or out.shape[1] != 64 or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous int16 [blocks][64] array")
    check(lib.hjd_jpeg_decode_coefs(buf, len(data), ctypes.byref(info), out.ctypes.data_as(_i16p), out.shape[0]),
          "hjd_jpeg_decode_coefs")
    return JpegInfo.from_c(info)


def decode_coefs_batch(datas: Sequence[bytes], nthreads: int = 0,
                       outs: Optional[Sequence[np.ndarray]] = None) -> List[np.ndarray]:
    """Decode many files on a host thread pool.  `outs`: one C-contiguous
    (>= nblocks, 64) int16 array per file to decode into (reused buffers: no
    allocation or first-touch page faults in the call), else new arrays."""
    lib = _lib.load()
    infos = [parse(d) for d in datas]
    if outs is None:
        outs = [np.empty((i.nblocks, 64), np.int16) for i in infos]
    else:
        outs = list(outs)
        if len(outs) != len(datas) or any(o.dtype != np.int16 or o.ndim != 2 or o.shape[1] != 64
                                          or not o.flags.c_contiguous for o in outs):
            raise ValueError("outs: one C-contiguous (n, 64) int16 array per file")
    cap = max([i.nblocks for i in infos] or [0])
    srcs = [_src(d) for d in datas]
    arr_d = (_u8p * len(srcs))(*[p for p, _, _ in srcs])
    arr_s = (ctypes.c_size_t * len(srcs))(*[n for _, n, _ in srcs])
    arr_o = (_i16p * len(outs))(*[o.ctypes.data_as(_i16p) for o in outs])
    status = (ctypes.c_int32 * len(datas))()
    # capacity checked per file (the library takes one capacity for the batch)
    for o, i in zip(outs, infos):
        if o.shape[0] < i.nblocks:
            raise ValueError(f"output of {o.shape[0]} blocks < {i.nblocks}")
    check(lib.hjd_jpeg_decode_batch(arr_d, arr_s, len(datas), arr_o, cap, nthreads, status),
          "hjd_jpeg_decode_batch")
    return outs


def decode_jpeg(ctx, data: bytes, stream=None, out_format: int = 0):
    """JPEG bytes -> device pixels (host Huffman, then the fused kernel on the
    device): an (H, W) int32 tensor of BGRX words, or with out_format=OUT_BGR24
    an (H, pitch) uint8 tensor of B,G,R bytes (pitch = (3W+3)&~3, the 24-bpp
    BMP row)."""
    import torch
    from .backend import IN_Q16_ZIGZAG, OUT_BGR24, FrameSpec, Plan, default_pitch
    coefs, info = decode_coefs(data)
    dev = torch.device("cuda", ctx.device)
    d_coefs = torch.from_numpy(coefs).to(dev)
    if out_format == OUT_BGR24:
        out = torch.empty((info.height, default_pitch(info.width, OUT_BGR24)), dtype=torch.uint8, device=dev)
    else:
        out = torch.empty((info.height, info.width), dtype=torch.int32, device=dev)
    plan = Plan(ctx, [FrameSpec(info.width, info.height, info.sampling, qt_index=(0, 1, 2), out_format=out_format)],
                IN_Q16_ZIGZAG, qtables=info.qt)
    plan.launch(d_coefs, out, stream)
    return out


class JpegStream:
    """hjd_stream: host Huffman workers -> pinned slots -> H2D -> fused kernel."""

    def __init__(self, ctx, max_blocks: int, nslots: int = 4, nthreads: int = 0, out_format: int = 0):
        self.lib = _lib.load()
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(self.lib.hjd_stream_create(ctx.handle, int(max_blocks), int(nslots), int(nthreads), ctypes.byref(h)),
              "hjd_stream_create")
        self.handle = h
        self._keep = []   # bytes must stay alive until sync
        if out_format:
            self.set_output_format(out_format)

    def set_output_format(self, out_format: int):
        """OUT_BGRX or OUT_BGR24 for subsequent submits."""
        check(self.lib.hjd_stream_set_output_format(self.handle, int(out_format)), "hjd_stream_set_output_format")

    def submit(self, data: bytes, out, out_pitch: Optional[int] = None):
        src, size, keep = _src(data)
        self._keep.append(keep)
        if isinstance(out, int):
            ptr = out
            assert out_pitch, "out_pitch required with a raw pointer"
        else:
            if not (out.is_cuda and out.is_contiguous()):
                raise ValueError("out must be a contiguous device tensor")
            ptr = out.data_ptr()
            out_pitch = out_pitch or out.shape[-1] * out.element_size()
        check(self.lib.hjd_stream_submit(self.handle, src, size, ptr, int(out_pitch)), "hjd_stream_submit")

    def sync(self) -> dict:
        stats = (ctypes.c_int64 * 5)()
        rc = self.lib.hjd_stream_sync(self.handle, stats)
        self._keep.clear()
        check(rc, "hjd_stream_sync")
        h2d_ns, kernel_ns = ctypes.c_int64(0), ctypes.c_int64(0)
        check(self.lib.hjd_stream_busy(self.handle, ctypes.byref(h2d_ns), ctypes.byref(kernel_ns)), "hjd_stream_busy")
        return {"images": stats[0], "pixels": stats[1], "host_decode_ns": stats[2], "h2d_bytes": stats[3],
                "kernel_launches": stats[4], "h2d_busy_ns": h2d_ns.value, "kernel_busy_ns": kernel_ns.value}

    def close(self):
        if self.handle:
            self.lib.hjd_stream_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pinned_bytes(data: bytes):
    """The bytes in a pinned (page-locked) host tensor: JPEGs submitted from
    pinned memory reach the GPU raw and are destuffed there (no host pass over
    the scan; include/hjd_host.h hjd_host_register).  Keep the tensor alive
    until the decoder's / stream's sync()."""
    import torch
    t = torch.empty(len(data), dtype=torch.uint8).pin_memory()
    t.numpy()[:] = np.frombuffer(data, np.uint8)
    return t


def _ptr_size(d):
    """(address, size) of bytes / ctypes array / (pinned) CPU uint8 tensor."""
    if isinstance(d, ctypes.Array):
        return ctypes.addressof(d), len(d), d
    if hasattr(d, "data_ptr") and hasattr(d, "is_cuda"):
        if d.is_cuda or not d.is_contiguous() or d.element_size() != 1:
            raise ValueError("JPEG tensors must be contiguous uint8 host tensors")
        return d.data_ptr(), d.numel(), d
    p, n, keep = _src(d)
    return ctypes.cast(p, ctypes.c_void_p).value or 0, n, keep


def _byte_arrays(datas):
    """(objects to keep alive, uint8* array, size_t array) of the inputs; bytes
    objects take the direct path (a decode call's Python cost is on the
    single-image latency path)."""
    ptrs, sizes, keep = [], [], []
    for d in datas:
        if isinstance(d, bytes):
            p, n, k = _src(d)
        else:
            a, n, k = _ptr_size(d)
            p = ctypes.cast(a, _u8p)
        ptrs.append(p)
        sizes.append(n)
        keep.append(k)
    return keep + ptrs, (_u8p * len(ptrs))(*ptrs), (ctypes.c_size_t * len(sizes))(*sizes)


def _stream_handle(stream):
    if stream is None:
        return None
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


class GpuDecoder:
    """hjd_gdec: JPEG bytes -> Huffman decode on the GPU -> fused pixel kernel.

    The host only parses headers and copies the scans (without byte stuffing)
    into pinned memory; the entropy decode is a verified parallel decode on
    the device, bit-identical to decode_coefs()."""

    def __init__(self, ctx, max_frames: int, max_scan_bytes: int, max_blocks: int, sub_bits: int = 0):
        self.lib = _lib.load()
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(self.lib.hjd_gdec_create(ctx.handle, int(max_frames), int(max_scan_bytes), int(max_blocks),
                                       int(sub_bits), ctypes.byref(h)), "hjd_gdec_create")
        self.handle = h
        self._n = 0

    def set_output_format(self, out_format: int):
        """OUT_BGRX (default) or OUT_BGR24 for the following decode() calls."""
        check(self.lib.hjd_gdec_set_output_format(self.handle, int(out_format)), "hjd_gdec_set_output_format")

    def decode(self, datas: Sequence[bytes], outs, stream=None):
        """outs: contiguous device tensors, one row per image row: (H, W) int32
        (or (H, pitch/4)) for BGRX, (H, pitch) uint8 for BGR24."""
        _keep, arr_d, arr_s = _byte_arrays(datas)
        n = len(datas)
        if len(outs) != n:
            raise ValueError("one output per JPEG")
        for o in outs:
            if not (o.is_cuda and o.is_contiguous()):
                raise ValueError("outputs must be contiguous device tensors")
        ptrs = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
        pitches = (ctypes.c_int32 * n)(*[o.shape[-1] * o.element_size() for o in outs])
        check(self.lib.hjd_gdec_decode(self.handle, arr_d, arr_s, n, ptrs, pitches, _stream_handle(stream)),
              "hjd_gdec_decode")
        self._n = n

    def decode_coefs(self, datas: Sequence[bytes], coefs, stream=None) -> List[int]:
        """Entropy decode only into `coefs` (int16 device tensor, [blocks][64]);
        returns each frame's first block."""
        _keep, arr_d, arr_s = _byte_arrays(datas)
        n = len(datas)
        if not (coefs.is_cuda and coefs.is_contiguous() and coefs.element_size() == 2):
            raise ValueError("coefs must be a contiguous int16 device tensor")
        offs = (ctypes.c_int64 * n)()
        check(self.lib.hjd_gdec_decode_coefs(self.handle, arr_d, arr_s, n, coefs.data_ptr(), offs,
                                             _stream_handle(stream)), "hjd_gdec_decode_coefs")
        self._n = n
        return list(offs)

    def last_bytes(self) -> dict:
        """Bytes of the most recent decode call: scan bytes the host CPU
        read + wrote (0 when every scan was destuffed on the GPU) and bytes
        moved host -> device."""
        hb, h2d = ctypes.c_int64(0), ctypes.c_int64(0)
        check(self.lib.hjd_gdec_last_bytes(self.handle, ctypes.byref(hb), ctypes.byref(h2d)), "hjd_gdec_last_bytes")
        return {"host_scan_bytes": hb.value, "h2d_bytes": h2d.value}

    def sync(self, raise_on_error: bool = True) -> List[int]:
        """Wait for the last call; per-frame status words (include/hjd_host.h:
        bit 0 HJD_GDEC_SEQUENTIAL is informational, a sequential verification
        or a chain repair; bits 1-2 are errors and raise unless
        raise_on_error is False)."""
        status = (ctypes.c_int32 * max(self._n, 1))()
        rc = self.lib.hjd_gdec_sync(self.handle, status)
        if raise_on_error:
            check(rc, "hjd_gdec_sync")
        return list(status)[: self._n]

    def close(self):
        if self.handle:
            self.lib.hjd_gdec_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GpuJpegStream:
    """hjd_gstream: worker threads parse/destuff JPEGs into pinned batches;
    each batch is Huffman-decoded and converted to BGRX on the GPU."""

    def __init__(self, ctx, max_frames: int, max_scan_bytes: int, max_blocks: int, nslots: int = 3,
                 nthreads: int = 0, out_format: int = 0):
        self.lib = _lib.load()
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(self.lib.hjd_gstream_create(ctx.handle, int(max_frames), int(max_scan_bytes), int(max_blocks),
                                          int(nslots), int(nthreads), ctypes.byref(h)), "hjd_gstream_create")
        self.handle = h
        self._keep = []
        if out_format:
            self.set_output_format(out_format)

    def set_output_format(self, out_format: int):
        """OUT_BGRX or OUT_BGR24 (between sync() and the next submit)."""
        check(self.lib.hjd_gstream_set_output_format(self.handle, int(out_format)), "hjd_gstream_set_output_format")

    def submit(self, data: bytes, out, out_pitch: Optional[int] = None):
        """out: contiguous device tensor, or a (pinned) host tensor / numpy
        array -- then the pixels are copied back to host memory (D2H sink)."""
        addr, size, keep = _ptr_size(data)
        self._keep.append(keep)
        src = ctypes.cast(addr, _u8p)
        if isinstance(out, np.ndarray):
            if not out.flags.c_contiguous:
                raise ValueError("out must be C-contiguous")
            self._keep.append(out)
            pitch = out_pitch or out.shape[-1] * out.itemsize
            check(self.lib.hjd_gstream_submit_host(self.handle, src, size, out.ctypes.data, int(pitch)),
                  "hjd_gstream_submit_host")
            return
        if not out.is_contiguous():
            raise ValueError("out must be contiguous")
        out_pitch = out_pitch or out.shape[-1] * out.element_size()
        if out.is_cuda:
            check(self.lib.hjd_gstream_submit(self.handle, src, size, out.data_ptr(), int(out_pitch)),
                  "hjd_gstream_submit")
        else:
            self._keep.append(out)
            check(self.lib.hjd_gstream_submit_host(self.handle, src, size, out.data_ptr(), int(out_pitch)),
                  "hjd_gstream_submit_host")

    def sync(self) -> dict:
        stats = (ctypes.c_int64 * 5)()
        rc = self.lib.hjd_gstream_sync(self.handle, stats)
        self._keep.clear()
        check(rc, "hjd_gstream_sync")
        hb = ctypes.c_int64(0)
        check(self.lib.hjd_gstream_host_bytes(self.handle, ctypes.byref(hb)), "hjd_gstream_host_bytes")
        return {"images": stats[0], "pixels": stats[1], "host_prep_ns": stats[2], "h2d_bytes": stats[3],
                "batches": stats[4], "host_scan_bytes": hb.value}

    def close(self):
        if self.handle:
            self.lib.hjd_gstream_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bmp_header(width: int, height: int, bpp: int = 32) -> bytes:
    """The reference's 54-byte BMP header (src/decoder.cpp:372-394): 32 bpp,
    top-down; bpp=24 gives the 24-bpp counterpart (rows padded to 4 bytes)."""
    lib = _lib.load()
    h = (ctypes.c_uint8 * 54)()
    if bpp == 32:
        check(lib.hjd_bmp_header(int(width), int(height), h), "hjd_bmp_header")
    elif bpp == 24:
        check(lib.hjd_bmp_header_bgr24(int(width), int(height), h), "hjd_bmp_header_bgr24")
    else:
        raise ValueError("bpp must be 32 or 24")
    return bytes(h)


def bmp_bytes(pixels, width: Optional[int] = None) -> bytes:
    """A BMP file from decoded pixels, as the reference writes it from the GPU
    path: an (H, W) array of BGRX words gives the reference's 32-bpp file; an
    (H, pitch) uint8 array of BGR24 rows (pitch = (3W+3)&~3, as decode_jpeg
    returns with OUT_BGR24) gives the 24-bpp file (width W required)."""
    a = np.ascontiguousarray(pixels)
    if a.dtype == np.uint8:
        if width is None or a.shape[1] != (3 * width + 3) & ~3:
            raise ValueError("BGR24 rows need width and pitch (3*width+3)&~3")
        return bmp_header(width, a.shape[0], 24) + a.tobytes()
    a = a.view(np.uint32)
    return bmp_header(a.shape[1], a.shape[0]) + a.astype("<u4").tobytes()


def emulate_entropy(data: bytes, sub_bits: int = 0):
    """Test hook: the GPU entropy algorithm run on the host (no GPU) ->
    (int16 [nblocks][64] coefficients, status bits)."""
    lib = _lib.load()
    info = parse(data)
    coefs = np.zeros((info.nblocks, 64), np.int16)
    status = ctypes.c_int32(0)
    check(lib.hjd_debug_entropy_emulate(_buf(data), len(data), int(sub_bits), coefs.ctypes.data_as(_i16p),
                                        info.nblocks, ctypes.byref(status)), "hjd_debug_entropy_emulate")
    return coefs, status.value
