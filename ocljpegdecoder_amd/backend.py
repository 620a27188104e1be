"""Python host API over the C ABI (include/hjd.h).

PyTorch is used only as plumbing: device memory (tensors), streams.  All pixel
work runs in the HIP kernels of libhjd.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import HjdFrame, check

YUV444 = 0
YUV420 = 1  # == the reference's ColorSpace::YUV411 (src/macro.h:114-119), H2V2
OTHER = 2
YUV422 = 3  # extension (Y H2V1), include/hjd.h
GRAY = 4    # extension (one component), include/hjd.h
YUV411_H4V1 = 5  # extension (Y H4V1: true 4:1:1, not the reference's "YUV411"), include/hjd.h
YUV440 = 6  # extension (Y H1V2), include/hjd.h

# sampling -> (MCU px width, MCU px height, blocks per MCU, luma blocks per MCU)
_GEOM = {YUV444: (8, 8, 3, 1), YUV420: (16, 16, 6, 4), YUV422: (16, 8, 4, 2), GRAY: (8, 8, 1, 1),
         YUV411_H4V1: (32, 8, 6, 4), YUV440: (8, 16, 4, 2)}

IN_Q16_ZIGZAG = 0
IN_I32_NATURAL = 1

KERNEL_AUTO, KERNEL_PERSISTENT, KERNEL_LATENCY = 0, 1, 2   # include/hjd.h hjd_kernel_mode

OUT_BGRX = 0    # 4 B/px: B, G, R, 0 (the reference's RGB32 / 32-bpp BMP rows)
OUT_BGR24 = 1   # 3 B/px: B, G, R (extension: 24-bpp BMP rows)
OUT_BYTES = {OUT_BGRX: 4, OUT_BGR24: 3}


def default_pitch(width: int, out_format: int = OUT_BGRX) -> int:
    """Tightest legal row pitch: bytes of one row rounded up to 4."""
    return (OUT_BYTES[out_format] * width + 3) & ~3


def mcu_geometry(width: int, height: int, sampling: int):
    """(mcu_w, mcu_h, blocks_per_mcu, (mcu_px_w, mcu_px_h)) -- src/decoder.cpp:161-192."""
    if sampling not in _GEOM:
        raise ValueError(f"unsupported sampling {sampling}")
    pw, ph, bpm, _ = _GEOM[sampling]
    return (width - 1) // pw + 1, (height - 1) // ph + 1, bpm, (pw, ph)


def block_components(sampling: int, nblocks: int) -> np.ndarray:
    """Component (0 Y, 1 Cb, 2 Cr) of each block of an MCU-major block list."""
    _, _, bpm, nluma = _GEOM[sampling]
    return np.array(([0] * nluma + [1, 2][: bpm - nluma]) * (nblocks // bpm), dtype=np.int64)


def frame_blocks(width: int, height: int, sampling: int) -> int:
    mw, mh, bpm, _ = mcu_geometry(width, height, sampling)
    return mw * mh * bpm


def device_count() -> int:
    lib = _lib.load()
    n = ctypes.c_int32(0)
    check(lib.hjd_device_count(ctypes.byref(n)), "hjd_device_count")
    return n.value


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class Context:
    """One device (hjd_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        check(self.lib.hjd_ctx_create(device, ctypes.byref(h)), "hjd_ctx_create")
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self.lib.hjd_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- kernels outside a plan -------------------------------------------------
    def idct_blocks(self, d_in, d_out, nblocks: int, stream=None):
        """IDCT only (int32 natural in -> int32 samples), tensors on this device."""
        for t in (d_in, d_out):
            if not (t.is_cuda and t.is_contiguous() and t.element_size() == 4 and t.numel() >= 64 * nblocks):
                raise ValueError("idct_blocks needs contiguous int32 device tensors of >= 64*nblocks elements")
        check(self.lib.hjd_idct_blocks(self.handle, d_in.data_ptr(), d_out.data_ptr(), int(nblocks),
                                       _stream_ptr(stream)), "hjd_idct_blocks")

    def debug_csc(self, y, u, v, out, mode: int = 0, stream=None):
        for t in (y, u, v, out):
            if not (t.is_cuda and t.is_contiguous() and t.element_size() == 4 and t.numel() >= y.numel()):
                raise ValueError("debug_csc needs contiguous 4-byte device tensors of equal length")
        check(self.lib.hjd_debug_csc(self.handle, y.data_ptr(), u.data_ptr(), v.data_ptr(), out.data_ptr(),
                                     y.numel(), mode, _stream_ptr(stream)), "hjd_debug_csc")

    def debug_csc_exhaustive(self, out, mode: int = 0, stream=None):
        assert out.numel() * out.element_size() >= 4 << 27
        check(self.lib.hjd_debug_csc_exhaustive(self.handle, out.data_ptr(), mode, _stream_ptr(stream)),
              "hjd_debug_csc_exhaustive")

    def debug_rw_mix(self, src, dst, read_kib: int, write_kib: int, units_per_wave: int = 2, flags: int = 3,
                     stream=None) -> int:
        """The box's streaming ceiling kernel (hjd_debug_rw_mix): one launch;
        returns the bytes it moves (read + written)."""
        for t in (src, dst):
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError("debug_rw_mix needs contiguous device tensors")
        units = ctypes.c_int64(0)
        check(self.lib.hjd_debug_rw_mix(self.handle, src.data_ptr(), dst.data_ptr(), src.numel() * src.element_size(),
                                        dst.numel() * dst.element_size(), int(read_kib), int(write_kib),
                                        int(units_per_wave), int(flags), _stream_ptr(stream), ctypes.byref(units)),
              "hjd_debug_rw_mix")
        return units.value * (read_kib + write_kib) * 1024

    def clock_probe(self, out, nsamples: int, interval_ticks: int, stream=None):
        """Launch the clock probe (hjd_debug_clock_probe) writing 2*nsamples
        int64 words into `out` (a device tensor); see clock_summary()."""
        if not (out.is_cuda and out.is_contiguous() and out.element_size() == 8 and out.numel() >= 2 * nsamples):
            raise ValueError("clock_probe needs a contiguous int64 device tensor of >= 2*nsamples elements")
        check(self.lib.hjd_debug_clock_probe(self.handle, out.data_ptr(), int(nsamples), int(interval_ticks),
                                             _stream_ptr(stream)), "hjd_debug_clock_probe")

    def d16_gather(self):
        """(probe_zeroes, selected) of hjd_debug_d16_gather for this device."""
        a, b = ctypes.c_int32(-1), ctypes.c_int32(-1)
        check(self.lib.hjd_debug_d16_gather(self.device, ctypes.byref(a), ctypes.byref(b)), "hjd_debug_d16_gather")
        return bool(a.value), bool(b.value)


@dataclass
class FrameSpec:
    width: int
    height: int
    sampling: int
    coef_offset: int = 0          # in blocks
    out_offset: int = 0           # bytes
    out_pitch: int = 0            # bytes (0 -> default_pitch(width, out_format))
    qt_index: Sequence[int] = field(default_factory=lambda: (0, 1, 1))
    out_format: int = OUT_BGRX

    @property
    def pitch(self) -> int:
        return self.out_pitch or default_pitch(self.width, self.out_format)

    def to_c(self) -> HjdFrame:
        f = HjdFrame()
        f.coef_offset = self.coef_offset
        f.out_offset = self.out_offset
        f.width = self.width
        f.height = self.height
        f.out_pitch = self.pitch
        f.sampling = self.sampling
        for i in range(3):
            f.qt_index[i] = int(self.qt_index[i])
        f.out_format = self.out_format
        return f


class Plan:
    """A validated batch of frames with its device-side frame table (hjd_plan)."""

    def __init__(self, ctx: Context, frames: Sequence[FrameSpec], input_format: int = IN_Q16_ZIGZAG,
                 qtables: Optional[np.ndarray] = None):
        self.ctx = ctx
        self.lib = ctx.lib
        self.frames = list(frames)
        arr = (HjdFrame * max(1, len(self.frames)))(*[f.to_c() for f in self.frames])
        if qtables is not None:
            q = np.ascontiguousarray(qtables, dtype=np.int32).reshape(-1, 64)
            qp, nq = q.ctypes.data_as(_lib.c_i32p), q.shape[0]
        else:
            q, qp, nq = None, None, 0
        h = ctypes.c_void_p()
        check(self.lib.hjd_plan_create(ctx.handle, arr, len(self.frames), input_format, qp, nq, ctypes.byref(h)),
              "hjd_plan_create")
        self.handle = h
        self.input_format = input_format
        self.tasks = self.lib.hjd_plan_tasks(h)
        self.pixels = self.lib.hjd_plan_pixels(h)
        self.coef_bytes = self.lib.hjd_plan_coef_bytes(h)
        # extents the kernel will touch: validated against the tensors at launch
        self.coef_elem_bytes = 2 if input_format == IN_Q16_ZIGZAG else 4
        self.coef_elems_needed = max([64 * (f.coef_offset + frame_blocks(f.width, f.height, f.sampling))
                                      for f in self.frames] or [0])
        self.out_bytes_needed = max([f.out_offset + (f.height - 1) * f.pitch + OUT_BYTES[f.out_format] * f.width
                                     for f in self.frames] or [0])

    def _check_tensor(self, t, what, elem_bytes, nbytes_needed):
        if isinstance(t, int):
            return t                       # raw device pointer: caller's responsibility
        if not t.is_cuda:
            raise ValueError(f"{what} must be a device tensor")
        if not t.is_contiguous():
            raise ValueError(f"{what} must be contiguous")
        if elem_bytes and t.element_size() != elem_bytes:
            raise ValueError(f"{what} must have {elem_bytes}-byte elements for this plan, got {t.dtype}")
        if t.numel() * t.element_size() < nbytes_needed:
            raise ValueError(f"{what} too small: {t.numel() * t.element_size()} B < {nbytes_needed} B")
        if t.device.index != self.ctx.device:
            raise ValueError(f"{what} is on {t.device}, plan is for device {self.ctx.device}")
        return t.data_ptr()

    def set_kernel(self, mode: int):
        """KERNEL_AUTO (default), KERNEL_PERSISTENT or KERNEL_LATENCY; identical outputs."""
        check(self.lib.hjd_plan_set_kernel(self.handle, int(mode)), "hjd_plan_set_kernel")

    def set_chunk(self, tasks: int):
        """Pin the persistent kernel's tasks per wave (hjd_plan_set_chunk); 0 = default."""
        check(self.lib.hjd_plan_set_chunk(self.handle, int(tasks)), "hjd_plan_set_chunk")

    def set_variant(self, variant: int):
        """Kernel variant bits (tuning/A-B only; outputs are identical)."""
        check(self.lib.hjd_plan_set_variant(self.handle, int(variant)), "hjd_plan_set_variant")

    def launch(self, coefs, out, stream=None, grid_blocks: int = 0):
        """Enqueue the fused kernel; coefs/out are device tensors (or raw pointers)."""
        cp = self._check_tensor(coefs, "coefs", self.coef_elem_bytes, self.coef_elems_needed * self.coef_elem_bytes)
        op = self._check_tensor(out, "out", 0, self.out_bytes_needed)
        check(self.lib.hjd_plan_launch(self.handle, cp, op, _stream_ptr(stream), grid_blocks), "hjd_plan_launch")

    def autotune(self, coefs, out, stream=None, rounds: int = 2):
        """hjd_plan_autotune: time the launch shapes on these buffers and keep
        the fastest for later launches; returns (tasks_per_wave, variant).
        The choice is cached per process by kernel and batch geometry
        (include/hjd.h): on a cache hit nothing is launched and `out` is NOT
        written -- call launch() for a decode (launch_shape()["autotune_cached"]
        tells which happened)."""
        cp = self._check_tensor(coefs, "coefs", self.coef_elem_bytes, self.coef_elems_needed * self.coef_elem_bytes)
        op = self._check_tensor(out, "out", 0, self.out_bytes_needed)
        tpw, var = ctypes.c_int32(0), ctypes.c_int32(0)
        check(self.lib.hjd_plan_autotune(self.handle, cp, op, _stream_ptr(stream), int(rounds), ctypes.byref(tpw),
                                         ctypes.byref(var)), "hjd_plan_autotune")
        return tpw.value, var.value

    def launch_shape(self) -> dict:
        """hjd_plan_launch_shape: the shape the next default launch uses, and
        what the last autotune did (launches made, cache hit)."""
        r = _lib.HjdLaunchShape()
        check(self.lib.hjd_plan_launch_shape(self.handle, ctypes.byref(r)), "hjd_plan_launch_shape")
        d = {n: getattr(r, n) for n, _ in r._fields_}
        d["kernel"] = {KERNEL_PERSISTENT: "persistent", KERNEL_LATENCY: "latency"}.get(d["kernel"], d["kernel"])
        return d

    def launch_stages(self, stages: int, coefs, out, stream=None, grid_blocks: int = 0):
        """Timing-only launch with kernel stages skipped (hjd_debug_plan_launch_stages;
        80 memory only, 4 no stores, ...): the output is WRONG by design."""
        cp = self._check_tensor(coefs, "coefs", self.coef_elem_bytes, self.coef_elems_needed * self.coef_elem_bytes)
        op = self._check_tensor(out, "out", 0, self.out_bytes_needed)
        check(self.lib.hjd_debug_plan_launch_stages(self.handle, int(stages), cp, op, _stream_ptr(stream),
                                                    int(grid_blocks)),
              "hjd_debug_plan_launch_stages")

    def close(self):
        if self.handle:
            self.lib.hjd_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def worker_cpus(bus: str, gpus: Sequence[str], sysfs_root: Optional[str] = None, only_allowed: bool = False):
    """hjd_debug_worker_cpus: the host CPUs the worker pool of the GPU at PCI
    address `bus` binds to, among the GPUs `gpus` (its NUMA node's CPUs split
    per GPU of that node), from the sysfs tree at `sysfs_root` (None: the real one)."""
    lib = _lib.load()
    arr = (ctypes.c_char_p * max(1, len(gpus)))(*[g.encode() for g in gpus])
    cap = 4096
    out = (ctypes.c_int32 * cap)()
    n = ctypes.c_int32(0)
    check(lib.hjd_debug_worker_cpus(sysfs_root.encode() if sysfs_root else None, bus.encode(), arr, len(gpus),
                                    int(only_allowed), out, cap, ctypes.byref(n)), "hjd_debug_worker_cpus")
    return list(out[:min(n.value, cap)])


def device_worker_cpus(device: int):
    """hjd_device_worker_cpus: the host CPUs the stream workers of HIP device
    `device` bind to (its share of its NUMA node; [] = unknown topology)."""
    lib = _lib.load()
    if getattr(lib, "hjd_device_worker_cpus", None) is None:   # an older HJD_LIB tuning build
        return []
    cap = 4096
    out = (ctypes.c_int32 * cap)()
    n = ctypes.c_int32(0)
    check(lib.hjd_device_worker_cpus(int(device), out, cap, ctypes.byref(n)), "hjd_device_worker_cpus")
    return list(out[:min(n.value, cap)])


def cpu_share(root: Optional[str] = None) -> int:
    """hjd_host_cpu_share (root None) or hjd_debug_cpu_share on a fake tree:
    affinity CPUs capped by the cgroup's CPU quota."""
    lib = _lib.load()
    return lib.hjd_host_cpu_share() if root is None else lib.hjd_debug_cpu_share(root.encode())


def stream_worker_threads(share: int, world: int, slice_cpus: int) -> int:
    """Host worker threads per GPU of a multi-rank stream job (bench.py config
    5): the process's CPU share split over the ranks on the host, capped by the
    GPU's CPU slice when the topology is known (every logical CPU of the slice:
    SMT pays for the Huffman decode, profiles/r06a_smt_probe.json)."""
    per_rank = max(1, share // max(1, world))
    return min(per_rank, slice_cpus) if slice_cpus > 0 else per_rank


def autotune_cache_clear():
    """Forget every cached hjd_plan_autotune choice of this process."""
    check(_lib.load().hjd_autotune_cache_clear(), "hjd_autotune_cache_clear")


def decode_frame(ctx: Context, coefs, qt: np.ndarray, width: int, height: int, sampling: int,
                 input_format: int = IN_Q16_ZIGZAG, stream=None):
    """Decode one frame already resident on the device; returns an int32 (H, W)
    device tensor holding BGRX words (0x00RRGGBB)."""
    import torch
    plan = Plan(ctx, [FrameSpec(width, height, sampling, qt_index=(0, 1, 2))], input_format,
                qtables=qt if input_format == IN_Q16_ZIGZAG else None)
    out = torch.empty((height, width), dtype=torch.int32, device=coefs.device)
    plan.launch(coefs, out, stream)
    return out, plan
