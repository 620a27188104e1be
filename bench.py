#!/usr/bin/env python3
"""bench.py -- fused dequant + IDCT + upsample + colour kernel on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 4k420|4k444|fhd420]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Workload (BASELINE.json configs[2], default): a batch of 1024 synthetic
3840x2160 4:2:0 frames resident in HBM as int16 quantised zigzag coefficients
(+ qtables); one step = ONE persistent-kernel launch decoding all 1024 frames to
BGRX in HBM.  Synthetic content: a pool of distinct frames (FDCT + quantisation
of smooth+noise blocks, generated on the device) replicated to 1024 frames.
Multi-GPU: every rank decodes its own 1024-frame batch (image-parallel shards,
no collective on the data path; weak scaling); value = all ranks' pixels /
max-over-ranks time.

Printed JSON line fields beyond the driver contract:
  roofline      achieved GB/s = algorithmic bytes per launch (int16 coefs in +
                BGRX out, 7 B/px at 4:2:0, 10 B/px at 4:4:4) / mean launch time
                measured with HIP events on the launch stream; peak 8.0 TB/s.
                traffic = per-launch HBM bytes from the committed rocprofv3 PMC
                summary (profiles/*pmc*.json), or null.
  cpu_baseline  the bit-exact C restatement (oracle/) on a thread pool over the
                host cores, one frame per task, bounded sample (rank 0, N=1);
                cpu_reference = the reference's own decode_mcu_data
                (oracle/_ref/libref.so, 1 thread) when that library is present.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import socket
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# JPEG zigzag: natural index of zigzag position k (src/zigzag.h)
ZIGZAG_NAT = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,
              7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
              39, 46, 53, 60, 61, 54, 47, 55, 62, 63]

WORKLOADS = {
    "4k420": dict(width=3840, height=2160, sampling=1, frames=1024,
                  desc="BASELINE configs[2]: batch of 1024 synthetic 3840x2160 4:2:0 frames, persistent kernel"),
    "4k444": dict(width=3840, height=2160, sampling=0, frames=1024,
                  desc="BASELINE configs[3]: batch of 1024 synthetic 3840x2160 4:4:4 frames, persistent kernel"),
    "4k422": dict(width=3840, height=2160, sampling=3, frames=1024,
                  desc="extension (SURVEY s8(f) rank 4): batch of 1024 synthetic 3840x2160 4:2:2 frames"),
    "4kgray": dict(width=3840, height=2160, sampling=4, frames=1024,
                   desc="extension (SURVEY s8(f) rank 4): batch of 1024 synthetic 3840x2160 grayscale frames"),
    "4k411": dict(width=3840, height=2160, sampling=5, frames=1024,
                  desc="extension: batch of 1024 synthetic 3840x2160 4:1:1 (Y H4V1) frames"),
    "4k440": dict(width=3840, height=2160, sampling=6, frames=1024,
                  desc="extension: batch of 1024 synthetic 3840x2160 4:4:0 (Y H1V2) frames"),
    "4k420_bgr24": dict(width=3840, height=2160, sampling=1, frames=1024, out_format=1,
                        desc="extension (SURVEY s8(f) rank 4): configs[2] with 3-byte BGR24 output (24-bpp BMP "
                             "rows) instead of BGRX"),
    "4k420_i32": dict(width=3840, height=2160, sampling=1, frames=1024, input="i32",
                      desc="configs[2] in the idct.h-compat input format (SURVEY s8(d)): int32 natural-order "
                           "dequantised blocks (jpg.mcu_data, src/jpeg.h:76), 10 B/px"),
    "4k444_i32": dict(width=3840, height=2160, sampling=0, frames=1024, input="i32",
                      desc="configs[3] in the idct.h-compat input format: int32 natural-order dequantised "
                           "blocks, 16 B/px"),
    "fhd420_jpeg": dict(width=1920, height=1080, sampling=1, frames=1, jpeg=True,
                        desc="BASELINE configs[1] end to end: one 1920x1080 4:2:0 q90 JPEG per step, bytes in host "
                             "memory -> BGRX in HBM (GPU Huffman decode + fused kernel), latency per image"),
    "fhd420": dict(width=1920, height=1080, sampling=1, frames=1,
                   desc="BASELINE configs[1]: single 1920x1080 4:2:0 frame, one launch (cache/launch bound)"),
    "stream4k420": dict(width=3840, height=2160, sampling=1, frames=1024, entropy="gpu",
                        desc="BASELINE configs[4] per GPU: stream of 4K 4:2:0 JPEGs (pool of 64 distinct q90 "
                             "files in pinned memory); host header parse || raw-scan DMA || GPU destuff + Huffman "
                             "decode + fused kernel"),
    "stream4k420_d2h": dict(width=3840, height=2160, sampling=1, frames=256, entropy="gpu", d2h=True,
                            desc="BASELINE configs[4] per GPU, D2H-on (SURVEY s8(e)): as stream4k420, and every "
                                 "frame's BGRX copied back to pinned host memory"),
    "stream4k420_d2h_bgr24": dict(width=3840, height=2160, sampling=1, frames=256, entropy="gpu", d2h=True,
                                  out_format=1,
                                  desc="BASELINE configs[4] per GPU, D2H-on, BGR24 sink (SURVEY s8(f) rank 4): as "
                                       "stream4k420_d2h with 3-byte pixels copied back"),
    "stream4k420_host": dict(width=3840, height=2160, sampling=1, frames=128, entropy="host",
                             desc="BASELINE configs[4] per GPU as north_star names it: host Huffman workers "
                                  "(jpeg_host.cpp) -> pinned int16 coefficient slots -> hipMemcpyAsync on a copy "
                                  "stream || fused kernel on a compute stream"),
}
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
POOL = 8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def std_qtables(scale=1.0):
    lum = np.array([16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                    14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99])
    chr_ = np.array([17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                     24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32)
    nat = np.stack([lum, chr_, chr_])
    return np.clip(np.rint(nat[:, ZIGZAG] * scale), 1, 255).astype(np.int32)


ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


SAMPLING_NAMES = {0: "4:4:4", 1: "4:2:0", 3: "4:2:2", 4: "gray", 5: "4:1:1", 6: "4:4:0"}


def synth_frame_gpu(torch, nblk, sampling, qt, seed, device):
    """Synthetic quantised zigzag coefficients for one frame, on the device:
    smooth+noise 8x8 sample blocks in [-128,127] -> float FDCT -> quantise
    (q=90-like tables).  Bounded samples keep the data in the reference's legal
    domain.  This is input generation, outside every timed region."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    k = torch.arange(8, device=device, dtype=torch.float32)
    cc = torch.where(k == 0, 1 / np.sqrt(2), 1.0)
    m = torch.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16) * cc[:, None] / 2
    yy, xx = torch.meshgrid(torch.arange(8, device=device), torch.arange(8, device=device), indexing="ij")
    base = torch.randint(-100, 100, (nblk, 1, 1), generator=g, device=device).float()
    grad = torch.randn((nblk, 2, 1, 1), generator=g, device=device) * 6
    pix = base + grad[:, 0] * yy + grad[:, 1] * xx + torch.randn((nblk, 8, 8), generator=g, device=device) * 20
    pix = pix.clamp(-128, 127)
    F = torch.einsum("ux,nxy,vy->nuv", m, pix, m).reshape(nblk, 64)
    qnat = torch.zeros((3, 64), device=device)
    qnat[:, torch.tensor(ZIGZAG, device=device)] = torch.from_numpy(qt).float().to(device)
    import ocljpegdecoder_amd as hjd
    comp = torch.from_numpy(hjd.block_components(sampling, nblk)).to(device)
    coef_nat = torch.round(F / qnat[comp])
    return coef_nat[:, torch.tensor(ZIGZAG, device=device)].to(torch.int16).contiguous()


def host_cpu_share():
    """(threads to use, logical CPUs in the affinity mask, cgroup CPU quota or None, nproc).

    A one-GPU box shows all 256 logical CPUs of the node (os.cpu_count(), the
    affinity mask) but its cgroup grants 16 CPUs of time (cpu.max 1600000/100000,
    profiles/r02_gpu_box_host_probe.txt) and `nproc` says 16: more threads than
    the quota only time-slice the same 16 CPUs (measured: `all_logical_cpus`)."""
    import math
    import subprocess
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout)
    except Exception:
        nproc = None
    share = min(aff, math.ceil(quota)) if quota else aff
    return share, aff, quota, nproc


def _port_rate(lib, O, pool, q, w, h, s, nframes, nthreads):
    stride = pool.shape[1] * 64
    out = np.empty((nthreads, h * w), dtype=np.uint32)
    t0 = time.perf_counter()
    rc = lib.oracle_decode_batch_q16_mt(pool.ctypes.data_as(O.i16p), stride, pool.shape[0],
                                        q[0].ctypes.data_as(O.i32p), q[1].ctypes.data_as(O.i32p),
                                        q[2].ctypes.data_as(O.i32p), w, h, s,
                                        out.ctypes.data_as(O.u32p), h * w, nframes, nthreads)
    dt = time.perf_counter() - t0
    assert rc == 0
    return nframes * w * h / dt / 1e6, dt


def host_huffman_rate(hjd, w, h, s, nthreads):
    """Host Huffman (csrc/jpeg_host.cpp, the config-5 host bound of SURVEY s8(d)):
    Mpx/s on 1 thread and on `nthreads` threads, q90 synthetic files of this shape."""
    if s not in (0, 1):
        return None
    pool = encode_pool(w, h, s, 2, seed0=99)
    res = {"sample": f"2 Pillow q90 {w}x{h} {SAMPLING_NAMES[s]} files (gradient + sigma-20 noise), "
                     f"hjd_jpeg_decode_batch -> int16 coefficients in RAM (preallocated), 4 files per thread",
           "mean_jpeg_bytes":
           int(np.mean([len(d) for d in pool]))}
    nblocks = hjd.parse(pool[0]).nblocks
    outs = [np.ones((nblocks, 64), np.int16) for _ in range(4 * nthreads)]   # touched: no page faults timed
    for key, nt, reps in (("one_thread_Mpx_s", 1, 4), ("all_threads_Mpx_s", nthreads, 4 * nthreads)):
        datas = [pool[i % 2] for i in range(reps)]
        hjd.decode_coefs_batch(datas[:2], nthreads=1, outs=outs[:2])
        t0 = time.perf_counter()
        hjd.decode_coefs_batch(datas, nthreads=nt, outs=outs[:reps])
        res[key] = round(reps * w * h / (time.perf_counter() - t0) / 1e6, 1)
    res["threads"] = nthreads
    return res


def cpu_baseline(coef_pool_host, qt, wl, frames_done_gpu_rate):
    """CPU leg (rank 0, N=1): oracle C restatement on a pthread pool over the
    host CPUs this process is granted (one frame per task), bounded sample; a
    1-thread figure; the host-Huffman rate; plus the reference's own
    decode_mcu_data (1 thread)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py as O
    import ocljpegdecoder_amd as hjd
    lib = O.oracle()
    w, h, s = wl["width"], wl["height"], wl["sampling"]
    share, aff, quota, nproc = host_cpu_share()
    nthreads = int(os.environ.get("HJD_CPU_THREADS", share))
    pool = np.ascontiguousarray(coef_pool_host)
    q = np.ascontiguousarray(qt, np.int32)
    # ~20 frames per thread: ~10-30 s of CPU work at ~0.05-0.15 s per 4K frame
    nframes = 20 * nthreads
    rate, dt = _port_rate(lib, O, pool, q, w, h, s, nframes, nthreads)
    rate1, dt1 = _port_rate(lib, O, pool, q, w, h, s, 12, 1)
    res = {"value": round(rate, 2), "unit": "Mpixels/s", "cores": nthreads, "kind": "port",
           "sample": f"{nframes} frames {w}x{h} {SAMPLING_NAMES[s]} (pool of {pool.shape[0]}), "
                     f"int16 zigzag -> BGRX in RAM, {nthreads} threads, {dt:.2f} s wall",
           "one_thread": {"value": round(rate1, 2), "unit": "Mpixels/s", "cores": 1,
                          "sample": f"12 frames, 1 thread, {dt1:.2f} s"},
           "cpu_model": _cpu_model(), "nproc": nproc, "logical_cpus": aff, "cgroup_cpu_quota": quota,
           "threads_rule": "threads = the process's CPU share: min(affinity CPUs, cgroup cpu.max quota); "
                           "equals nproc on the GPU box"}
    if aff > nthreads and "HJD_CPU_THREADS" not in os.environ:
        rate_all, dt_all = _port_rate(lib, O, pool, q, w, h, s, 2 * aff, aff)
        res["all_logical_cpus"] = {"value": round(rate_all, 2), "unit": "Mpixels/s", "threads": aff,
                                   "sample": f"{2 * aff} frames on {aff} threads, {dt_all:.2f} s (bounded by the "
                                             f"cgroup quota, not by the thread count)"}
    try:
        res["host_huffman"] = host_huffman_rate(hjd, w, h, s, nthreads)
    except Exception as e:  # pragma: no cover (Pillow missing)
        res["host_huffman"] = {"error": str(e)}
    if O.ref_available() and s in (0, 1):   # the reference rejects other samplings
        try:
            lib_ref = O.ref()
            lib_ref.ref_decode_mcu_data.argtypes = [O.i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
            nat = O.dequant_natural(pool[0], q, s)
            reps, t_sum = 3, 0.0
            cwd = os.getcwd()
            tmp = tempfile.mkdtemp(prefix="hjd_refbench_")
            try:
                os.chdir(tmp)
                for _ in range(reps):
                    buf = nat.copy()
                    t0 = time.perf_counter()
                    lib_ref.ref_decode_mcu_data(buf.ctypes.data_as(O.i32p), w, h, s)
                    t_sum += time.perf_counter() - t0
            finally:
                os.chdir(cwd)
            one = {"value": round(reps * w * h / t_sum / 1e6, 2), "unit": "Mpixels/s", "cores": 1,
                   "sample": f"{reps} x decode_mcu_data (src/decoder.cpp:397, USE_CPU_ONLY, incl. its "
                             f"BMP fwrite to a temp dir) on one {w}x{h} frame, 1 thread"}
            res["reference"] = reference_multicore(O, pool, q, w, h, s, nthreads)
            res["reference"]["one_thread"] = one
        except Exception as e:  # pragma: no cover
            res["reference"] = {"error": str(e)}
    return res


def reference_multicore(O, pool, q, w, h, s, nworkers, reps=8):
    """The REFERENCE CPU path on all of this process's cores: `nworkers`
    processes (tests/ref_cpu_worker.py), one per core, each running the
    reference's own decode_mcu_data (oracle/_ref/libref.so) on its own pool
    frame in its own temp dir (the reference keeps global state and writes
    its BMP into the cwd, src/decoder.cpp:420).  All workers load their frame
    copies, then start together; Mpx/s = all frames / wall time until the last
    one finishes."""
    import shutil
    import subprocess
    worker = os.path.join(REPO, "tests", "ref_cpu_worker.py")
    tmp = tempfile.mkdtemp(prefix="hjd_refmc_")
    procs = []
    try:
        paths = []
        for i in range(min(pool.shape[0], nworkers)):
            pth = os.path.join(tmp, f"frame{i}.npy")
            np.save(pth, O.dequant_natural(pool[i], q, s))
            paths.append(pth)
        for k in range(nworkers):
            wd = os.path.join(tmp, f"w{k}")
            os.makedirs(wd)
            procs.append(subprocess.Popen([sys.executable, worker, paths[k % len(paths)], str(w), str(h), str(s),
                                           str(reps), wd], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True))
        for p in procs:
            if p.stdout.readline().strip() != "ready":
                raise RuntimeError("reference worker failed to start")
        t0 = time.perf_counter()
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
        outs = [json.loads(p.stdout.readline()) for p in procs]
        wall = time.perf_counter() - t0
        for p in procs:
            p.wait(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        shutil.rmtree(tmp, ignore_errors=True)
    if any("error" in o for o in outs):
        return {"error": [o for o in outs if "error" in o][:2]}
    frames = sum(o["frames"] for o in outs)
    return {"value": round(frames * w * h / wall / 1e6, 2), "unit": "Mpixels/s", "cores": nworkers,
            "kind": "reference", "processes": nworkers,
            "sample": f"{nworkers} processes x {reps} frames {w}x{h} {SAMPLING_NAMES[s]} (pool of {pool.shape[0]}): "
                      f"the reference's own decode_mcu_data (src/decoder.cpp:397-523, USE_CPU_ONLY, incl. its BMP "
                      f"fwrite to each process's temp dir), started together, {wall:.2f} s wall",
            "mean_s_per_frame_per_process": round(sum(o["seconds"] for o in outs) / frames, 4)}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def check_batch_vs_oracle(torch, out, pool_host, qt, wl, ofmt):
    """Compare EVERY frame of the last timed launch's output with the oracle
    (frame i holds pool[i % P]'s coefficients, so P oracle decodes cover the
    whole batch); the comparison itself runs on the device.  Outside the timed
    region.  Returns {"ok", "frames_checked", "frames_bad", ...}."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py as O
    w, h, s = wl["width"], wl["height"], wl["sampling"]
    nf, npool = out.shape[0], pool_host.shape[0]
    nbytes = 4 * w if ofmt == 0 else 3 * w
    exp = []
    for i in range(npool):
        e = O.decode_q16(pool_host[i], qt, w, h, s).view(np.uint8).reshape(h, w, 4)
        e = e.reshape(h, 4 * w) if ofmt == 0 else np.ascontiguousarray(e[..., :3]).reshape(h, 3 * w)
        exp.append(torch.from_numpy(np.ascontiguousarray(e)).to(out.device))
    bad = [i for i in range(nf) if not torch.equal(out[i, :, :nbytes], exp[i % npool])]
    return {"ok": not bad, "frames_checked": nf, "frames_bad": len(bad), "first_bad": bad[:4],
            "how": f"all {nf} frames of the last timed launch vs oracle_decode_frame_q16 of their pool frame "
                   f"({npool} oracle decodes), compared on the device"}


def committed_traffic(workload, frames):
    """Per-launch HBM bytes from the committed PMC summary for this workload,
    if it was profiled at this launch size (else None: the bytes of another
    launch size would not describe this one)."""
    best = None
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if (d.get("workload") == workload and d.get("hbm_bytes_per_launch") and
                d.get("frames_per_launch") == frames):
            best = (d["hbm_bytes_per_launch"], os.path.relpath(p, REPO), d.get("box", "not recorded"))
    return best


def encode_pool(w, h, sampling, n, seed0):
    """n distinct synthetic JPEGs (gradient + sigma-20 noise, q=90)."""
    import io
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image

    def one(i):
        rng = np.random.default_rng(seed0 + i)
        x = np.arange(w, dtype=np.float32)[None, :]
        y = np.arange(h, dtype=np.float32)[:, None]
        img = np.stack([x * 255 / w + 0 * y, y * 255 / h + 0 * x, (x + y) * 255 / (w + h)], axis=-1)
        img = np.clip(img + rng.normal(0, 20, (h, w, 3)).astype(np.float32), 0, 255).astype(np.uint8)
        b = io.BytesIO()
        Image.fromarray(img).save(b, format="JPEG", quality=90, subsampling=2 if sampling == 1 else 0)
        return b.getvalue()

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        return list(ex.map(one, range(n)))


STREAM_POOL = 64          # distinct files the global frame-id list cycles over
CHECK_PRIME = (1 << 31) - 1


def frame_checksum(torch, t, weights):
    """Position-weighted checksum of one output frame (device or host tensor),
    computed on the device: sum_k word_k * w_k mod (2^31 - 1) over its 32-bit words."""
    x = t.reshape(-1).view(torch.int32).to(weights.device, non_blocking=True).to(torch.int64) & 0xFFFFFFFF
    return int(((x * weights[:x.numel()]) % CHECK_PRIME).sum().item() % CHECK_PRIME)


def jpeg_single_latency(args, wl, hjd, torch, dist, world, dev, steps, warmup):
    """Config 1 end to end, one image at a time (the reference program's use:
    decode one file, src/main.cpp + src/decoder.cpp:397-416): JPEG bytes in
    host memory -> BGRX in HBM, each step = submit + sync of ONE image.  Three
    paths on the same file: GPU Huffman from pageable bytes (host destuff; the
    headline), GPU Huffman from pinned bytes (device destuff), and host
    Huffman + the fused kernel.  The last timed step's output of the first
    path is checked against the oracle on the host decoder's coefficients."""
    w, h, s = wl["width"], wl["height"], wl["sampling"]
    data = encode_pool(w, h, s, 1, seed0=4242)[0]
    info = hjd.parse(data)
    ctx = hjd.Context(dev.index)
    out = torch.empty((h, w), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    gd = hjd.GpuDecoder(ctx, 1, len(data), info.nblocks)
    pinned = hjd.pinned_bytes(data)
    # host Huffman path: coefficients into pinned host memory, one H2D, one launch
    coefs_h = torch.empty((info.nblocks, 64), dtype=torch.int16).pin_memory()
    coefs_d = torch.empty((info.nblocks, 64), dtype=torch.int16, device=dev)
    plan = hjd.Plan(ctx, [hjd.FrameSpec(w, h, s, qt_index=(0, 1, 2))], hjd.IN_Q16_ZIGZAG, qtables=info.qt)

    def gpu_pageable():
        gd.decode([data], [out], stream)
        gd.sync()

    def gpu_pinned():
        gd.decode([pinned], [out], stream)
        gd.sync()

    def host_huffman():
        hjd.decode_coefs_into(data, coefs_h.numpy())
        coefs_d.copy_(coefs_h, non_blocking=True)
        plan.launch(coefs_d, out, stream)
        torch.cuda.synchronize()

    def timed(fn, k):
        for _ in range(warmup):
            fn()

        def body():
            for _ in range(k):
                fn()
        return timed_region(dist, world, body, torch.cuda.synchronize)[1] / k

    t_gpu = timed(gpu_pageable, steps)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py as O
    ref, rinfo = hjd.decode_coefs(data)
    ok = bool(np.array_equal(out.cpu().numpy().view(np.uint32), O.decode_q16(ref, rinfo.qt, w, h, s)))
    t_pin = timed(gpu_pinned, steps)
    t_host = timed(host_huffman, steps)
    gd.close()
    plan.close()
    return {"t_gpu": t_gpu, "ok": ok, "jpeg_bytes": len(data),
            "latency_ms_per_image": {"gpu_huffman_pageable_bytes": round(t_gpu * 1e3, 4),
                                     "gpu_huffman_pinned_bytes_device_destuff": round(t_pin * 1e3, 4),
                                     "host_huffman_then_kernel": round(t_host * 1e3, 4)}}


def run_jpeg_single(args, wl, hjd, torch, dist, world, rank, dev):
    """--workload fhd420_jpeg: jpeg_single_latency as its own line."""
    w, h, s = wl["width"], wl["height"], wl["sampling"]
    r = jpeg_single_latency(args, wl, hjd, torch, dist, world, dev, args.steps, args.warmup)
    t_gpu, ok = r["t_gpu"], r["ok"]
    px = w * h
    if rank == 0:
        res = {
            "metric": "Mpixels/s decoded (dequant+IDCT+colour) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(px * world / t_gpu / 1e6, 1), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_gpu * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": f"synthetic JPEG (Pillow q90, gradient + sigma-20 noise), {r['jpeg_bytes']} bytes",
            "config": {"workload": wl["desc"], "width": w, "height": h, "sampling": SAMPLING_NAMES[s],
                       "images_per_step_per_gpu": 1, "parallelism": f"image-parallel x{world} (no collective)"},
            "latency_ms_per_image": r["latency_ms_per_image"],
            "output_checked_vs_oracle": ok,
            "roofline": None,
        }
        print(json.dumps(res), flush=True)
    if world > 1 and dist.is_initialized():
        dist.destroy_process_group()
    if not ok:
        log("FATAL: the decoded image differs from the oracle")
        sys.exit(1)


def configs1_legs(args, hjd, torch, dist, world, rank, dev, qt):
    """BASELINE configs[1] in the default line: one 1920x1080 4:2:0 frame per
    launch (`fhd420`: resident coefficients -> BGRX, the single-image kernel
    launch, src/decoder.cpp:402-409 + src/oclDCT8x8.cpp:275-304) and one FHD
    JPEG end to end per step (`fhd420_jpeg`: bytes in host memory -> BGRX in
    HBM with the GPU Huffman decode).  Both are latency-bound (the frame is
    cache-resident), so they report time per launch / per image, not a
    roofline fraction; both are checked against the oracle."""
    wl = dict(WORKLOADS["fhd420"])
    k = max(args.steps, 200)
    r = pixel_batch(args, wl, hjd, torch, dist, world, rank, dev, qt, k, max(args.warmup, 10), measure=False)
    r.pop("_pool_host")
    fhd = {"value": r["value"], "unit": "Mpixels/s", "n_gpus": world, "launches": k,
           "us_per_launch_kernel": round(r["_kernel_ms"] * 1e3, 3),
           "us_per_launch_wall": round(r["_wall_max"] / k * 1e6, 3),
           "workload": wl["desc"], "output_checked_vs_oracle": r["output_check"]["ok"],
           "how": f"{k} back-to-back launches of one plan over one resident FHD frame; kernel time from HIP events "
                  f"on the launch stream, wall time over the timed region (barrier + synchronize on both sides)",
           "reference_path": "src/decoder.cpp:402-409 + src/oclDCT8x8.cpp:275-304 (clidct_run of one image)"}
    wj = dict(WORKLOADS["fhd420_jpeg"])
    j = jpeg_single_latency(args, wj, hjd, torch, dist, world, dev, args.steps, args.warmup)
    fj = {"value": round(wj["width"] * wj["height"] * world / j["t_gpu"] / 1e6, 1), "unit": "Mpixels/s",
          "n_gpus": world, "images": args.steps, "ms_per_image": round(j["t_gpu"] * 1e3, 4),
          "latency_ms_per_image": j["latency_ms_per_image"], "jpeg_bytes": j["jpeg_bytes"],
          "workload": wj["desc"], "output_checked_vs_oracle": j["ok"],
          "reference_path": "src/decoder.cpp:262-416 (decode_huffman_data + decode_mcu_data of one file)"}
    return fhd, fj


def run_stream(args, wl, hjd, torch, dist, world, rank, dev):
    """Config 5: end-to-end JPEG bytes (host memory) -> BGRX in HBM, one stream
    per GPU with its own host worker pool.  The stream is ONE global list of
    frame ids (file = id % 64 over a shared pool of 64 encoded 4K files); step k
    covers ids [k*G, (k+1)*G), G = frames_per_gpu * world, and rank r decodes
    shard_round_robin(G, r, world) of them (no collective).  After timing, every
    surviving frame of the last step gets a checksum, aggregated over ranks
    with shard.aggregate and compared with the oracle's pixels of the same ids.
    entropy="gpu": workers only parse + destuff, the Huffman decode runs on the
    GPU (hjd_gstream); entropy="host": host Huffman workers (hjd_stream)."""
    from ocljpegdecoder_amd import shard
    w, h, s, nf = wl["width"], wl["height"], wl["sampling"], wl["frames"]
    share = host_cpu_share()[0]
    # the GPU's CPU slice (its NUMA node's CPUs split over the node's GPUs),
    # every logical CPU of it (SMT: profiles/r06a_smt_probe.json), within this
    # rank's part of the process CPU share
    slice_cpus = len(hjd.device_worker_cpus(dev.index))
    nthreads = int(os.environ.get("HJD_STREAM_THREADS", hjd.stream_worker_threads(share, world, slice_cpus)))
    npool = int(os.environ.get("HJD_STREAM_POOL", STREAM_POOL))
    pool = encode_pool(w, h, s, npool, seed0=7919)       # identical on every rank: ids map to the same files
    infos = [hjd.parse(d) for d in pool]
    max_blocks = max(i.nblocks for i in infos)
    # N>1 from a parent bench run: this GPU's previous-generation rank must have
    # released its HBM before this rank allocates (max over ranks, reported)
    released = shard.aggregate(device_released(torch, dev), reduce_max=("hbm_wait_s", "hbm_busy_GiB"))
    ctx = hjd.Context(dev.index)
    gpu_entropy = wl.get("entropy") == "gpu"
    d2h = bool(wl.get("d2h"))
    # 32-frame batches x 10 slots keep several batches on the GPU at once; the
    # stream's decoders take S = 8192 in the entropy kernels (hjd_entropy.hip
    # stream_sub_bits): 102-104 Gpx/s against 95-97 for 48 x 8 and 91-94 at
    # S = 4096 on the same boxes (profiles/r02_stream_subbits.json)
    per_batch = int(os.environ.get("HJD_STREAM_BATCH", 16 if d2h else 32))
    nslots = int(os.environ.get("HJD_STREAM_SLOTS", 4 if d2h else 10))
    ofmt = wl.get("out_format", hjd.OUT_BGRX)
    pitch = hjd.default_pitch(w, ofmt)
    shape, dtype = ((h, w), torch.int32) if ofmt == hjd.OUT_BGRX else ((h, pitch), torch.uint8)
    if d2h:
        # pinned host ring, one buffer per frame that can be in flight
        ring = [torch.empty(shape, dtype=dtype).pin_memory() for _ in range(min(nf, per_batch * nslots))]
        outs = [ring[i % len(ring)] for i in range(nf)]
    else:
        ring = None
        outs = [torch.empty(shape, dtype=dtype, device=dev) for _ in range(nf)]
    # the middle timed step writes a second set of outputs, so that two steps
    # (the middle and the last) are checked after the timed region
    mid_step = args.warmup + args.steps // 2
    outs_mid = outs if d2h else [torch.empty(shape, dtype=dtype, device=dev) for _ in range(nf)]
    if gpu_entropy:
        st = hjd.GpuJpegStream(ctx, per_batch, per_batch * max(len(d) for d in pool) + (1 << 20),
                               per_batch * max_blocks, nslots=nslots, nthreads=nthreads, out_format=ofmt)
        stat_key = "host_prep_ns"
    else:
        # two jobs per worker in flight (hjd_stream pairs its Huffman decodes) + a few for the GPU side
        st = hjd.JpegStream(ctx, max_blocks, nthreads=nthreads,
                            nslots=int(os.environ.get("HJD_STREAM_HOST_SLOTS", 2 * nthreads + 4)))
        stat_key = "host_decode_ns"

    # the pool is held the way a loader would read files: into pinned host memory
    # (HJD_STREAM_PINNED=1, default), so the scans go to the GPU raw and are
    # destuffed there -- the host parses headers only; with 0, pageable ctypes
    # buffers take the host destuff path.  Made once: submit() passes pointers.
    pinned_pool = gpu_entropy and os.environ.get("HJD_STREAM_PINNED", "1") == "1"
    if pinned_pool:
        # one pinned arena, files back to back in id order (a loader's read-ahead ring):
        # consecutive frames' scans then move to the GPU in one DMA per run
        import torch as _t
        arena = _t.empty(sum(len(d) for d in pool), dtype=_t.uint8).pin_memory()
        pool_c, pos = [], 0
        for d in pool:
            arena[pos:pos + len(d)] = _t.frombuffer(bytearray(d), dtype=_t.uint8)
            pool_c.append(arena[pos:pos + len(d)])
            pos += len(d)
    else:
        pool_c = pool   # the bytes themselves: submit passes their address, no copy
    G = nf * world

    def step(k):
        o = outs_mid if k == mid_step else outs
        for i, fid in enumerate(stream_step_ids(k, nf, rank, world)):
            st.submit(pool_c[fid % npool], o[i])

    # Steps are submitted back to back: the stream does not drain between
    # steps (a drain idles the DMA engine for the last batch's kernels, ~6 % of
    # a 1024-frame step).  One sync before the last step makes its writes the
    # only ones in flight into `outs` (consecutive steps reuse those buffers on
    # different slot streams), so the checked outputs are the last step's.
    for k in range(args.warmup):
        step(k)
    st.sync()
    stats = {}
    step_sync = os.environ.get("HJD_BENCH_STEP_SYNC") == "1"   # A/B knob: drain after every step (round-2/3 behaviour)

    def body():
        stats["before"] = st.sync()                 # stats are cumulative
        for act, k in stream_schedule(args.warmup, args.steps, step_sync):
            if act == "sync":
                stats["after"] = st.sync()
                continue
            step(k)
            if (k - args.warmup) % 16 == 15:
                log(f"stream step {k - args.warmup + 1}/{args.steps} submitted")

    wall, wall_max = timed_region(dist, world, body, torch.cuda.synchronize)   # max over ranks
    before, after = stats["before"], stats["after"]
    host_ns = after[stat_key] - before[stat_key]
    busy = None
    if not gpu_entropy:
        # the pipeline's overlap, this rank: how much of the wall time the copy
        # engine and the kernel were busy (HIP timing events around every
        # upload and launch, hjd_stream_busy), and the bytes moved
        h2d_b = after["h2d_bytes"] - before["h2d_bytes"]
        busy = {"h2d_GBps": round(h2d_b / wall / 1e9, 2),
                "h2d_busy_frac": round((after["h2d_busy_ns"] - before["h2d_busy_ns"]) / 1e9 / wall, 4),
                "kernel_busy_frac": round((after["kernel_busy_ns"] - before["kernel_busy_ns"]) / 1e9 / wall, 4),
                "kernel_us_per_frame": round((after["kernel_busy_ns"] - before["kernel_busy_ns"]) / 1e3 /
                                             max(1, after["kernel_launches"] - before["kernel_launches"]), 2),
                "host_threads": nthreads,
                "host_huffman_Mpx_per_core_s": round(nf * args.steps * w * h / (host_ns / 1e9) / 1e6, 1)
                if host_ns else None}
        kbusy_s = (after["kernel_busy_ns"] - before["kernel_busy_ns"]) / 1e9
        # the ceilings of this pipeline: the kernel alone on these
        # single-frame launches, the host Huffman threads decoding all the time, and
        # the pinned upload of the int16 coefficients (measured after the check)
        busy["kernel_only_Mpx_s"] = round(nf * args.steps * w * h / kbusy_s / 1e6, 1) if kbusy_s else None
        if busy["host_huffman_Mpx_per_core_s"]:
            busy["host_huffman_ceiling_Mpx_s"] = round(busy["host_huffman_Mpx_per_core_s"] * nthreads, 1)
        busy["coef_bytes_per_frame"] = int(h2d_b / max(1, after["images"] - before["images"]))
    host_scan = after.get("host_scan_bytes", 0) - before.get("host_scan_bytes", 0)
    px = nf * w * h * args.steps * world

    # ---- correctness of the middle and the last step, outside the timed region ----
    # expected pixels per pool file: host Huffman coefficients -> oracle (the checker)
    last_step = args.warmup + args.steps - 1
    checks = [(last_step, outs)]
    if not d2h and mid_step != last_step:
        checks.insert(0, (mid_step, outs_mid))
    live = range(nf - len(ring), nf) if d2h else range(nf)     # D2H ring: only the last frames survive
    g = torch.Generator(device=dev)
    g.manual_seed(12345)
    nwords = outs[0].numel() * outs[0].element_size() // 4
    weights = torch.randint(1, CHECK_PRIME, (nwords,), generator=g, device=dev, dtype=torch.int64)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_py as O
    import scale_pins as SP
    # the pool's host coefficients against the reference's own mcu_data hashes
    # (tests/scale_pins.py; the manifest pins config 5's 64-file 4K pool)
    pins = SP.manifest_scale().get("bench_pool_4k420_q90", {}).get("files", []) \
        if (w, h, s, npool) == (3840, 2160, 1, STREAM_POOL) else []
    pin_count = {"pinned": 0, "unpinned": 0, "MISMATCH": 0}
    exp_cs = {}
    got = exp = id_sum = nchecked = 0
    for k, o in checks:
        ids = stream_step_ids(k, nf, rank, world)
        for i in live:
            f = ids[i] % npool
            if f not in exp_cs:
                coefs, info = hjd.decode_coefs(pool[f])
                pin_count[SP.check_coefs(pins[f], pool[f], coefs, info.qt, info.sampling, natural=False)
                          if f < len(pins) else "unpinned"] += 1
                e = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
                if ofmt != hjd.OUT_BGRX:
                    e = np.zeros((h, pitch), np.uint8)
                    e[:, :3 * w] = O.decode_q16(coefs, info.qt, w, h, s).view(np.uint8).reshape(h, w, 4)[..., :3] \
                        .reshape(h, 3 * w)
                exp_cs[f] = frame_checksum(torch, torch.from_numpy(np.ascontiguousarray(e)), weights)
            got += frame_checksum(torch, o[i], weights)
            exp += exp_cs[f]
            id_sum += ids[i]
            nchecked += 1
    # sums of < 2^31 values over <= 2^21 frames are exact in float64 (shard.aggregate's dtype)
    agg, ok = stream_check_totals(got, exp, id_sum, nchecked)
    # PCIe ceilings measured the way the stream moves bytes (concurrent slot streams, batch-sized pieces)
    jpeg_mean = float(np.mean([len(d) for d in pool]))
    h2d = pcie_ceiling(torch, dev, "h2d", per_batch * jpeg_mean, sorted({2, 4, nslots})) if gpu_entropy else None
    if busy:   # hjd_stream uploads one frame's coefficients per copy on one copy stream
        c = pcie_ceiling(torch, dev, "h2d", busy["coef_bytes_per_frame"], [1, 2])
        busy["pcie_ceiling_GBps"] = c["GBps"]
        busy["pcie_ceiling_Mpx_s"] = round(c["GBps"] * 1e9 / (busy["coef_bytes_per_frame"] / (w * h)) / 1e6, 1)
    d2h_c = pcie_ceiling(torch, dev, "d2h", h * pitch, sorted({2, 4, nslots}), host_bufs=ring) if d2h else None
    if rank == 0:
        jpeg_bytes = int(np.mean([len(d) for d in pool]))
        res = {
            "metric": "Mpixels/s decoded (dequant+IDCT+colour) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(px / wall_max / 1e6, 1), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": f"synthetic JPEG files (Pillow q90, gradient + sigma-20 noise), one pool of {npool} shared by all "
                    f"ranks, cycled over a global frame-id list",
            "config": {"workload": wl["desc"], "frames_per_gpu_per_step": nf, "width": w, "height": h,
                       "sampling": SAMPLING_NAMES[s], "host_threads_per_gpu": nthreads,
                       "host_cpu_share": share, "gpu_cpu_slice": slice_cpus,
                       "entropy_decode": "gpu" if gpu_entropy else "host", "mean_jpeg_bytes": jpeg_bytes,
                       "output": ("pinned host memory (D2H-on)" if d2h else "in HBM (D2H-off)") +
                                 (", BGR24" if ofmt == hjd.OUT_BGR24 else ", BGRX"),
                       "sharding": f"global frame ids 0..{(args.warmup + args.steps) * G - 1} (file = id % {npool}); "
                                   f"step k = ids [k*{G}, (k+1)*{G}), shard_round_robin over {world} rank(s)",
                       "timed_frame_ids": args.steps * G,
                       "parallelism": f"image-parallel x{world} (no collective)"},
            "end_to_end": {
                ("host_prep_Mpx_per_thread_s" if gpu_entropy else "host_huffman_Mpx_per_thread_s"):
                    round(nf * args.steps * w * h / (host_ns / 1e9) / 1e6, 1) if host_ns else None,
                "jpeg_GBps_in": round(nf * args.steps * jpeg_bytes * world / wall_max / 1e9, 2),
                "destuff": ("gpu (pinned JPEG pool, raw scans DMA'd)" if pinned_pool else "host (pageable pool)")
                           if gpu_entropy else "n/a (host Huffman)",
                "host_scan_bytes_per_frame": round(host_scan / (nf * args.steps), 1) if gpu_entropy else None,
                "h2d_ceiling": None if h2d is None else {
                    "pinned_h2d_GBps": h2d["GBps"],
                    "jpeg_GBps_in_per_gpu": round(nf * args.steps * jpeg_bytes / wall_max / 1e9, 2),
                    "frac": round(nf * args.steps * jpeg_bytes / wall_max / 1e9 / h2d["GBps"], 3),
                    "rows": h2d["rows"],
                    "how": "pinned host -> device copies on this GPU after the timed region, as the stream moves "
                           "its JPEG scans: 2, 4 and the stream's slot count of concurrent streams, each copying "
                           "one batch's bytes at a time (plus one stream of 256 MiB copies); the best rate is "
                           "the ceiling"},
                "d2h_ceiling": None if d2h_c is None else {
                    "pinned_d2h_GBps": d2h_c["GBps"],
                    "bgrx_GBps_out_per_gpu": round(nf * args.steps * h * pitch / wall_max / 1e9, 2),
                    "frac": round(nf * args.steps * h * pitch / wall_max / 1e9 / d2h_c["GBps"], 3),
                    "rows": d2h_c["rows"],
                    "how": "device -> pinned host copies on this GPU after the timed region, as the stream "
                           "returns frames: 2, 4 and the stream's slot count of concurrent streams, one frame's "
                           "output per copy, into a fresh pinned buffer and into the stream's own ring (plus one "
                           "stream of 256 MiB copies); the best rate is the ceiling"},
                "pipeline": busy,
                "output_checked_vs_oracle": bool(ok),
                "coefs_vs_reference_mcu_data": dict(pin_count, how="sha256 of each checked pool file's host "
                                                    "coefficients (and their dequantised natural-order form) vs the "
                                                    "reference's own mcu_data hashes, tests/golden/manifest.json "
                                                    "scale.bench_pool_4k420_q90 (rank 0's files)")},
            "hbm_at_start": {"wait_s_max_over_ranks": round(released["hbm_wait_s"], 2),
                             "busy_GiB_max_over_ranks": round(released["hbm_busy_GiB"], 2),
                             "how": "hipMemGetInfo polled before the first allocation until at most "
                                    f"{HBM_BUSY_FRAC:.0%} of the device is held by any process (<= 60 s)"},
            "timed_seconds": round(wall_max, 3),
            "stream_check": {"frames_checked": int(agg["frames_checked"]), "checksum": int(agg["checksum"]),
                             "checksum_oracle": int(agg["checksum_oracle"]), "id_sum": int(agg["id_sum"]),
                             "steps_checked": [k for k, _ in checks],
                             "how": "middle and last timed steps (separate output buffers): per-frame "
                                    "position-weighted checksum of the output, summed over ranks "
                                    "(shard.aggregate); oracle = host Huffman coefficients -> "
                                    "oracle_decode_frame_q16 of the same ids"},
            "roofline": None, "cpu_baseline": None,
        }
        print(json.dumps(res), flush=True)
    st.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        log("FATAL: stream output differs from the oracle")
        sys.exit(1)
    if pin_count["MISMATCH"]:
        log("FATAL: host Huffman coefficients differ from the reference's mcu_data")
        sys.exit(1)


def pcie_ceiling(torch, dev, direction, chunk_bytes, stream_counts, total_bytes=4 << 30, host_bufs=None):
    """Pinned host <-> device copy rate on this GPU (GB/s) the way the stream
    uses PCIe: `n` concurrent HIP streams, each copying `chunk_bytes` pieces
    (one batch's JPEG scans for H2D, one frame's BGRX for D2H) round-robin,
    for every n in stream_counts, plus one stream of 256 MiB copies (the
    round-3 measurement).  With host_bufs (pinned tensors of >= chunk_bytes:
    the stream's own), the n-stream rows are repeated on them, so that where
    the pages of a fresh buffer land does not set the ceiling below the rate
    the stream's buffers allow.  Returns {"GBps": best, "rows": [...]} -- the
    best of these is the ceiling the stream's rate is divided by."""
    chunk = max(1 << 20, int(chunk_bytes) // 4096 * 4096)
    nmax = max(stream_counts)
    span = max(256 << 20, chunk * nmax)
    host = torch.empty(span, dtype=torch.uint8).pin_memory()
    devb = torch.empty(span, dtype=torch.uint8, device=dev)
    rows = []
    own = [b.view(-1).view(torch.uint8)[:chunk] for b in host_bufs] if host_bufs else []
    own = [b for b in own if b.numel() == chunk]
    runs = [(1, 256 << 20, False)] + [(n, chunk, False) for n in stream_counts] + \
        [(n, chunk, True) for n in stream_counts if own]
    for n, size, on_own in runs:
        streams = [torch.cuda.Stream(dev) for _ in range(n)]
        ncopies = max(n, int(total_bytes // size))
        pieces = max(1, span // size)

        def issue(k):
            st = streams[k % n]
            off = (k % pieces) * size
            hb = own[k % len(own)] if on_own else host[off:off + size]
            with torch.cuda.stream(st):
                if direction == "h2d":
                    devb[off:off + size].copy_(hb, non_blocking=True)
                else:
                    hb.copy_(devb[off:off + size], non_blocking=True)
        for k in range(n):
            issue(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(ncopies):
            issue(k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rows.append({"streams": n, "copy_bytes": size, "GBps": round(ncopies * size / dt / 1e9, 2),
                     **({"host": "the stream's buffers"} if on_own else {})})
    del host, devb
    return {"GBps": max(r["GBps"] for r in rows), "rows": rows}


def numa_nodes():
    try:
        return sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and
                      d[4:].isdigit())
    except OSError:
        return []


def run_host_prep(args):
    """--host-prep-only: the host side of the config-5 stream with no GPU, as N
    concurrent per-GPU worker pools (pool p on NUMA node p % nodes), to state
    the host ceiling of the 8-GPU stream.  Modes: host destuff
    (parse + tables + destuff into staging: what a pageable JPEG costs), header
    only (the GPU-destuff path for pinned JPEGs), plain memcpy (DRAM reference).
    Per configuration: wall-clock JPEG GB/s and implied Gpx/s (4K 4:2:0 q90),
    and the rate per thread from thread CPU clocks, which stays meaningful when
    pools x threads exceed the box's CPU quota (then wall-clock is the quota's)."""
    import threading
    import ocljpegdecoder_amd as hjd
    from ocljpegdecoder_amd import _lib
    lib = _lib.load()
    w, h = 3840, 2160
    files = encode_pool(w, h, 1, 16, seed0=7919)
    mean_bytes = float(np.mean([len(d) for d in files]))
    bufs = [(ctypes.c_uint8 * len(d)).from_buffer_copy(d) for d in files]
    arr_d = (ctypes.POINTER(ctypes.c_uint8) * len(bufs))(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    arr_s = (ctypes.c_size_t * len(bufs))(*[len(d) for d in files])
    nodes = numa_nodes() or [-1]
    share, aff, quota, nproc = host_cpu_share()
    pools_list = [int(x) for x in args.pools.split(",")]
    tpp_list = [int(x) for x in args.threads_per_pool.split(",")] if args.threads_per_pool else None
    rows = []
    for npools in pools_list:
        for tpp in (tpp_list or sorted({max(1, share // npools), 16})):
            for mode, name in ((0, "host_destuff"), (1, "header_only"), (2, "memcpy")):
                per = 400 * tpp if mode != 1 else 4000 * tpp
                outs = [(ctypes.c_int64 * 4)() for _ in range(npools)]
                rcs = [0] * npools
                barrier = ctypes.c_int32(0)

                def one(p):
                    rcs[p] = lib.hjd_debug_host_prep(arr_d, arr_s, len(bufs), mode, tpp, nodes[p % len(nodes)],
                                                     per, args.arena_mb << 20, args.ring_mb << 20,
                                                     ctypes.byref(barrier), npools, outs[p])
                th = [threading.Thread(target=one, args=(p,)) for p in range(npools)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                wall = max(o[0] for o in outs) / 1e9      # timed phases start together (barrier)
                if any(rcs):
                    raise RuntimeError(f"host prep failed: {_lib.error_string()}")
                nbytes = sum(o[2] for o in outs)
                cpu_s = sum(o[1] for o in outs) / 1e9
                frames = sum(o[3] for o in outs)
                rows.append({"pools": npools, "threads_per_pool": tpp, "mode": name,
                             "wall_GBps": round(nbytes / wall / 1e9, 2),
                             "wall_Gpx_s": round(frames * w * h / wall / 1e9, 1),
                             "per_thread_GBps_cpu_clock": round(nbytes / cpu_s / 1e9, 2) if cpu_s else None,
                             "per_pool_Gpx_s_cpu_clock": round(frames / npools * w * h / (cpu_s / (npools * tpp))
                                                               / 1e9, 1) if cpu_s else None,
                             "oversubscribed": npools * tpp > share})
                log(json.dumps(rows[-1]))
    print(json.dumps({"what": "config-5 host preparation ceiling (no GPU)", "cpu_model": _cpu_model(),
                      "arena_MB_per_pool": args.arena_mb, "staging_ring_MB_per_pool": args.ring_mb,
                      "logical_cpus": aff, "cgroup_cpu_quota": quota, "nproc": nproc, "numa_nodes": len(nodes),
                      "frame": f"{w}x{h} 4:2:0 q90, mean {mean_bytes / 1e6:.2f} MB",
                      "gpu_demand_GBps_per_gpu_at_100Gpx_s": round(100e9 / (w * h) * mean_bytes / 1e9, 1),
                      "rows": rows}), flush=True)


def timed_region(dist, world, body, sync):
    """The contract's timed region on every code path: barrier + device
    synchronize, body(), synchronize + barrier.  Returns (this rank's wall
    seconds, the max over ranks via shard.aggregate's MAX all-reduce).  With N
    ranks over RCCL this is the only cross-GPU traffic: two barriers and the
    two all-reduces of shard.aggregate."""
    from ocljpegdecoder_amd import shard
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    body()
    sync()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    return wall, shard.aggregate({"seconds": wall})["seconds"]


def stream_schedule(warmup, steps, step_sync=False):
    """The stream leg's timed region as actions ("step", k) / ("sync", None).
    Steps are submitted back to back; the only drains are one before the last
    step (consecutive steps write the same output buffers from different slot
    streams, so the checked last step must be the only writer in flight) and
    the final one.  step_sync=True drains after every step (A/B knob)."""
    acts, last = [], warmup + steps - 1
    for k in range(warmup, warmup + steps):
        if step_sync or (k == last and k != warmup):
            acts.append(("sync", None))
        acts.append(("step", k))
    acts.append(("sync", None))
    return acts


def stream_step_ids(k, frames_per_gpu, rank, world):
    """Global frame ids rank `rank` decodes in stream step k: step k covers ids
    [k*G, (k+1)*G), G = frames_per_gpu * world, dealt round-robin over ranks."""
    from ocljpegdecoder_amd import shard
    G = frames_per_gpu * world
    return [k * G + p for p in shard.shard_round_robin(G, rank, world)]


def stream_check_totals(got, exp, id_sum, nchecked):
    """Sums of the per-rank stream checks over ranks (shard.aggregate: SUM);
    ok when the output checksums equal the oracle's."""
    from ocljpegdecoder_amd import shard
    agg = shard.aggregate({"frames_checked": nchecked, "checksum": got, "checksum_oracle": exp, "id_sum": id_sum})
    return agg, agg["checksum"] == agg["checksum_oracle"]


_TORCHRUN_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
                  "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
                  "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_ERROR_FILE",
                  "TORCHELASTIC_ENABLED")


def stream_leg_command(world, dist_backend, frame_ids, per_gpu, port, environ, workload="stream4k420"):
    """The config-5 child run rank 0 starts: (argv, env, steps).  N=1: plain
    python; N>1: torch.distributed.run over the same N GPUs on `port` at
    127.0.0.1.  Enough steps of per_gpu frames per GPU to cover frame_ids
    global ids (>= 3).  The env drops this rank's torchrun variables, so the
    child agent sets its own."""
    steps = max(3, -(-frame_ids // (per_gpu * world)))
    args = [os.path.abspath(__file__), "--gpus", str(world), "--workload", workload, "--steps", str(steps),
            "--warmup", "1", "--no-cpu", "--dist-backend", dist_backend, "--frames", str(per_gpu)]
    if world == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    env = {k: v for k, v in environ.items() if k not in _TORCHRUN_VARS}
    return cmd, env, steps


def roofline_obj(achieved, bytes_per_launch, kernel_ms, traffic, box=None):
    """The line's roofline object.  Measured in THIS run: achieved =
    algorithmic bytes per launch / the mean launch time from HIP events on the
    launch stream; box_ceiling_GBps / frac_of_box_ceiling = the same bytes
    against this box's own streaming rate for the kernel's read:write mix
    (hjd_debug_rw_mix, same process, same buffers).  From ANOTHER run, and
    labelled so: traffic = per-launch HBM bytes of the committed rocprofv3 PMC
    passes of the same command (profiles/*pmc*.json), with their path and box."""
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBPS, 4),
         "traffic": traffic[0] if traffic else None,
         "algorithmic_bytes_per_launch": bytes_per_launch,
         "kernel_ms_per_launch": round(kernel_ms, 4),
         "kernel_ms_source": "this run: HIP events on the launch stream around the timed launches"}
    if traffic:
        r["traffic_other_run"] = {"path": traffic[1], "box": traffic[2],
                                  "what": "committed rocprofv3 PMC passes of the same command (FETCH_SIZE x2 + "
                                          "WRITE_SIZE per launch), not measured in this run"}
    if box:
        r["box_ceiling_GBps"] = box["ceiling_GBps"]
        r["frac_of_box_ceiling"] = round(achieved / box["ceiling_GBps"], 4)
        r["box_ceiling_source"] = "this run: " + box["how"]
    return r


def box_ceiling(torch, ctx, src, dst, stream, mix, memory_only=None, reps=5):
    """This box's streaming rate for the fused kernel's read:write mix (KiB
    per task: 6:8 at 4:2:0, 6:4 at 4:4:4), measured on the bench's own buffers
    after the output check.  Candidates, all measured in this run:
      * hjd_debug_rw_mix with the kernel's launch shape (nt, XCD order, the
        next unit's loads issued before this unit's stores) and its store
        geometry (two 512-B row segments per store instruction, 3840-px
        rows), at 1/2/4 units per wave; the same with contiguous stores;
      * the kernel's own memory-only variant (stage_times: loads, staging, LDS
        reads and stores of the product, no IDCT or colour math).
    Each is a rate this box reaches for these bytes, so the best of them is
    the tightest ceiling measured; the product's frac_of_box_ceiling is
    against it.  Read-only and write-only rates of the same buffers are
    reported beside it."""
    r, w = mix

    def rate(rk, wk, upw, flags):
        nbytes = ctx.debug_rw_mix(src, dst, rk, wk, upw, flags, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            ctx.debug_rw_mix(src, dst, rk, wk, upw, flags, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        return round(nbytes / (e0.elapsed_time(e1) / reps) / 1e6, 1)
    rows = [{"kernel": "rw_mix", "stores": "image rows", "units_per_wave": upw, "GBps": rate(r, w, upw, 15)}
            for upw in (1, 2, 4)]
    rows.append({"kernel": "rw_mix", "stores": "contiguous", "units_per_wave": 2, "GBps": rate(r, w, 2, 7)})
    if memory_only:
        rows.append({"kernel": "fused kernel, memory-only variant (stages 80)", "GBps": round(memory_only, 1)})
    best = max(rows, key=lambda x: x["GBps"])
    return {"ceiling_GBps": best["GBps"], "ceiling_from": best["kernel"], "mix_kib": f"{r}:{w}", "rows": rows,
            "read_only_GBps": rate(6, 0, 4, 3), "write_only_GBps": rate(0, 8, 4, 3),
            "how": f"best of: hjd_debug_rw_mix {r}:{w} KiB read:write per wave-unit (the kernel's per-task bytes), "
                   f"16 B per lane, nt, XCD-contiguous in-order grid, pipelined, with the kernel's image-row store "
                   f"geometry at 1/2/4 units per wave and with contiguous stores; and the kernel's own memory-only "
                   f"variant; {reps} launches each on the bench's own coefficient and output buffers"}


def box_identity(torch):
    """Which GPU this line was measured on (the container hostname is not
    unique): the amdgpu unique id and product serial from sysfs.  No
    subprocess (rocm-smi is a Python script started through /usr/bin/env; run
    from a process that has initialised the GPU -- under rocprofv3 every
    process has -- that exec is refused on the GPU box)."""
    ident = {"hostname": socket.gethostname(), "device": torch.cuda.get_device_name(0)}
    for card in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            if open(os.path.join(card, "vendor")).read().strip() != "0x1002":
                continue
            for key, f in (("unique_id", "unique_id"), ("serial", "serial_number")):
                pth = os.path.join(card, f)
                if os.path.exists(pth):
                    ident[key] = open(pth).read().strip()
            if "unique_id" in ident or "serial" in ident:
                break
        except OSError:
            continue
    return ident


def clock_under_load(torch, ctx, dev, stream, launch, steps, kernel_ms):
    """The shader clock the chip holds while `launch` runs (MI355X lowers it
    under load, and devices differ: MI355X_MICROARCH.md 'DVFS give-back'):
    hjd_debug_clock_probe samples s_memtime / s_memrealtime every 20 us on a
    side stream beside `steps` more launches (untimed, after the timed region).
    Returns the median / p10 / p90 of the per-interval clock, first 10 % of the
    samples dropped (ramp)."""
    interval = 2000                                   # 100-MHz ticks = 20 us
    n = int(max(32, min(100000, steps * kernel_ms * 1e-3 * 1e8 * 0.9 // interval)))
    buf = torch.zeros(2 * n, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    ctx.clock_probe(buf, n, interval, side)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    smp = buf.cpu().numpy().reshape(n, 2).astype(np.float64)
    f = np.diff(smp[:, 1]) / np.maximum(np.diff(smp[:, 0]), 1) * 0.1    # GHz (real-time ticks are 10 ns)
    f = f[len(f) // 10:]
    return {"sclk_GHz_median": round(float(np.median(f)), 3), "sclk_GHz_p10": round(float(np.percentile(f, 10)), 3),
            "sclk_GHz_p90": round(float(np.percentile(f, 90)), 3), "samples": int(len(f)),
            "kernel_ms_beside_probe": round(e0.elapsed_time(e1) / steps, 4),
            "how": "hjd_debug_clock_probe: one wave on a side stream samples (s_memtime, s_memrealtime) every 20 us "
                   f"while {steps} more launches run (after the timed region); clock = d(cycles) / d(10-ns ticks)"}


STAGE_VARIANTS = {80: "memory_only", 4: "no_stores"}


def stage_times(torch, plan, coefs, out, stream, product_ms, reps):
    """Same-run ablation of the fused kernel on the bench's own plan and
    buffers (after the output check; outputs are wrong by design): the
    memory-only variant (loads, staging, LDS reads, stores; no IDCT, no colour
    math) and the no-store variant.  What binds the kernel in THIS run is read
    off these times, not asserted."""
    res = {"product_ms": round(product_ms, 4)}
    for st, name in STAGE_VARIANTS.items():
        plan.launch_stages(st, coefs, out, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            plan.launch_stages(st, coefs, out, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        res[name + "_ms"] = round(e0.elapsed_time(e1) / reps, 4)
    over = product_ms / res["memory_only_ms"] - 1
    res["product_over_memory_only_pct"] = round(100 * over, 2)
    if over <= 0.02:
        res["binding"] = ("memory: the product runs within 2 % of its own memory-only variant (same loads, LDS "
                          "traffic and stores, no IDCT or colour math)")
    else:
        res["binding"] = (f"instruction issue on top of memory: the product takes {100 * over:.1f} % longer than its "
                          f"memory-only variant (same loads, LDS traffic and stores)")
    res["how"] = (f"hjd_debug_plan_launch_stages on this run's plan and buffers, {reps} launches each after one warmup, "
                  f"HIP events; timing-only variants with wrong outputs by design")
    return res


def pixel_batch(args, wl, hjd, torch, dist, world, rank, dev, qt, steps, warmup, measure=True):
    """One pixel workload on this rank: inputs resident in HBM, W untimed + K
    timed launches of one plan over the whole batch (barrier + synchronize on
    both sides, max over ranks), then every frame of the last launch checked
    against the oracle.  Frees its device buffers before returning."""
    from ocljpegdecoder_amd import shard
    w, h, s, nf = wl["width"], wl["height"], wl["sampling"], wl["frames"]
    mw, mh, bpm, _ = hjd.mcu_geometry(w, h, s)
    nblk = mw * mh * bpm
    npool = min(POOL, nf)
    i32 = wl.get("input") == "i32"
    pool16 = torch.empty((npool, nblk, 64), dtype=torch.int16, device=dev)
    for i in range(npool):
        pool16[i] = synth_frame_gpu(torch, nblk, s, qt, seed=1000 * rank + i, device=dev)
    if i32:
        # the idct.h format: dequantised (src/decoder.cpp:338-342) int32 in natural order
        inv = [0] * 64
        for k, n in enumerate(ZIGZAG_NAT):
            inv[n] = k
        comp = torch.from_numpy(hjd.block_components(s, nblk)).to(dev)
        qz = torch.from_numpy(np.asarray(qt, dtype=np.int32)).to(dev)[comp]          # [nblk, 64] file order
        src = (pool16.to(torch.int32) * qz)[:, :, torch.tensor(inv, device=dev)]     # natural order
        coefs = torch.empty((nf, nblk, 64), dtype=torch.int32, device=dev)
        for i in range(npool):
            coefs[i] = src[i]
        del src
    else:
        coefs = torch.empty((nf, nblk, 64), dtype=torch.int16, device=dev)
        for i in range(npool):
            coefs[i] = pool16[i]
    for i in range(npool, nf):
        coefs[i].copy_(coefs[i % npool])
    ofmt = wl.get("out_format", hjd.OUT_BGRX)
    pitch = hjd.default_pitch(w, ofmt)
    out = torch.empty((nf, h, pitch), dtype=torch.uint8, device=dev)
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * pitch, out_pitch=pitch,
                           qt_index=(0, 1, 2), out_format=ofmt) for i in range(nf)]
    ctx = hjd.Context(dev.index)
    plan = hjd.Plan(ctx, specs, hjd.IN_I32_NATURAL if i32 else hjd.IN_Q16_ZIGZAG, qtables=None if i32 else qt)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    # adapt the launch shape to this device (hjd_plan_autotune: tasks per wave x
    # store policy, timed on these buffers; untimed setup, identical pixels)
    launch = {"autotuned": False, "tasks_per_wave": None, "variant": 0}
    if not args.no_autotune and not args.grid:
        t0 = time.perf_counter()
        tpw, var = plan.autotune(coefs, out, stream)
        launch = {"autotuned": tpw > 0, "tasks_per_wave": tpw or None, "variant": var,
                  "stores": "plain" if var & 1 else "nt", "seconds": round(time.perf_counter() - t0, 2),
                  "shape": plan.launch_shape(),
                  "how": "hjd_plan_autotune: 1/2/4/8/16 tasks per wave x nt/plain stores, 2 interleaved rounds of "
                         "one warm + two timed launches each on this run's buffers; fastest kept (cached per "
                         "process by shape)"}
    for _ in range(warmup):
        plan.launch(coefs, out, stream, grid_blocks=args.grid)
    torch.cuda.synchronize()

    # ---- timed region: exactly K launches ----------------------------------------
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def body():
        ev0.record(stream)
        for _ in range(steps):
            plan.launch(coefs, out, stream, grid_blocks=args.grid)
        ev1.record(stream)

    wall, wall_max = timed_region(dist, world, body, torch.cuda.synchronize)   # max over ranks
    kernel_ms = ev0.elapsed_time(ev1) / steps   # HIP events on the launch stream

    px_per_launch = plan.pixels
    bytes_per_launch = plan.coef_bytes + hjd.OUT_BYTES[ofmt] * plan.pixels
    total_px = px_per_launch * steps * world
    value = total_px / wall_max / 1e6
    achieved = bytes_per_launch / (kernel_ms / 1e3) / 1e9

    # device-to-device copy bandwidth for context (same-size read+write)
    copy_gbps = None
    try:
        a = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        b.copy_(a); torch.cuda.synchronize()
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for _ in range(5):
            b.copy_(a)
        c1.record(stream); torch.cuda.synchronize()
        copy_gbps = round(2 * 5 * a.numel() / (c0.elapsed_time(c1) / 1e3) / 1e9, 1)
        del a, b
    except Exception:
        pass

    # every frame of the timed launch's output vs the oracle (outside the timed region)
    pool_host = pool16.cpu().numpy()
    checked = check_batch_vs_oracle(torch, out, pool_host, qt, wl, ofmt)
    # same-run measurements on the same buffers (they overwrite `out`, so after the check)
    stages = box = clock = None
    if measure and not i32 and ofmt == hjd.OUT_BGRX and s in (0, 1) and not args.no_stages:
        clock = clock_under_load(torch, ctx, dev, stream, lambda: plan.launch(coefs, out, stream, grid_blocks=args.grid),
                                 steps, kernel_ms)
        stages = stage_times(torch, plan, coefs, out, stream, kernel_ms, min(steps, 10))
        box = box_ceiling(torch, ctx, coefs, out, stream, (6, 8) if s == 1 else (6, 4),
                          memory_only=bytes_per_launch / (stages["memory_only_ms"] / 1e3) / 1e9)
    tasks = plan.tasks
    plan.close()
    del coefs, out, pool16, plan
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return {"value": round(value, 1), "output_check": checked, "device_copy_GBps": copy_gbps,
            "stages": stages, "box": box, "clock": clock, "launch": launch,
            "_pool_host": pool_host, "_wall_max": wall_max, "_kernel_ms": kernel_ms, "_achieved": achieved,
            "_bytes_per_launch": bytes_per_launch, "_tasks": tasks}


def _leg_summary(leg):
    """One leg of the compact line: its headline number, time, roofline
    fraction, same-run ceiling fraction and oracle check."""
    if not leg:
        return None
    if "error" in leg:
        return {"error": str(leg["error"])[:60]}
    r = {"Mpx_s": leg.get("value"), "ms": leg.get("ms_per_step")}
    rf = leg.get("roofline")
    if rf:
        r["frac"] = rf.get("frac")
        r["box_frac"] = rf.get("frac_of_box_ceiling")
    r["ok"] = leg.get("output_checked_vs_oracle")
    return r


def _stream_summary(leg, ceiling_key=None):
    if not leg or "error" in leg:
        return _leg_summary(leg)
    r = {"Mpx_s": leg["value"], "frame_ids": leg["timed_frame_ids"]}
    c = leg.get(ceiling_key) if ceiling_key else None
    if c:
        r[ceiling_key.split("_")[0] + "_frac"] = c["frac"]
    p = leg.get("pipeline")
    if p:
        r.update({"host_Mpx_s_per_core": p["host_huffman_Mpx_per_core_s"], "cores": p["host_threads"],
                  "h2d_GBps": p["h2d_GBps"], "kernel_busy": p["kernel_busy_frac"], "h2d_busy": p["h2d_busy_frac"],
                  "kernel_only_Mpx_s": p.get("kernel_only_Mpx_s"), "pcie_ceiling_Mpx_s": p.get("pcie_ceiling_Mpx_s")})
    if leg.get("gpu_cpu_slice") is not None:
        r["cpu_slice"] = leg["gpu_cpu_slice"]
        r["cpu_share"] = leg["host_cpu_share"]
    r["ok"] = leg["output_checked_vs_oracle"]
    pins = leg.get("coefs_vs_reference_mcu_data")
    if pins:
        r["ref_pinned"] = f"{pins['pinned']}/{pins['pinned'] + pins['unpinned'] + pins['MISMATCH']}"
    return r


def compact_line(res, detail_path):
    """The stdout line: the driver keeps only the tail of stdout, so the line
    stays short (~2 KB) and ends with `summary`, one entry per leg; the full
    result goes to `detail_path` and stderr (emit)."""
    rf = res["roofline"]
    cpu = res.get("cpu_baseline") or {}
    c4, f1, fj = res.get("config4_444"), res.get("fhd420"), res.get("fhd420_jpeg")
    ref = res.get("cpu_reference") or {}
    summary = {
        "4k420": _leg_summary(res),
        "4k444": _leg_summary(c4),
        "fhd420_us_per_launch": f1 and {"us": f1["us_per_launch_kernel"], "ok": f1["output_checked_vs_oracle"]},
        "fhd420_jpeg_ms_per_image": fj and {"ms": fj["ms_per_image"], "ok": fj["output_checked_vs_oracle"]},
        "c5_gpu_huffman": _stream_summary(res.get("config5_stream"), "h2d_ceiling"),
        "c5_host_huffman": _stream_summary(res.get("config5_stream_host")),
        "c5_d2h": _stream_summary(res.get("config5_stream_d2h"), "d2h_ceiling"),
        "cpu_port": cpu.get("value") and {"Mpx_s": cpu["value"], "cores": cpu["cores"]},
        "cpu_reference": ref.get("value") and {"Mpx_s": ref["value"], "cores": ref.get("cores")},
    }
    oks = [v.get("ok") for v in summary.values() if isinstance(v, dict) and "ok" in v]
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype")
    line = {k: res[k] for k in keep}
    line["data"] = "synthetic, resident in HBM"
    cfg = res["config"]
    line["config"] = {"workload": "configs[2]: %d x %dx%d %s, int16 zigzag in, %s" % (
        cfg["frames_per_gpu"], cfg["width"], cfg["height"], cfg["sampling"],
        "BGRX out" if "BGRX" in cfg["output"] else "BGR24 out"), "parallelism": cfg["parallelism"]}
    line["roofline"] = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                "algorithmic_bytes_per_launch", "kernel_ms_per_launch",
                                                "frac_of_box_ceiling")}
    line["cpu_baseline"] = cpu and {k: cpu.get(k) for k in ("value", "unit", "cores", "kind")}
    if cpu:
        line["cpu_baseline"]["sample"] = cpu.get("sample", "")[:60]
    line["output_checked_vs_oracle"] = all(o is not False for o in oks)
    line["detail"] = detail_path
    line["summary"] = summary
    return line


def emit(res, detail_path):
    """Full result to `detail_path` (and stderr), compact line to stdout."""
    full = json.dumps(res)
    try:
        d = os.path.dirname(os.path.abspath(detail_path))
        os.makedirs(d, exist_ok=True)
        with open(detail_path, "w") as f:
            f.write(full + "\n")
    except OSError as e:
        log(f"could not write {detail_path}: {e}")
    log("BENCH_DETAIL " + full)
    print(json.dumps(compact_line(res, detail_path)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="4k420", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=0, help="override batch size")
    ap.add_argument("--grid", type=int, default=0, help="persistent grid (workgroups), 0 = default")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-autotune", action="store_true",
                    help="pixel batches: keep the shape-default launch instead of hjd_plan_autotune's choice")
    ap.add_argument("--no-stages", action="store_true",
                    help="skip the same-run stage ablation and box-ceiling measurements of the pixel batches")
    ap.add_argument("--no-fhd", action="store_true",
                    help="4k420: skip the configs[1] legs (single FHD launch, one FHD JPEG end to end)")
    ap.add_argument("--no-d2h", action="store_true",
                    help="skip the D2H-on config-5 stream leg (config5_stream_d2h)")
    ap.add_argument("--no-444", action="store_true",
                    help="4k420: skip the configs[3] 4:4:4 batch reported under config4_444")
    ap.add_argument("--stream-frame-ids", type=int, default=100000,
                    help="config-5 stream leg: global frame ids to cover (BASELINE configs[4]: 100k images)")
    ap.add_argument("--stream-host-frame-ids", type=int, default=10240,
                    help="config-5 host-Huffman leg (config5_stream_host): global frame ids to cover")
    ap.add_argument("--no-stream-host", action="store_true",
                    help="skip the host-Huffman config-5 leg (config5_stream_host)")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where the full result (every leg's measurements and how they were taken) is written; "
                         "stdout carries the compact line")
    ap.add_argument("--no-stream", action="store_true",
                    help="N=1 pixel workloads: skip the config-5 stream leg (a child bench.py run, reported "
                         "under config5_stream)")
    ap.add_argument("--host-prep-only", action="store_true",
                    help="config-5 host side only, no GPU: per-GPU worker pools (see run_host_prep)")
    ap.add_argument("--pools", default="1,2,4,8", help="--host-prep-only: pool counts")
    ap.add_argument("--threads-per-pool", default="", help="--host-prep-only: threads per pool (default: share/N and 16)")
    ap.add_argument("--arena-mb", type=int, default=1024, help="--host-prep-only: JPEG source arena per pool")
    ap.add_argument("--ring-mb", type=int, default=512, help="--host-prep-only: pinned-staging ring per pool")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for the barrier/timing reduction (no data-path collective)")
    args = ap.parse_args()
    if args.host_prep_only:
        return run_host_prep(args)

    import torch
    import torch.distributed as dist

    from ocljpegdecoder_amd import shard
    rank, world, local_rank = shard.env_rank()
    # HJD_BENCH_SAME_DEVICE=1 + --dist-backend gloo: rehearse the N-rank path on
    # one GPU (every rank on device 0); the real multi-GPU run uses RCCL ("nccl").
    gpu = 0 if os.environ.get("HJD_BENCH_SAME_DEVICE") == "1" else local_rank
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import ocljpegdecoder_amd as hjd

    wl = dict(WORKLOADS[args.workload])
    if args.frames:
        wl["frames"] = args.frames
    w, h, s, nf = wl["width"], wl["height"], wl["sampling"], wl["frames"]
    qt = std_qtables(1.0)

    if args.workload.startswith("stream"):
        return run_stream(args, wl, hjd, torch, dist, world, rank, dev)
    if wl.get("jpeg"):
        return run_jpeg_single(args, wl, hjd, torch, dist, world, rank, dev)

    res_px = pixel_batch(args, wl, hjd, torch, dist, world, rank, dev, qt, args.steps, args.warmup)
    checked = res_px["output_check"]
    value = res_px["value"]
    pool_host = res_px.pop("_pool_host")
    npool = pool_host.shape[0]
    i32 = wl.get("input") == "i32"
    ofmt = wl.get("out_format", hjd.OUT_BGRX)
    wall_max, kernel_ms, achieved = res_px["_wall_max"], res_px["_kernel_ms"], res_px["_achieved"]
    bytes_per_launch, tasks = res_px["_bytes_per_launch"], res_px["_tasks"]

    # configs[3] (1024 x 4K 4:4:4) in the same default run, after configs[2]
    config4 = None
    if args.workload == "4k420" and not args.no_444:
        wl4 = dict(WORKLOADS["4k444"])
        if args.frames:
            wl4["frames"] = args.frames
        r4 = pixel_batch(args, wl4, hjd, torch, dist, world, rank, dev, qt, args.steps, args.warmup)
        r4.pop("_pool_host")
        traffic4 = committed_traffic("4k444", wl4["frames"])
        config4 = {
            "metric": "Mpixels/s decoded (dequant+IDCT+colour)", "value": r4["value"], "unit": "Mpixels/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(r4["_wall_max"] / args.steps * 1e3, 4),
            "workload": wl4["desc"], "frames_per_gpu": wl4["frames"], "sampling": "4:4:4",
            "output_checked_vs_oracle": r4["output_check"]["ok"], "output_check": r4["output_check"],
            "roofline": roofline_obj(r4["_achieved"], r4["_bytes_per_launch"], r4["_kernel_ms"], traffic4, r4["box"]),
            "stages": r4["stages"], "box_ceiling": r4["box"], "clock_under_load": r4["clock"], "launch": r4["launch"],
            "reference_path": "src/idct8x8.cl:168-192 (batch_idct_csc_444), src/decoder.cpp:457-471"}
        checked_all_ok = checked["ok"] and r4["output_check"]["ok"]
    else:
        checked_all_ok = checked["ok"]
    # configs[1] (single FHD 4:2:0 launch; one FHD JPEG end to end) in the same default run
    fhd = fhd_jpeg = None
    if args.workload == "4k420" and not args.no_fhd:
        fhd, fhd_jpeg = configs1_legs(args, hjd, torch, dist, world, rank, dev, qt)
        checked_all_ok = checked_all_ok and fhd["output_checked_vs_oracle"] and fhd_jpeg["output_checked_vs_oracle"]

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            log("running CPU baseline leg ...")
            cpu = cpu_baseline(pool_host, qt, wl, value)
        stream5 = stream5_d2h = stream5_host = None
        if not args.no_stream and args.workload == "4k420":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            if world > 1:
                dist.destroy_process_group()   # the other ranks are leaving; the child run has its own group
            stream5 = config5_stream_leg(world, args.dist_backend, args.stream_frame_ids)
            if not args.no_stream_host:
                stream5_host = config5_stream_leg(world, args.dist_backend, args.stream_host_frame_ids,
                                                  workload="stream4k420_host")
            if not args.no_d2h:
                stream5_d2h = config5_stream_leg(world, args.dist_backend, args.stream_frame_ids,
                                                 workload="stream4k420_d2h")
        traffic = committed_traffic(args.workload, nf)
        res = {
            "metric": "Mpixels/s decoded (dequant+IDCT+colour) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(value, 1),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (device-generated FDCT+quantised smooth+noise blocks, pool of "
                    f"{npool} distinct frames replicated to {nf}); inputs resident in HBM",
            "config": {"workload": wl["desc"], "frames_per_gpu": nf, "width": w, "height": h,
                       "sampling": SAMPLING_NAMES[s],
                       "input": "int32 natural-order dequantised (idct.h format)" if i32
                                else "int16 quantised zigzag + qtables",
                       "output": "BGRX 4 B/px in HBM" if ofmt == hjd.OUT_BGRX else "BGR24 3 B/px in HBM",
                       "parallelism": f"image-parallel x{world} (no collective)",
                       "tasks_per_launch": tasks},
            "output_checked_vs_oracle": checked["ok"],
            "output_check": checked,
            "roofline": roofline_obj(achieved, bytes_per_launch, kernel_ms, traffic, res_px["box"]),
            "stages": res_px["stages"], "box_ceiling": res_px["box"], "clock_under_load": res_px["clock"],
            "launch": res_px["launch"],
            "box": box_identity(torch),
            "cpu_baseline": cpu,
            "device_copy_GBps": res_px["device_copy_GBps"],
            "config4_444": config4,
            "config5_stream": stream5,
            "config5_stream_host": stream5_host,
            "config5_stream_d2h": stream5_d2h,
            "fhd420": fhd,
            "fhd420_jpeg": fhd_jpeg,
        }
        if cpu and "reference" in cpu:
            res["cpu_reference"] = cpu.pop("reference")
        emit(res, args.detail_out)
    if world > 1 and dist.is_initialized():
        dist.destroy_process_group()
    if not checked_all_ok:
        log("FATAL: a timed launch's output differs from the oracle")
        sys.exit(1)


def _wait_sibling_ranks_exit(timeout_s=60.0):
    """Best effort, N>1: before rank 0 starts the child ranks, let the other
    ranks of this run (children of the same torchrun agent) exit, so the GPUs
    never carry both generations of processes.  Returns how many were still
    alive at the deadline (each child rank also waits for its GPU's HBM to be
    released: device_released)."""
    agent, me = os.getppid(), os.getpid()
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        alive = 0
        for d in os.listdir("/proc"):
            if not d.isdigit() or int(d) == me:
                continue
            try:
                with open(f"/proc/{d}/stat") as f:
                    fields = f.read().rsplit(")", 1)[1].split()
            except OSError:
                continue
            if int(fields[1]) == agent and fields[0] not in ("Z", "X"):
                alive += 1
        if alive == 0:
            return 0
        time.sleep(0.5)
    return alive


HBM_BUSY_FRAC = 0.10


def device_released(torch, dev, timeout_s=60.0):
    """Poll the device's free HBM (hipMemGetInfo counts every process's
    allocations) until at most HBM_BUSY_FRAC of it is in use, so a child run
    started right after the parent's ranks left does not share the GPU with
    them.  Returns the wait and the HBM still in use when it ended."""
    t0 = time.time()
    while True:
        free, total = torch.cuda.mem_get_info(dev)
        busy = total - free
        if busy <= HBM_BUSY_FRAC * total or time.time() - t0 >= timeout_s:
            return {"hbm_wait_s": time.time() - t0, "hbm_busy_GiB": busy / 2**30}
        time.sleep(0.25)


def config5_stream_leg(world, dist_backend, frame_ids=100000, workload="stream4k420"):
    """BASELINE configs[4] on the same GPUs, measured in the same default run:
    rank 0 starts a child `bench.py --workload stream4k420` (N=1: plain python;
    N>1: torch.distributed.run over the same N GPUs on a fresh port, the frame
    ids sharded round-robin, no data-path collective) and summarises its line.
    The child has its own processes and HIP contexts (started as children,
    never exec'd; the torchrun variables of this rank are not passed on).  Its
    Mpx/s is the whole-job end-to-end figure (JPEG bytes in pinned host memory
    -> BGRX in HBM), not the headline `value`."""
    import signal
    import socket
    import subprocess
    # BASELINE configs[4] is a 100k-image stream: enough steps of 1024 frames per
    # GPU (G = 1024 * world ids per step) to cover `frame_ids` global ids
    per_gpu = int(os.environ.get("HJD_BENCH_STREAM_FRAMES", WORKLOADS[workload]["frames"]))  # tests: smaller
    port = 0
    if world > 1:
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
    cmd, env, _ = stream_leg_command(world, dist_backend, frame_ids, per_gpu, port, os.environ, workload)
    siblings_alive = _wait_sibling_ranks_exit() if world > 1 else 0
    log("running config-5 stream leg:", " ".join(cmd[1:]))
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=900)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)   # the child's own process group (its torchrun workers included)
        p.communicate()
        return {"error": "timeout after 900 s"}
    line = next((l for l in reversed(out.splitlines()) if l.startswith("{")), None)
    if p.returncode != 0 or line is None:
        # the child ranks' own error lines (torchrun's summary fills the tail)
        errs = [ln[-300:] for ln in err.splitlines() if "Error" in ln or "FATAL" in ln or "error:" in ln][-6:]
        return {"error": f"rc {p.returncode}", "stderr_tail": err[-400:], "error_lines": errs}
    d = json.loads(line)
    return {"value": d["value"], "unit": d["unit"], "n_gpus": d["n_gpus"], "ms_per_step": d["ms_per_step"],
            "steps": d["steps"], "frames_per_gpu_per_step": d["config"]["frames_per_gpu_per_step"],
            "timed_frame_ids": d["config"]["timed_frame_ids"], "timed_seconds": d["timed_seconds"],
            "workload": d["config"]["workload"], "sharding": d["config"]["sharding"],
            "value_per_gpu": round(d["value"] / d["n_gpus"], 1),
            "jpeg_GBps_in": d["end_to_end"]["jpeg_GBps_in"], "destuff": d["end_to_end"]["destuff"],
            "h2d_ceiling": d["end_to_end"].get("h2d_ceiling"),
            "d2h_ceiling": d["end_to_end"].get("d2h_ceiling"),
            "pipeline": d["end_to_end"].get("pipeline"),
            "host_threads_per_gpu": d["config"]["host_threads_per_gpu"],
            "host_cpu_share": d["config"].get("host_cpu_share"), "gpu_cpu_slice": d["config"].get("gpu_cpu_slice"),
            "output": d["config"]["output"],
            "output_checked_vs_oracle": d["end_to_end"]["output_checked_vs_oracle"],
            "coefs_vs_reference_mcu_data": d["end_to_end"].get("coefs_vs_reference_mcu_data"),
            "steps_checked": d["stream_check"]["steps_checked"],
            "parent_ranks_alive_at_start": siblings_alive, "hbm_at_start": d.get("hbm_at_start"),
            "command": " ".join(["python"] + [os.path.basename(c) if c.endswith("bench.py") else c
                                              for c in cmd[1:]])}


if __name__ == "__main__":
    main()
