"""tools/ktrace_dispatch.py picks the bench line's own timed launches out of a
kernel trace of `python bench.py`: after the launch autotune's candidate
launches of the same kernel, before the clock probe and the stage variants
(bench.py pixel_batch), for the exact instantiation the line ran (launch
variant bits, plus the d16 gather bit at 4:4:4 when present)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import ktrace_dispatch  # noqa: E402

K420 = "void hjd::decode_kernel<1, 0, {}>(void const*, int const*, hjd::FrameDev const*, int, long, unsigned char*, long, long)"
K444 = "void hjd::decode_kernel<0, 0, {}>(void const*, int const*, hjd::FrameDev const*, int, long, unsigned char*, long, long)"
CLOCK = "void (anonymous namespace)::clock_probe_kernel(unsigned long*, int, int)"


def trace(autotune=30, warmup=3, steps=20, t420=9.0, t444=15.0, stages=True):
    rows, t = [], 0

    def add(name, ms, n):
        nonlocal t
        for _ in range(n):
            rows.append((t, t + int(ms * 1e6), name))
            t += int(ms * 1e6) + 1000

    for key, ms, var, stage in ((K420, t420, 0, 80), (K444, t444, 128, 208)):
        add(key.format(var), ms * 1.3, autotune // 2)          # autotune: nt candidates
        add(key.format(var | 1), ms * 1.2, autotune // 2)      # ... and plain-store ones
        add(key.format(var), ms, warmup + steps)               # the bench's warmup + timed launches
        if stages:                                             # (bench.py --no-stages skips these)
            add(CLOCK, 0.02, 1)
            add(key.format(var), ms * 1.1, steps)              # clock_under_load
            add(key.format(stage), ms * 0.9, 11)               # stage variants
    return rows


LINE = {"launch": {"variant": 0}, "roofline": {"algorithmic_bytes_per_launch": 59454259200,
                                               "kernel_ms_per_launch": 9.0, "frac": 0.8258},
        "config4_444": {"launch": {"variant": 0},
                        "roofline": {"algorithmic_bytes_per_launch": 84934656000, "kernel_ms_per_launch": 15.0,
                                     "frac": 0.7078}}}


def test_split_skips_autotune_and_later_launches():
    w = ktrace_dispatch.split(trace(), LINE, 3, 20, 1024)
    assert w["4k420"]["kernel"] == "hjd::decode_kernel<1,0,0>"
    assert w["4k444"]["kernel"] == "hjd::decode_kernel<0,0,128>"   # the d16 gather instantiation
    for wl, ms in (("4k420", 9.0), ("4k444", 15.0)):
        e = w[wl]
        assert e["dispatches_of_kernel_before_timed"] == 15 and e["timed_dispatches"] == 20
        assert abs(e["timed_mean_ms"] - ms) < 1e-3 and abs(e["timed_max_ms"] - ms) < 1e-3
        assert abs(e["frac_from_timed_dispatches"] - e["bench_frac_same_run"]) < 1e-3


def test_split_without_autotune_or_stages():
    # bench.py --no-autotune --no-stages: no candidates before, no probe after;
    # the bench's launches are then the last W + K of the instantiation
    w = ktrace_dispatch.split(trace(autotune=0, stages=False), LINE, 3, 20, 1024)
    for wl, ms in (("4k420", 9.0), ("4k444", 15.0)):
        assert w[wl]["timed_dispatches"] == 20 and w[wl]["dispatches_of_kernel_before_timed"] == 0
        assert abs(w[wl]["timed_mean_ms"] - ms) < 1e-3


def test_split_follows_the_plain_store_variant():
    line = {"launch": {"variant": 1}, "roofline": LINE["roofline"], "config4_444": LINE["config4_444"]}
    rows = []
    t = 0
    for var, n, ms in ((1, 15, 8.0), (0, 15, 9.5), (1, 23, 8.5)):
        for _ in range(n):
            rows.append((t, t + int(ms * 1e6), K420.format(var)))
            t += int(ms * 1e6) + 1000
    rows.append((t, t + 20000, CLOCK))
    w = ktrace_dispatch.split(rows, line, 3, 20, 1024)
    assert w["4k420"]["kernel"] == "hjd::decode_kernel<1,0,1>" and abs(w["4k420"]["timed_mean_ms"] - 8.5) < 1e-3
