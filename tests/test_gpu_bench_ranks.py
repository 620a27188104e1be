"""bench.py's N-rank path on the one-GPU box: two ranks launched exactly as the
driver launches the scaling bench (torch.distributed.run, 127.0.0.1), but
with HJD_BENCH_SAME_DEVICE=1 and the gloo process group so both ranks share
device 0 (RCCL cannot put two ranks on one GPU).  Checks the contract fields
of the single JSON line rank 0 prints: n_gpus, whole-job value, weak scaling,
no data-path collective.  The real N>1 run (RCCL over xGMI) is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(workload, frames, extra=(), ranks=2, steps=3, timeout=110):
    """Rank 0's one stdout line; for the pixel workloads, whose line is the
    compact one, the full result from the --detail-out file (with the line
    itself under "_line")."""
    import tempfile
    env = dict(os.environ, HJD_BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    detail = os.path.join(tempfile.mkdtemp(prefix="hjd_bench_"), "detail.json")
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--steps", str(steps), "--warmup", "1",
            "--workload", workload, "--frames", str(frames), "--no-cpu", "--detail-out", detail, *extra]
    if ranks == 1:
        cmd = [sys.executable, *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args, "--dist-backend", "gloo"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]           # rank 0 only, one line
    line = json.loads(lines[0])
    if not os.path.exists(detail):
        return line
    full = json.load(open(detail))
    assert full["value"] == line["value"] and line["detail"] == detail
    full["_line"] = line
    return full


@pytest.mark.gpu
def test_two_ranks_pixel_bench():
    """The driver's N>1 command line: the pixel line, and the config-5 stream leg
    that rank 0 runs as a child torch.distributed.run over the same ranks
    (HJD_BENCH_STREAM_FRAMES keeps its steps small here)."""
    extra_env = {"HJD_BENCH_STREAM_FRAMES": "12", "HJD_STREAM_POOL": "8"}
    os.environ.update(extra_env)
    try:
        r = _run("4k420", 8, extra=("--stream-frame-ids", "72", "--stream-host-frame-ids", "48"), timeout=300)
    finally:
        for k in extra_env:
            os.environ.pop(k, None)
    assert r["n_gpus"] == 2 and r["steps"] == 3 and r["warmup"] == 1
    assert r["scaling"] == "weak" and r["higher_is_better"] is True
    assert r["value"] > 0 and r["ms_per_step"] > 0
    # whole-job value: both ranks' pixels over the max-over-ranks wall time
    px = 2 * 3 * 8 * 3840 * 2160
    assert abs(r["value"] - px / (r["ms_per_step"] * 3 / 1e3) / 1e6) / r["value"] < 0.02
    assert "no collective" in r["config"]["parallelism"] or "x2" in r["config"]["parallelism"]
    c4 = r["config4_444"]                                  # configs[3] in the same run
    assert c4["output_checked_vs_oracle"] is True and c4["frames_per_gpu"] == 8 and c4["n_gpus"] == 2
    assert abs(c4["value"] - px / (c4["ms_per_step"] * 3 / 1e3) / 1e6) / c4["value"] < 0.02
    s5 = r["config5_stream"]
    assert "error" not in s5, s5
    assert s5["n_gpus"] == 2 and s5["value"] > 0 and s5["output_checked_vs_oracle"] is True
    assert s5["frames_per_gpu_per_step"] == 12 and "shard_round_robin over 2 rank(s)" in s5["sharding"]
    assert s5["steps"] == 3 and s5["timed_frame_ids"] == 72 and s5["steps_checked"] == [2, 3]
    # the child ranks started on GPUs the parent's ranks had left and released
    assert s5["parent_ranks_alive_at_start"] == 0
    assert s5["hbm_at_start"]["wait_s_max_over_ranks"] < 60, s5["hbm_at_start"]
    # the north star's host-Huffman pipeline over the same 2 ranks
    sh = r["config5_stream_host"]
    assert "error" not in sh, sh
    assert sh["n_gpus"] == 2 and sh["output_checked_vs_oracle"] is True and sh["timed_frame_ids"] == 72   # >= 3 steps of 12 x 2
    p = sh["pipeline"]
    assert 0 < p["kernel_busy_frac"] <= 1 and 0 < p["h2d_busy_frac"] <= 1 and p["h2d_GBps"] > 0, p
    # the compact stdout line carries every leg's headline
    sm = r["_line"]["summary"]
    assert sm["4k444"]["Mpx_s"] == c4["value"] and sm["c5_host_huffman"]["Mpx_s"] == sh["value"]
    assert r["_line"]["output_checked_vs_oracle"] is True


@pytest.mark.gpu
def test_two_ranks_stream_bench():
    r = _run("stream4k420", 16)
    assert r["n_gpus"] == 2 and r["value"] > 0
    assert r["end_to_end"]["output_checked_vs_oracle"] is True
    assert r["config"]["entropy_decode"] == "gpu"


@pytest.mark.gpu
def test_stream_sharding_matches_one_rank():
    """Config 5's shape: one global frame-id list (file = id % pool) sharded
    round-robin over ranks.  Two ranks x 12 frames and one rank x 24 frames
    cover the same ids in every step, so the per-frame checksums of the last
    step, summed over ranks (shard.aggregate), must be identical -- and equal
    to the oracle's checksum of those ids."""
    extra_env = {"HJD_STREAM_POOL": "8"}
    os.environ.update(extra_env)
    try:
        two = _run("stream4k420", 12, steps=2)
        one = _run("stream4k420", 24, ranks=1, steps=2)
    finally:
        for k in extra_env:
            os.environ.pop(k, None)
    for r in (one, two):
        c = r["stream_check"]
        assert c["frames_checked"] == 24 and c["checksum"] == c["checksum_oracle"], c
    assert two["stream_check"]["id_sum"] == one["stream_check"]["id_sum"] == sum(range(48, 72))
    assert two["stream_check"]["checksum"] == one["stream_check"]["checksum"]
