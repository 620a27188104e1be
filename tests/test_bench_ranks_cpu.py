"""bench.py's N-rank bookkeeping on CPU: the functions every
bench code path times and aggregates through, run by two gloo ranks.

- timed_region: barrier + synchronize around the body, and the wall time is
  the MAX over ranks (shard.aggregate's MAX all-reduce), on every rank;
- stream_step_ids: the config-5 global frame-id list, dealt round-robin, covers
  every id of a step exactly once whatever the rank count;
- stream_check_totals: the stream's checksums are SUMMED over ranks;
- stream_leg_command: the child run rank 0 starts (plain python at N=1,
  torch.distributed.run at 127.0.0.1 for N>1), its step count for 100k ids,
  and the scrubbing of this rank's torchrun variables from its environment.

The real N=8 run uses the same functions over RCCL (DESIGN.md s7 lists its
collectives); only the device layer differs (torch.cuda.synchronize).
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import time

    import torch.distributed as dist

    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    syncs = []
    # rank r's body takes (r + 1) * 50 ms: every rank must report the slowest
    wall, wall_max = bench.timed_region(dist, world, lambda: time.sleep(0.05 * (rank + 1)),
                                        lambda: syncs.append(1))
    ids = [bench.stream_step_ids(k, 6, rank, world) for k in range(3)]
    got = sum(3 * i for i in ids[-1])           # stand-ins for per-frame checksums
    agg, ok = bench.stream_check_totals(got, got, sum(ids[-1]), len(ids[-1]))
    agg_bad, ok_bad = bench.stream_check_totals(got, got + rank, 0, 0)
    q.put((rank, wall, wall_max, len(syncs), ids, agg, ok, ok_bad))
    dist.destroy_process_group()


def test_two_rank_timing_and_stream_bookkeeping():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    walls = [r[1] for r in res]
    for rank, wall, wall_max, nsync, ids, agg, ok, ok_bad in res:
        assert nsync == 2                                   # synchronize before and after the body
        assert wall_max == max(walls) and wall_max >= 0.1   # max over ranks, on every rank
        assert ok and not ok_bad
        assert agg["frames_checked"] == 12                  # 6 frames per GPU x 2 ranks, summed
        assert agg["id_sum"] == sum(range(24, 36))          # step 2 covers ids [24, 36)
        assert agg["checksum"] == 3 * sum(range(24, 36))
    # every id of every step exactly once over the ranks
    for k in range(3):
        allids = sorted(i for r in res for i in r[4][k])
        assert allids == list(range(12 * k, 12 * (k + 1)))


def test_stream_step_ids_match_one_rank():
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 3, 8):
        for k in (0, 5):
            allids = sorted(i for r in range(world) for i in bench.stream_step_ids(k, 1024, r, world))
            assert allids == list(range(k * 1024 * world, (k + 1) * 1024 * world))


@pytest.mark.parametrize("warmup,steps", [(1, 98), (1, 13), (3, 2), (1, 1), (0, 5)])
def test_stream_schedule(warmup, steps):
    """The stream leg submits steps back to back: every timed step exactly
    once in order, a drain right before the last step (its output buffers are
    then written by it alone) and at the end, and no other drain."""
    sys.path.insert(0, ROOT)
    import bench
    acts = bench.stream_schedule(warmup, steps)
    assert [k for a, k in acts if a == "step"] == list(range(warmup, warmup + steps))
    assert acts[-1] == ("sync", None)
    syncs = [i for i, (a, _) in enumerate(acts) if a == "sync"]
    last = acts.index(("step", warmup + steps - 1))
    if steps > 1:
        assert syncs == [last - 1, len(acts) - 1]
    else:
        assert syncs == [len(acts) - 1]
    # the A/B knob: a drain before every step after the first and at the end
    per = bench.stream_schedule(warmup, steps, step_sync=True)
    assert [a for a, _ in per] == ["sync", "step"] * steps + ["sync"]


@pytest.mark.parametrize("world", [1, 2, 8])
def test_stream_leg_command(world):
    sys.path.insert(0, ROOT)
    import bench
    environ = {"RANK": "3", "WORLD_SIZE": str(world), "LOCAL_RANK": "3", "MASTER_PORT": "29500",
               "TORCHELASTIC_RUN_ID": "x", "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
               "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PATH": "/usr/bin"}
    cmd, env, steps = bench.stream_leg_command(world, "nccl", 100000, 1024, 41234, environ)
    assert steps * 1024 * world >= 100000 and (steps - 1) * 1024 * world < 100000
    assert steps == {1: 98, 2: 49, 8: 13}[world]
    assert cmd[0] == sys.executable
    i = cmd.index("--steps")
    assert cmd[i + 1] == str(steps)
    assert cmd[cmd.index("--frames") + 1] == "1024" and cmd[cmd.index("--gpus") + 1] == str(world)
    assert cmd[cmd.index("--workload") + 1] == "stream4k420" and "--no-cpu" in cmd
    if world == 1:
        assert "torch.distributed.run" not in cmd
    else:
        assert cmd[1:3] == ["-m", "torch.distributed.run"]
        assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
        assert cmd[cmd.index("--master-port") + 1] == "41234"
        assert cmd[cmd.index("--nproc-per-node") + 1] == str(world)
    # this rank's torchrun identity is not inherited; the rest of the environment is
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "GROUP_RANK"):
        assert k not in env
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["MASTER_ADDR"] == "127.0.0.1"
    assert env["PATH"] == "/usr/bin"
    # small runs (tests) still time >= 3 steps
    assert bench.stream_leg_command(world, "gloo", 10, 12, 1, environ)[2] == 3


def test_eight_rank_torchrun_rehearsal(tmp_path):
    """bench.py's N = 8 bookkeeping, launched the way the
    driver launches the 8-GPU bench (python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1), over gloo on CPU:
    timed_region's max over 8 ranks, each global frame id of a stream step
    decoded by exactly one of the 8 ranks, checksums summed over all 8 (one bad
    rank fails the whole check), the config-5 child commands (both stream legs)
    for N = 8 with this rank's torchrun identity scrubbed, and rank 0 seeing
    its 7 siblings gone before it would start the child run."""
    import json
    import subprocess
    world = 8
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "bench_rank_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(world)]
    walls = [x["wall"] for x in res]
    assert sorted(x["rank"] for x in res) == list(range(world))
    assert sorted(x["local_rank"] for x in res) == list(range(world))
    assert len({x["ppid"] for x in res}) == 1                      # one torchrun agent
    for x in res:
        assert x["world"] == world and x["nsync"] == 2
        assert x["wall_max"] == max(walls) and x["wall_max"] >= 0.16
        assert x["ok"] and not x["ok_bad"]                         # a single bad rank fails everyone's check
        assert x["agg"]["frames_checked"] == 6 * world
        G = 6 * world
        assert x["agg"]["id_sum"] == sum(range(2 * G, 3 * G))
        assert x["steps"] == 13 and x["steps_host"] == 10          # 100,000 / (1024 x 8); 10,240 / (128 x 8)
        assert x["env_torchrun_keys"] == [] and x["env_master_addr"] == "127.0.0.1"
        for c, wl in ((x["cmd"], "stream4k420"), (x["cmd_host"], "stream4k420_host")):
            assert c[1:3] == ["-m", "torch.distributed.run"] and c[c.index("--nproc-per-node") + 1] == "8"
            assert c[c.index("--workload") + 1] == wl and c[c.index("--gpus") + 1] == "8"
    for k in range(3):
        allids = sorted(i for x in res for i in x["ids"][k])
        assert allids == list(range(6 * world * k, 6 * world * (k + 1)))
    assert res[0]["siblings_alive"] == 0
