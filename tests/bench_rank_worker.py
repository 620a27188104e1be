"""One rank of the N-rank rehearsal of bench.py's bookkeeping (tests/
test_bench_ranks_cpu.py::test_eight_rank_torchrun_rehearsal), started by
torch.distributed.run exactly as the driver starts bench.py: every rank reads
its identity from the torchrun environment, runs bench.py's own helpers over
a gloo group and writes what it saw to <out_dir>/rank<r>.json.  Rank 0 then
waits for its sibling ranks to exit (bench._wait_sibling_ranks_exit, what it
does before starting the config-5 child run) and records how many were left."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir = sys.argv[1]
    import torch.distributed as dist

    import bench
    from ocljpegdecoder_amd import shard
    rank, world, local_rank = shard.env_rank()
    dist.init_process_group("gloo")
    syncs = []
    wall, wall_max = bench.timed_region(dist, world, lambda: time.sleep(0.02 * (rank + 1)), lambda: syncs.append(1))
    ids = [bench.stream_step_ids(k, 6, rank, world) for k in range(3)]
    got = sum(3 * i for i in ids[-1])
    agg, ok = bench.stream_check_totals(got, got, sum(ids[-1]), len(ids[-1]))
    _, ok_bad = bench.stream_check_totals(got, got + (1 if rank == world - 1 else 0), 0, 0)
    cmd, env, steps = bench.stream_leg_command(world, "nccl", 100000, 1024, 40000 + world, os.environ)
    cmd_h, _, steps_h = bench.stream_leg_command(world, "nccl", 10240, 128, 40001, os.environ, "stream4k420_host")
    res = {"rank": rank, "world": world, "local_rank": local_rank, "wall": wall, "wall_max": wall_max,
           "nsync": len(syncs), "ids": ids, "agg": agg, "ok": ok, "ok_bad": ok_bad, "steps": steps,
           "steps_host": steps_h, "cmd": cmd, "cmd_host": cmd_h,
           "env_torchrun_keys": sorted(k for k in env if k in bench._TORCHRUN_VARS),
           "env_master_addr": env.get("MASTER_ADDR"), "ppid": os.getppid()}
    dist.destroy_process_group()
    if rank == 0:
        res["siblings_alive"] = bench._wait_sibling_ranks_exit(timeout_s=60)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
