"""The RCCL calls of an N-GPU bench run, on one real device.

bench.py under torchrun (N > 1) makes exactly these cross-GPU calls
(DESIGN.md s7): init_process_group("nccl", device_id=...), barriers around
the timed region, and shard.aggregate's two float64 all-reduces (SUM of
counters, MAX of wall seconds).  The box has one GPU, so this runs them in a
one-rank RCCL group: it proves RCCL initialises on MI355X and that the
aggregation code path (not only its gloo twin, tests/test_multiproc.py) runs
on the device.  It cannot show multi-GPU scaling.
"""
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["HJD_REPO"])
import torch
import torch.distributed as dist
from ocljpegdecoder_amd import shard
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["HJD_PORT"], rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
dist.barrier()
stats = {"seconds": 1.25, "frames_checked": 1024.0, "checksum": 123456789.0}
got = shard.allreduce_stats(stats)
dist.barrier()
torch.cuda.synchronize()
ver = torch.cuda.nccl.version()
dist.destroy_process_group()
print(json.dumps({"got": got, "rccl_version": list(ver) if isinstance(ver, tuple) else ver}))
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_one_rank_aggregate():
    env = dict(os.environ, HJD_REPO=REPO, HJD_PORT=str(_free_port()))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["got"] == {"seconds": 1.25, "frames_checked": 1024.0, "checksum": 123456789.0}
    print("RCCL", out["rccl_version"])
