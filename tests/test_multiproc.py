"""world_size-2 gloo run on CPU of the image-parallel sharding: every frame is
decoded by exactly one rank and the host-side aggregation reproduces the
single-process totals (pixel counts, per-frame checksums, max time)."""
import hashlib
import os
import socket

import numpy as np
import pytest

import oracle_py as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def frame_digest(name):
    """Host Huffman (product front end) + oracle pixels -> 64-bit checksum."""
    import ocljpegdecoder_amd as hjd
    data = open(os.path.join(O.GOLDEN, name + ".jpg"), "rb").read()
    coefs, info = hjd.decode_coefs(data)
    px = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
    return int.from_bytes(hashlib.sha256(px.tobytes()).digest()[:6], "little"), info.width * info.height


def _worker(rank, world, port, names, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from ocljpegdecoder_amd import shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, _ = shard.env_rank()
    if mode == "range":
        b, e = shard.shard_range(len(names), r, w)
        mine = list(range(b, e))
    else:
        mine = shard.shard_round_robin(len(names), r, w)
    digest = pixels = 0
    for i in mine:
        d, p = frame_digest(names[i])
        digest += d
        pixels += p
    agg = shard.aggregate({"digest": digest, "pixels": pixels, "frames": len(mine), "seconds": 1.0 + r},
                          reduce_max=("seconds",))
    q.put((r, agg, mine))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["range", "round_robin"])
def test_two_rank_gloo_sharding(mode):
    import torch.multiprocessing as mp
    names = O.golden_cases() * 2 + O.golden_cases()[:3]     # 23 frames: uneven split
    expect_digest = expect_px = 0
    for n in names:
        d, p = frame_digest(n)
        expect_digest += d
        expect_px += p
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, names, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = sorted(i for _, _, mine in res for i in mine)
    assert shards == list(range(len(names)))               # each frame exactly once
    for _, agg, _ in res:
        assert agg["frames"] == len(names)
        assert agg["pixels"] == expect_px
        assert agg["digest"] == expect_digest
        assert agg["seconds"] == 2.0                        # max over ranks


def test_shard_helpers():
    from ocljpegdecoder_amd import shard
    for n in (0, 1, 7, 1024, 100000):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1
            rr = sorted(i for r in range(w) for i in shard.shard_round_robin(n, r, w))
            assert rr == list(range(n))
    with pytest.raises(ValueError):
        shard.shard_range(4, 2, 2)
