"""World-size-2 test of the multi-GPU data path on CPU (gloo): ranks own
tiles t % N == rank, pack them like the kernel's packed output,
and rank 0 gathers + un-permutes them into the frame (bench.py's gather)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_package


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, width, height, tile, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = load_package()
    rng = np.random.default_rng(5)
    full = rng.integers(0, 256, (height, width, 3), dtype=np.uint8)  # same on every rank
    mine = pkg.pack_tiles(full, width, height, tile, rank, world)
    n = torch.tensor([mine.size])
    dist.all_reduce(n, op=dist.ReduceOp.MAX)
    send = torch.zeros(int(n.item()), dtype=torch.uint8)
    send[: mine.size] = torch.from_numpy(mine)
    gl = [torch.zeros_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, gl, dst=0)
    # max-over-ranks timing as bench.py does it
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        out = np.zeros_like(full)
        for r in range(world):
            cnt = len(pkg.owned_tiles(width, height, tile, r, world)) * tile * tile * 3
            pkg.unpack_tiles(gl[r].numpy()[:cnt], width, height, tile, r, world, out)
        q.put((bool(np.array_equal(out, full)), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("width,height,tile", [(100, 70, 32), (64, 64, 32), (33, 17, 8)])
def test_tile_shard_gather_two_ranks(width, height, tile):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, width, height, tile, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    ok, tmax = q.get(timeout=10)
    assert ok
    assert tmax == 2.0


def test_tiles_partition_the_frame():
    pkg = load_package()
    for n in (1, 2, 3, 8):
        seen = []
        for r in range(n):
            seen += pkg.owned_tiles(1920, 1080, 32, r, n)
        assert sorted(seen) == list(range(60 * 34))


def test_tile_deal_is_diagonal():
    # rows are rotated by their index, so when N divides the 60 tile columns
    # a shard still owns tiles in every column (not column stripes)
    pkg = load_package()
    for n in (2, 4):
        for r in range(n):
            cols = {t % 60 for t in pkg.owned_tiles(1920, 1080, 32, r, n)}
            assert cols == set(range(60))
    # deal index d = shard + k * n -> tile (row d // 60, column (d % 60 + row) % 60)
    assert pkg.owned_tiles(1920, 1080, 32, 1, 2)[:3] == [1, 3, 5]
    assert pkg.owned_tiles(1920, 1080, 32, 0, 2)[30:32] == [61, 63]
