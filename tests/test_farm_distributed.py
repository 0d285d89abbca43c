"""The multi-GPU fit farm's host-side protocol on CPU ranks (gloo, world 2 and 3):
each rank takes its LPT share of the 280 fits, results are gathered with an
object all-gather, elapsed time is max-reduced.  No collective carries fit
data."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nerf_attention import CONFIGS_FULL, engine, farm


def _costs():
    return [engine.fit_flops(2048, 128, c, 2000) for c in CONFIGS_FULL] * 40


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        costs = _costs()
        mine = farm.rank_share(costs, world, rank)
        # stand-in for the per-fit records the GPU would produce
        local = {i: {"fit": i, "rank": rank, "cos": 1.0 - 1e-6 * i} for i in mine}
        merged = farm.gather_records(local)
        t = farm.max_over_ranks(float(rank + 1))
        farm.barrier()
        q.put((rank, sorted(mine), sorted(merged), t, sum(costs[i] for i in mine)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_farm_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    shares = [r[1] for r in res]
    flat = sorted(i for s in shares for i in s)
    assert flat == list(range(280))                       # every fit exactly once
    for r in res:
        assert r[2] == list(range(280))                   # everyone sees the union
        assert r[3] == float(world)                       # max over ranks
    loads = [r[4] for r in res]
    assert max(loads) / (sum(loads) / world) < 1.05       # LPT balance
    # rank shares are what a single process computes for that rank
    costs = _costs()
    for rank, s in enumerate(shares):
        assert s == farm.rank_share(costs, world, rank)


def test_single_process_share_is_everything():
    assert farm.rank_share([3.0, 1.0, 2.0], 1, 0) == [0, 1, 2]
    assert farm.max_over_ranks(2.5) == 2.5
    assert farm.gather_records({1: "a"}) == {1: "a"}
