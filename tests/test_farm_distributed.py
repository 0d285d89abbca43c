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


# ---- bench.py launcher (world 2 on CPU, gloo; no device work) -------------

import json as _json
import subprocess as _sp
import sys as _sys
from pathlib import Path as _Path

_BENCH = _Path(__file__).resolve().parent.parent / "bench.py"


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


@pytest.mark.parametrize("world", [2, 8])
def test_bench_spawns_ranks(world):
    """`python bench.py --gpus N` without a launcher starts N ranks itself
    (N = 8 is the driver's full-node case); they form a gloo group, split the
    280 fits (farm.auto_partition: width-blocked at 2, LPT at 8) and meet in
    the barrier, max and gather; rank 0 prints one line that saw every rank."""
    r = _sp.run([_sys.executable, str(_BENCH), "--gpus", str(world), "--dry-run"],
                env=_bench_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = _json.loads(lines[0])
    assert line["n_gpus"] == world and line["ranks_seen"] == world
    assert line["fits"] == list(range(280)) and set(line["owner"]) == set(range(world))
    costs = _costs()
    widths = [c.hidden_features for c in CONFIGS_FULL] * 40
    assert [farm.rank_share(costs, world, k, widths) for k in range(world)] == \
        [[i for i, o in enumerate(line["owner"]) if o == k] for k in range(world)]
    loads = line["rank_flops"]
    assert max(loads) / min(loads) < 1.05


def test_partitions_cover_and_balance():
    costs = _costs()
    widths = [c.hidden_features for c in CONFIGS_FULL] * 40
    for n in (2, 3, 4, 8):
        for p in farm.PARTITIONS:
            shares = [farm.rank_share(costs, n, r, widths, p) for r in range(n)]
            assert sorted(i for s in shares for i in s) == list(range(280))
            loads = [sum(costs[i] for i in s) for s in shares]
            assert max(loads) / (sum(loads) / n) < 1.06, (n, p)
    # blocked: each rank holds few widths
    for r in range(2):
        ws = {widths[i] for i in farm.rank_share(costs, 2, r, widths, "blocked")}
        assert len(ws) <= 4
    assert farm.auto_partition(2) == "blocked" and farm.auto_partition(8) == "lpt"


def test_bench_rejects_world_mismatch():
    """A launcher world that disagrees with --gpus is an error, not a silent
    single-GPU run."""
    r = _sp.run([_sys.executable, str(_BENCH), "--gpus", "2", "--dry-run"],
                env=_bench_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_spawn_ranks_propagates_failure(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "sys.exit(3) if r == 1 else time.sleep(30)\n")
    t0 = __import__("time").time()
    rc = farm.spawn_ranks(2, [], str(script))
    assert rc == 3 and __import__("time").time() - t0 < 20   # rank 0 was terminated


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_dry_run_leaves_no_child(gpus):
    """bench.py reports the processes it started that are still alive when it
    exits (the driver's record showed one process outliving the
    bench); the dry run — rank spawn, gloo group, shares, barrier, gather — ends
    with none."""
    r = _sp.run([_sys.executable, str(_BENCH), "--gpus", str(gpus), "--dry-run"],
                env=_bench_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "children at exit: 0" in r.stderr, r.stderr[-2000:]
