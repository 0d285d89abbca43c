"""Multi-GPU fit farm: one process per GPU, independent fits, no data collective.

SURVEY.md §8e: the sweep's fits are independent, so the only multi-GPU work
is assigning them to ranks (LPT on the FLOP model of §8d) and gathering the
small per-fit results on the host afterwards.  xGMI/RCCL carry nothing: the
control collectives (barrier, max of the elapsed time, object gather of the
records) run on a gloo process group, so no GPU collective is ever set up.

There is ONE multi-GPU design, used by every entry point:
  * `bench.py --gpus N` under torch.distributed.run (or self-spawned, see
    `spawn_ranks`): every rank trains `rank_share(costs, N, rank)` on its own
    GPU and the ranks meet only at the gloo barrier / max / gather;
  * `fit_kv_cache(gpus=N)` / `run_fits(devices=[...])`: `run_farm` starts one
    worker process per device (fresh interpreters, started before this
    process needs the GPU for anything), each worker trains its share
    (rank_share under farm.auto_partition / NERFHIP_FARM_PARTITION) on its
    device and sends the outputs back to the parent over a pipe.
The reference loop being farmed is fit.py:54-86 (strictly sequential there).
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

from .engine import lpt_partition


def world() -> tuple:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def blocked_partition(costs: list, widths: list, n_bins: int) -> list:
    """Bin per item: the items sorted by (width desc, cost desc, index) and cut
    into n_bins contiguous runs of about equal total cost, so every bin holds
    few widths and large same-width groups (one kernel launch per group per
    epoch) instead of a sliver of every width."""
    order = sorted(range(len(costs)), key=lambda i: (-widths[i], -costs[i], i))
    total = float(sum(costs))
    out = [0] * len(costs)
    acc, b = 0.0, 0
    for i in order:
        # move to the next bin once this one holds its share (an item goes to
        # the bin whose share boundary its midpoint falls before)
        while b < n_bins - 1 and acc + 0.5 * costs[i] > total * (b + 1) / n_bins:
            b += 1
        out[i] = b
        acc += costs[i]
    return out


PARTITIONS = ("auto", "lpt", "blocked")


def auto_partition(n_ranks: int) -> str:
    """Measured on the 280-fit sweep (tools/rank_probe.py, every rank's share
    alone on one MI355X, profiles/r02/rank_probe_*.log): width-blocked shares
    win at 2 ranks (52.5 vs 49.5 predicted fits/s: each rank keeps 40-fit
    groups), LPT wins from 4 ranks on (94 vs 88 at 4, 177 vs 148 at 8: a rank of
    W=512 fits alone leaves the chip underused, a mix overlaps them with W=256
    kernels on the other streams)."""
    return "blocked" if n_ranks == 2 else "lpt"


def rank_share(costs: list, n_ranks: int, rank: int, widths: list | None = None,
               partition: str | None = None) -> list:
    """Indices of the fits rank `rank` trains (deterministic on every rank).
    partition: 'lpt' (longest processing time first over all fits),
    'blocked' (width-contiguous runs, needs `widths`) or 'auto'
    (auto_partition); default NERFHIP_FARM_PARTITION or 'auto'."""
    if n_ranks <= 1:
        return list(range(len(costs)))
    partition = partition or os.environ.get("NERFHIP_FARM_PARTITION", "auto")
    if partition == "auto":
        partition = auto_partition(n_ranks) if widths is not None else "lpt"
    if partition == "blocked" and widths is not None:
        owner = blocked_partition(costs, widths, n_ranks)
    elif partition in PARTITIONS:
        owner = lpt_partition(costs, n_ranks)
    else:
        raise ValueError(f"partition must be one of {PARTITIONS}, got {partition!r}")
    return [i for i, o in enumerate(owner) if o == rank]


def init_control_group() -> tuple:
    """gloo process group from the torch.distributed.run environment
    (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT).  Control traffic only."""
    n = int(os.environ.get("WORLD_SIZE", "1"))
    if n > 1 and not dist.is_initialized():
        dist.init_process_group("gloo")
    return world()


def barrier() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world()[0] > 1:
        dist.barrier()


def max_over_ranks(x: float) -> float:
    if world()[0] <= 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_records(local: dict) -> dict:
    """Union of every rank's {fit index: record} (host-side object gather)."""
    n, _ = world()
    if n <= 1:
        return dict(local)
    parts = [None] * n
    dist.all_gather_object(parts, local)
    out = {}
    for p in parts:
        out.update(p)
    return out


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list, script: str, poll_s: float = 0.2) -> int:
    """Run `python script argv…` as n ranks of one local job, the way
    torch.distributed.run would (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR =
    127.0.0.1, MASTER_PORT).  Must be called before this process touches the
    GPU: the ranks are fresh child processes, nothing is exec'd in place.  If
    one rank fails the others are terminated.  Returns the job's exit code."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(poll_s)
    return rc


# --------------------------------------------------------------------------
# in-library farm (fit_kv_cache(gpus=N), run_fits(devices=[…]))
# --------------------------------------------------------------------------

# Tensors cross the process boundary as numpy arrays: torch's multiprocessing
# pickler would share their storage by file descriptor, which dies with the
# worker that sends its outputs and exits.
_TENSOR_FIELDS = ("params", "target_mean", "target_std")


def _pack(o):
    for f in _TENSOR_FIELDS:
        setattr(o, f, getattr(o, f).detach().to("cpu").numpy())
    return o


def _unpack(o):
    for f in _TENSOR_FIELDS:
        setattr(o, f, torch.from_numpy(getattr(o, f)))
    return o


def _farm_worker(device: int, jobs: list, epochs: int, lr: float, log_every: int,
                 precision, conn) -> None:
    """One farm rank: train `jobs` [(target, config, init) as numpy] on
    `device`, send the outputs home."""
    try:
        from . import engine
        specs = [engine.FitSpec(target=torch.from_numpy(t), config=c, init=torch.from_numpy(i))
                 for t, c, i in jobs]
        outs = engine.run_fits(specs, epochs, lr=lr, log_every=log_every, devices=[device],
                               precision=precision)
        conn.send(("ok", [_pack(o) for o in outs]))
    except BaseException as e:   # report, then exit non-zero
        conn.send(("error", f"{type(e).__name__}: {e}"))
        raise
    finally:
        conn.close()


def run_farm(specs: list, epochs: int, devices: list, lr: float = 1e-4, log_every: int = 0,
             precision=None, timeout: float | None = None) -> list:
    """Train `specs` over `devices`, one worker process per device, each on its
    share: rank_share on the FLOP model with the partition auto_partition picks
    for this device count (width-blocked at 2, LPT from 4) or
    NERFHIP_FARM_PARTITION names.  Returns FitOutput per spec, in
    spec order, with `params` on the host and `device` naming where it
    trained.  Per-fit arithmetic does not depend on the device count beyond
    the engine's own group sizing (see engine.SPLIT_MAX_FITS)."""
    import multiprocessing as mp
    from .engine import fit_flops
    if not specs:
        return []
    costs = [fit_flops(int(s.target.shape[0]), int(s.target.shape[1]), s.config, 1)
             for s in specs]
    widths = [s.config.hidden_features for s in specs]
    n = len(devices)
    shares = [rank_share(costs, n, r, widths) for r in range(n)]
    ctx = mp.get_context("spawn")
    jobs = []
    for r, dev in enumerate(devices):
        if not shares[r]:
            continue
        # host copies as numpy: the worker owns its own device
        part = [(s.target.detach().to("cpu").numpy(), s.config, s.init.detach().to("cpu").numpy())
                for s in (specs[i] for i in shares[r])]
        recv, send = ctx.Pipe(duplex=False)
        p = ctx.Process(target=_farm_worker,
                        args=(dev, part, epochs, lr, log_every, precision, send), daemon=True)
        p.start()
        send.close()
        jobs.append((r, p, recv))
    outs = [None] * len(specs)
    err = None
    for r, p, recv in jobs:
        try:
            if timeout is not None and not recv.poll(timeout):
                raise TimeoutError(f"farm rank {r} sent nothing in {timeout}s")
            status, payload = recv.recv()
        except (EOFError, TimeoutError) as e:
            status, payload = "error", f"farm rank {r} died: {e}"
        if status != "ok":
            err = err or payload
        else:
            for i, o in zip(shares[r], payload):
                outs[i] = _unpack(o)
    for _r, p, _recv in jobs:
        p.join(timeout=60)
        if p.is_alive():
            p.terminate()
    if err is not None:
        from ._native import NerfhipError
        raise NerfhipError(f"fit farm failed: {err}")
    return outs
