"""bench.py — SIREN fits/sec on the 280-fit sweep (BASELINE.json metric).

One "step" = the whole 280-fit sweep (7 architectures × layers {0,8,16,24,31}
× heads 0-3 × K/V, seq_len 2048, 2000 Adam epochs each) trained from its
seed-0 initialisation, with every input already resident in HBM.  With
`--gpus N` (launched by torch.distributed.run, one process per GPU) the 280
fits are split over the ranks by longest-processing-time on their FLOP cost —
no collective touches the data path; a barrier and a max-over-ranks of the
elapsed time bracket the timed steps.  value = 280·steps / max time.

Precision (--precision, default bf16x3): the GEMMs run either on the exact
f32 MFMA ("fp32") or as exact 3-way bf16 splits with six bf16 MFMA products
per fp32 product and fp32 accumulation ("bf16x3": fp32-class accuracy,
nerfhip.h nerfhip_precision); everything else is fp32 in both.  Both are held
to the same per-fit parity bar (cos_delta_vs_ref).  With --also-fp32 (default
on at N=1) the line also carries the fp32 sweep, timed under the same
protocol (one warm-up, three timed sweeps).

Also reported (rank 0):
  roofline      the dominant kernel's algorithmic TFLOP/s against the
                matrix-core peak of its arithmetic (157.3 TFLOP/s f32 MFMA, or
                2.5 PFLOP/s bf16 dense / 6 products = 416.7 TFLOP/s
                fp32-equivalent for bf16x3).  `frac` / `achieved` /
                `avg_launch_ms` are the kernel on the engine's heaviest group
                of its width timed alone (hipEvents on 25 launches of a
                101-epoch run right after the timed region, the cold first
                launch excluded; the same leg under rocprofv3 is committed in
                profiles/r05, tools/r4/iso_prof.sh); `frac_concurrent` is the same
                kernel's launches inside the timed sweep, where ~7 group
                streams share the GPU; `job_frac` is the whole sweep's
                algorithmic rate;
  cpu_baseline  the package's own host path (nerf_attention/host_fit.py: the
                reference loop in eager PyTorch) timed on a bounded sample of
                the same workload on this host's CPUs (N=1 only);
  cos_delta_vs_ref  per-fit |Δ final_cosine_mean| against the reference's own
                seed-0 sweep (tests/golden/sweep_ref_seed0_e2000.json).
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

# one hardware queue per width-group stream (the engine runs ~7 streams per
# GPU; HIP's default of 4 queues makes some of them share a queue, in order:
# the 2000-epoch sweep measured 27.0 fits/s with 4, 27.7 with 8 on one box,
# profiles/r04/queues_ab.log).  The GPU boxes export HIP's default (4), so an
# unset value or HIP's default is raised to 8; any other explicit value wins,
# and NERFHIP_KEEP_HW_QUEUES=1 keeps even the default (4-vs-8 A/B).  Must be
# set before the HIP runtime initialises.
if (os.environ.get("NERFHIP_KEEP_HW_QUEUES") != "1"
        and os.environ.get("GPU_MAX_HW_QUEUES", "").strip() in ("", "4")):
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np
import torch
import torch.distributed as dist

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 / 16x16x4
BF16_MFMA_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 (no sparsity)
PEAK = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16x3": BF16_MFMA_PEAK_TFLOPS / 6}
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E 8 TB/s
RTX4060_FITS_PER_S = 0.232         # BASELINE.md §1 (280 fits / Σ train_time_seconds)
GOLDEN_SWEEP = ROOT / "tests" / "golden" / "sweep_ref_seed0_e2000.json"
PMC_TRAFFIC = ROOT / "profiles" / "pmc_traffic.json"


_T_START = time.perf_counter()


def progress(msg: str) -> None:
    """One progress line on stderr (the JSON result stays the only stdout line):
    a long default run under a profiler keeps writing, and a hang shows where."""
    print(f"[bench {time.perf_counter() - _T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def rows_flops(N, D, cfgs):
    """k_step_rows: forward + backward-dX GEMMs of one epoch (2·N·K·M each)."""
    return sum(4.0 * N * (c.hidden_layers * c.hidden_features ** 2 + c.hidden_features * D)
               for c in cfgs)


def params_flops(N, D, cfgs):
    """k_step_params: weight-gradient GEMMs of one epoch incl. the K=1 first layer."""
    return sum(2.0 * N * (c.hidden_layers * c.hidden_features ** 2 + c.hidden_features * D)
               + 2.0 * N * c.hidden_features for c in cfgs)


def host_cpus() -> dict:
    """The CPUs this process may use: the affinity mask, bounded by the cgroup
    CPU quota (a GPU box exposes the whole machine's CPUs in the mask but gives
    one GPU's job a share of them), and the CPU model."""
    logical = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = min(logical, quota) if quota else logical
    # one CPU of a quota left to the process's other threads (HIP runtime,
    # Python): with every quota CPU busy in torch the cgroup throttles the
    # whole process for part of each 100-ms period, which is where most of the
    # repeat spread came from (round 3: 11 s throttled in one run)
    if quota and quota >= 8 and threads == quota:
        threads -= 1
    return {"affinity_cpus": logical, "cgroup_cpu_quota": quota, "model": model,
            "threads": threads}


def cgroup_throttled_us() -> int | None:
    """Microseconds this cgroup has been throttled by its CPU quota (cpu.stat)."""
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k == "throttled_usec":
                return int(v)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(seq_len: int, sample_epochs: int, repeats: int = 3,
                 warmup_epochs: int = 10, sample_s: float | None = 2.0) -> dict:
    """Time the package's own host path (host_fit.fit_on_host: the reference
    loop, siren.py:80-149, in eager PyTorch) on every architecture: one untimed
    warm-up fit of `warmup_epochs` per architecture (thread pool, allocator,
    first-touch; it also prices the architecture), then `repeats` rounds over
    the architectures, on every CPU this process may use.  Each timed fit runs
    about `sample_s` seconds (its epoch count from the warm-up's per-epoch time,
    at least `sample_epochs` — so the cheap architectures are not timed over
    0.1-s windows that a co-tenant's burst or a CFS quota period dominates);
    sample_s=None: exactly `sample_epochs` each.  The median per-epoch time of
    each architecture is extrapolated to the 280-fit sweep (dense cost is
    data-independent)."""
    from nerf_attention import CONFIGS_FULL, SIREN
    from nerf_attention.host_fit import fit_on_host
    from nerf_attention.synthetic import kv_slice
    cpus = host_cpus()
    threads = cpus["threads"]
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    keys, _ = kv_slice(16, 2, seq_len=seq_len)
    samples = {c.name: [] for c in CONFIGS_FULL}
    thr0 = cgroup_throttled_us()
    epochs_of = {}

    def one(cfg, epochs):
        torch.manual_seed(0)
        m = SIREN(cfg, 128)
        return fit_on_host(keys, cfg, m, epochs, 1e-4, 0).train_time_seconds / epochs

    try:
        for cfg in CONFIGS_FULL:
            t = one(cfg, warmup_epochs)
            epochs_of[cfg.name] = sample_epochs if sample_s is None else \
                max(sample_epochs, int(round(sample_s / max(t, 1e-6))))
        for rep in range(repeats):
            for cfg in CONFIGS_FULL:
                samples[cfg.name].append(one(cfg, epochs_of[cfg.name]))
            progress(f"cpu baseline round {rep + 1}/{repeats}")
    finally:
        torch.set_num_threads(prev)
    per_epoch = {k: float(np.median(v)) for k, v in samples.items()}
    sweep_s = 40 * 2000 * sum(per_epoch.values())
    # spread of the repeats around the median: worst architecture, and weighted
    # by each architecture's share of the extrapolated sweep time
    spread_of = {k: (max(v) - min(v)) / float(np.median(v)) for k, v in samples.items()}
    spread = max(spread_of.values())
    tot = sum(per_epoch.values())
    spread_w = sum(spread_of[k] * per_epoch[k] / tot for k in per_epoch)
    timed_s = sum(epochs_of[k] * sum(v) for k, v in samples.items())
    thr1 = cgroup_throttled_us()
    cpus["throttled_s_during_baseline"] = (thr1 - thr0) / 1e6 if thr0 is not None and thr1 is not None \
        else None
    return {"value": 280.0 / sweep_s, "unit": "fits/s", "cores": threads, "kind": "port",
            "port": "package host path (nerf_attention/host_fit.py)",
            "sample": f"nerf_attention/host_fit.py (the reference loop in eager PyTorch), each of "
                      f"the 7 archs: 1 untimed warm-up of {warmup_epochs} epochs, then "
                      f"{repeats} rounds of one fit per arch of ~{sample_s}s (epochs "
                      f"{epochs_of}) on synthetic L16 H2 key [{seq_len},128], {timed_s:.1f}s "
                      f"timed in all; median per-epoch time per arch; sweep = "
                      f"40x2000x(sum of medians) = {sweep_s:.0f}s; {cpus['model']}, "
                      f"{threads} torch threads (affinity {cpus['affinity_cpus']} CPUs, "
                      f"cgroup quota {cpus['cgroup_cpu_quota']})",
            "host": cpus, "repeat_spread": round(spread, 4),
            "repeat_spread_kind": "(max - min) / median of the timed repeats, worst arch",
            "repeat_spread_weighted": round(spread_w, 4),
            "repeat_spread_weighted_kind": "per-arch (max - min) / median weighted by the arch's "
                                           "share of the extrapolated sweep time",
            "per_epoch_ms": {k: round(v * 1e3, 3) for k, v in per_epoch.items()},
            "spread_per_arch": {k: round((max(v) - min(v)) / float(np.median(v)), 4)
                                for k, v in samples.items()}}


def e2e_fit_kv_cache(seq_len: int, epochs: int, precision: str) -> dict:
    """SURVEY §8d primary metric: wall clock of the whole drop-in call
    `fit_kv_cache(kv_dir, out, epochs)` (metadata + layer loads + 280 inits in
    the reference order + training + result records + 40 medium checkpoints +
    fit_results.json), on the reference's on-disk cache format.  The cache
    (only the 5 layers the sweep reads, plus metadata.json) is written first,
    outside the timed call."""
    import contextlib
    import io
    import tempfile
    from nerf_attention import fit_kv_cache
    from nerf_attention.synthetic import write_kv_cache
    with tempfile.TemporaryDirectory(prefix="nerf_e2e_") as tmp:
        kv = Path(tmp) / "kv_cache"
        write_kv_cache(kv, seq_len=seq_len, num_layers=32, num_kv_heads=8, head_dim=128,
                       layers=[0, 8, 16, 24, 31])
        torch.manual_seed(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            recs = fit_kv_cache(kv, Path(tmp) / "fits", epochs=epochs, device="cuda",
                                precision=precision)
        dt = time.perf_counter() - t0
    return {"fits": len(recs), "seconds": round(dt, 3), "fits_per_s": round(len(recs) / dt, 4),
            "note": "whole fit_kv_cache call incl. loads, inits, D2H, checkpoints and JSON"}


ISO_EPOCHS = 101   # isolated leg: 25 timed launches (every 4th epoch from epoch 3)
# the committed rocprofv3 summary of exactly that leg (tools/r4/iso_prof.sh runs
# tools/r4/isokernel.py, which calls isolated_kernel below, under
# rocprofv3 --kernel-trace --stats, and its PMC passes)
ISO_PROFILE = "profiles/r06/rocprof_kernel_stats_isolated_256.csv"
ISO_PMC = ROOT / "profiles" / "r06" / "pmc_isolated_256.json"


def lib_sha16() -> str:
    """First 16 hex digits of the engine library's SHA-256: a committed PMC
    summary names the library it measured, and its bytes / MFMA-busy figures
    are reported only for that same library."""
    from nerf_attention import _build
    return hashlib.sha256(Path(os.environ.get("NERFHIP_LIB", _build.LIB)).read_bytes()).hexdigest()[:16]


def committed_pmc(path: Path, key: str, cur_lib: str):
    """The committed PMC summary of `key` (tools/r4/iso_summary.py), or None;
    a summary measured on another build of the library comes back as a stale
    marker without its figures (its bytes / MFMA busy would describe other
    code)."""
    if not path.exists():
        return None
    pmc = json.loads(path.read_text()).get(key)
    if pmc and pmc.get("lib_sha16") != cur_lib:
        return {"stale": True, "pmc_lib_sha16": pmc.get("lib_sha16"), "lib_sha16": cur_lib}
    return pmc


def heaviest_group(specs, width: int, device: int = 0) -> list:
    """Indices (into `specs`) of the engine's heaviest group of hidden width
    `width`, exactly as engine.plan_groups chunks the job (the sweep's W = 256
    group: the first of four 40-fit chunks)."""
    from nerf_attention import engine
    for _d, members in engine.plan_groups(specs, device):
        if specs[members[0]].config.hidden_features == width:
            return list(members)
    raise ValueError(f"no group of width {width}")


def isolated_kernel(gspecs, kname, flops, precision, peak, device,
                    epochs=ISO_EPOCHS) -> dict:
    """The dominant kernel's group trained alone (no concurrent groups) for
    `epochs` epochs: its undisturbed launch time (hipEvents around every 4th
    epoch's launches from epoch 3, so never the cold first one)."""
    from nerf_attention import engine
    job = engine.FitJob(gspecs, epochs, devices=[device], precision=precision)
    job.launch(timed=True)
    job.wait()
    t = job.timing[0]
    if t.launches == 0:
        raise ValueError(f"isolated leg needs >= 4 epochs (got {epochs}): no timed launch")
    ms = (t.rows_ms if "rows" in kname else t.params_ms) / t.launches
    other_ms = (t.params_ms if "rows" in kname else t.rows_ms) / t.launches
    tf = flops / (ms * 1e-3) / 1e12
    return {"avg_launch_ms": round(ms, 4), "achieved": round(tf, 2), "frac": round(tf / peak, 4),
            "frac_of_f32_mfma_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 4), "epochs": epochs,
            "launches": t.launches, "partner_kernel_avg_ms": round(other_ms, 4),
            "epoch_ms": round(job.group_seconds()[0] * 1e3 / epochs, 4)}


def fp32_sweep(specs, epochs, device, plan, ref_cos, n_total, warmup: int = 1,
               steps: int = 3) -> dict:
    """The exact f32 MFMA path timed under the headline's protocol (same fits,
    same parity bar): `warmup` untimed sweeps, then `steps` timed sweeps
    bracketed by device synchronisation."""
    from nerf_attention import engine
    job = engine.FitJob(specs, epochs, devices=[device], precision="fp32")
    for _ in range(warmup):
        job.launch()
        job.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        job.launch()
        job.wait()
        progress("fp32 step done")
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {"value": round(len(specs) / dt, 4), "unit": "fits/s", "ms_per_step": round(dt * 1e3, 2),
           "warmup": warmup, "steps": steps,
           "note": f"{warmup} untimed warm-up sweep(s), then {steps} timed sweeps (the headline's "
                   "protocol)"}
    if ref_cos is not None and GOLDEN_SWEEP.exists():
        ref = {r["name"]: r["final_cosine_mean"]
               for r in json.loads(GOLDEN_SWEEP.read_text())["records"]}
        d = np.array([abs(float(torch.from_numpy(o.row_cos).mean()) - ref[plan[i][0]])
                      for i, o in enumerate(job.outputs())])
        out["cos_delta_vs_ref"] = {"max": float(d.max()), "mean": float(d.mean()),
                                   "within_1e-3": int((d <= 1e-3).sum()), "n": int(d.size)}
    return out


def dry_run(args, world: int, rank: int) -> None:
    """The multi-rank protocol of main() with the device work left out: every
    rank takes its LPT share of the sweep's FLOP costs, 'trains' nothing, and
    the shares meet in the same barrier / max / gather; rank 0 prints a line
    with the rank count and the union of the shares (tests drive this on CPU)."""
    from nerf_attention import CONFIGS_FULL, engine, farm
    costs = [engine.fit_flops(args.seq_len, 128, c, args.epochs) for c in CONFIGS_FULL] * 40
    widths = [c.hidden_features for c in CONFIGS_FULL] * 40
    mine = farm.rank_share(costs, world, rank, widths)
    farm.barrier()
    t0 = time.perf_counter()
    share_flops = sum(costs[i] for i in mine)
    farm.barrier()
    t_max = farm.max_over_ranks(time.perf_counter() - t0)
    merged = farm.gather_records({i: rank for i in mine})
    loads = farm.gather_records({rank: share_flops})
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": world,
                          "fits": sorted(merged), "owner": [merged[i] for i in sorted(merged)],
                          "rank_flops": [loads[r] for r in range(world)],
                          "max_elapsed_s": t_max}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=2000)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--cpu-sample-epochs", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"])
    ap.add_argument("--also-fp32", dest="also_fp32", action="store_true", default=None,
                    help="also time one fp32 sweep (default: on at N=1 with bf16x3)")
    ap.add_argument("--no-also-fp32", dest="also_fp32", action="store_false")
    ap.add_argument("--no-e2e", action="store_true", help="skip the fit_kv_cache wall-clock leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher self-test without a GPU: rank spawn, gloo group, LPT shares, "
                         "barrier, max-over-ranks and record gather, no device work")
    args = ap.parse_args()

    from nerf_attention import farm
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start one rank per GPU ourselves (fresh child processes,
        # before this process has touched the GPU) and exit with the job's code
        sys.exit(farm.spawn_ranks(args.gpus, sys.argv[1:], str(Path(__file__).resolve())))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    # control collectives only (barrier, max of the elapsed time, record
    # gather): gloo on the host, no RCCL communicator at all
    farm.init_control_group()
    if args.dry_run:
        return dry_run(args, world, rank)
    # one GPU per rank; more ranks than GPUs (a rehearsal of the N-rank path on
    # a smaller box) share them round-robin.  device_count() does not
    # initialise HIP.
    n_dev = torch.cuda.device_count()
    local = local % n_dev if n_dev else local
    torch.cuda.set_device(local)

    from nerf_attention import engine
    from nerf_attention.workloads import sweep_280

    plan, specs = sweep_280(args.seq_len, seed=0)
    n_total = len(specs)
    costs = [engine.fit_flops(args.seq_len, 128, s.config, args.epochs) for s in specs]
    widths = [s.config.hidden_features for s in specs]
    mine = farm.rank_share(costs, world, rank, widths)
    job = engine.FitJob([specs[i] for i in mine], args.epochs, devices=[local],
                        precision=args.precision)
    progress(f"rank {rank}: {len(mine)} fits in {len(job.groups)} groups, warm-up")

    for _ in range(args.warmup):
        job.launch()
        job.wait()
    progress("warm-up done, timed steps")

    barrier = farm.barrier
    barrier()
    t0 = time.perf_counter()
    kt = [[0.0, 0.0, 0] for _ in job.groups]       # per group: rows ms, params ms, launches
    for _ in range(args.steps):
        job.launch(timed=not args.no_kernel_timing)
        job.wait()
        for acc, t in zip(kt, job.timing or []):
            acc[0] += t.rows_ms
            acc[1] += t.params_ms
            acc[2] += t.launches
        progress("timed step done")
    barrier()
    elapsed = time.perf_counter() - t0
    t_max = farm.max_over_ranks(elapsed)

    # per-fit results for the parity summary (host-side gather; not timed)
    outs = job.outputs()
    my_cos = {mine[k]: float(torch.from_numpy(o.row_cos).mean()) for k, o in enumerate(outs)}
    all_cos = farm.gather_records(my_cos)

    if rank == 0:
        value = n_total * args.steps / t_max
        roof = None
        if any(k[2] for k in kt):
            # dominant kernel = largest summed device time over the timed steps,
            # summed over every group (chunk) of that width
            N = args.seq_len
            per_kernel = {}     # name -> [total ms, launches, total flops, heaviest group]
            for g, (r_ms, p_ms, n) in zip(job.groups, kt):
                if n == 0:
                    continue
                cf = [specs[mine[i]].config for i in g.members]
                for name, ms, fl in ((f"k_step_rows<{g.W},128>", r_ms, rows_flops(N, 128, cf)),
                                     (f"k_step_params<{g.W},128>", p_ms,
                                      params_flops(N, 128, cf))):
                    acc = per_kernel.setdefault(name, [0.0, 0, 0.0, None, 0.0])
                    acc[0] += ms
                    acc[1] += n
                    acc[2] += fl * n
                    if ms > acc[4]:
                        acc[3], acc[4] = g, ms
            kname, (tot_ms, n_launch, tot_flops, g, _) = max(per_kernel.items(),
                                                             key=lambda kv: kv[1][0])
            avg_ms = tot_ms / n_launch
            flops = tot_flops / n_launch
            achieved = tot_flops / (tot_ms * 1e-3) / 1e12
            traffic = None
            if PMC_TRAFFIC.exists():
                traffic = json.loads(PMC_TRAFFIC.read_text()).get(f"{kname}[{args.precision}]")
            step_flops = sum(engine.fit_flops(N, 128, specs[i].config, args.epochs)
                             for i in mine)
            peak = PEAK[args.precision]
            job_tf = step_flops / (t_max / args.steps) / 1e12
            hbm = None
            if traffic:
                # PMC bytes per launch (separate, serialised rocprofv3 passes of the
                # same workload, tools/profile_round.sh) over this run's launch time
                hbm = traffic["bytes"] / (avg_ms * 1e-3) / 1e9
            # the isolated leg: the engine's heaviest group of the dominant width
            # (deterministic, the same group tools/r4/isokernel.py profiles)
            my_specs = [specs[i] for i in mine]
            gw = int(kname.split("<")[1].split(",")[0])
            gsel = heaviest_group(my_specs, gw, local)
            gcf = [my_specs[i].config for i in gsel]
            g_flops = (rows_flops if "rows" in kname else params_flops)(N, 128, gcf)
            progress(f"isolated {kname}")
            iso = isolated_kernel([my_specs[i] for i in gsel], kname, g_flops,
                                  args.precision, peak, local)
            iso["fits"] = len(gsel)
            sha = lib_sha16()
            iso_pmc = committed_pmc(ISO_PMC, f"{kname}[{args.precision}]", sha)
            iso_bytes = iso_pmc and iso_pmc.get("bytes")
            hbm_iso = iso_bytes and iso_bytes / (iso["avg_launch_ms"] * 1e-3) / 1e9
            alg_bytes = sum(4 * N * 128 + 24 * c.num_parameters(128) for c in gcf)
            # the chunk-epoch: the row and the parameter kernel of the same
            # isolated group, both counted
            pname = (kname.replace("k_step_rows", "k_step_params") if "rows" in kname
                     else kname.replace("k_step_params", "k_step_rows"))
            partner_pmc = committed_pmc(ISO_PMC, f"{pname}[{args.precision}]", sha)
            partner_bytes = partner_pmc and partner_pmc.get("bytes")
            epoch_bytes = iso_bytes and partner_bytes and iso_bytes + partner_bytes
            roof = {"bound": "mfma", "achieved": iso["achieved"],
                    "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": iso["frac"],
                    "frac_kind": "dominant kernel on the engine's heaviest group of its width, "
                                 "timed alone right after the timed region: algorithmic FLOPs "
                                 f"per launch / mean hipEvent launch duration ({iso['launches']} "
                                 f"launches of {iso['epochs']} epochs, cold first launch "
                                 "excluded)",
                    "avg_launch_ms": iso["avg_launch_ms"], "flops_per_launch": g_flops,
                    "fits_per_launch": len(gsel),
                    "rocprof_isolated": ISO_PROFILE,
                    "rocprof_isolated_avg_ms": iso_pmc and iso_pmc.get("rocprof_avg_ms"),
                    "traffic": iso_bytes,
                    "traffic_detail": iso_pmc,
                    "traffic_source": "rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes of the "
                                      "same isolated group (tools/r4/iso_prof.sh, "
                                      f"{ISO_PMC.relative_to(ROOT)})",
                    "mfma_busy": iso_pmc and iso_pmc.get("mfma_busy"),
                    "algorithmic_bytes": alg_bytes,
                    "algorithmic_bytes_kind": "SURVEY.md §8d per fit-epoch 4·N·D target + 24·P "
                                              "params/Adam read+write, x fits of the group "
                                              "(activations assumed on-chip)",
                    "traffic_chunk_epoch": epoch_bytes,
                    "traffic_chunk_epoch_kind": f"PMC bytes of {kname} + {pname} per epoch of "
                                                "the isolated group (FETCH_SIZE x2 + WRITE_SIZE)",
                    "partner_traffic_detail": partner_pmc,
                    "traffic_over_algorithmic": epoch_bytes and round(epoch_bytes / alg_bytes, 2),
                    "dominant_over_algorithmic": iso_bytes and round(iso_bytes / alg_bytes, 2),
                    "mfma_busy_kind": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GPU-active "
                                      "cycles), rocprofv3 PMC pass of the same isolated group",
                    "hbm_gbs": hbm_iso and round(hbm_iso, 1),
                    "hbm_frac": hbm_iso and round(hbm_iso / HBM_PEAK_GBS, 4),
                    "sweep_context_traffic": traffic and traffic["bytes"],
                    "sweep_context_mfma_busy": traffic and traffic.get("mfma_busy"),
                    "kernel": f"{kname} [{args.precision}]",
                    "flops_unit": "algorithmic fp32 GEMM FLOPs (2 per multiply-add), "
                                  "SURVEY.md §8d",
                    "peak_basis": ("f32 MFMA" if args.precision == "fp32" else
                                   "bf16 MFMA 2.5 PF dense / 6 bf16 products per fp32 product"),
                    "isolated": iso,
                    "frac_concurrent": round(achieved / peak, 4),
                    "concurrent": {
                        "achieved": round(achieved, 3), "avg_launch_ms": round(avg_ms, 4),
                        "flops_per_launch": flops,
                        "fits_per_launch": round(sum(x.n for x in job.groups
                                                     if f"<{x.W}," in kname) /
                                                 sum(1 for x in job.groups if f"<{x.W}," in kname),
                                                 2),
                        "hbm_gbs": hbm and round(hbm, 1),
                        "note": "the same kernel's launches inside the timed sweep (every 4th "
                                "epoch), summed over every group of its width, while ~7 group "
                                "streams share the GPU: a share of the chip, not a kernel "
                                "property"},
                    "kernels_avg_ms_concurrent": {k: round(v[0] / v[1], 4)
                                                  for k, v in per_kernel.items()},
                    "groups": len(job.groups),
                    "job_achieved_tflops": round(job_tf, 2),
                    "job_frac": round(job_tf / peak, 4),
                    "job_frac_of_f32_mfma_peak": round(job_tf / FP32_MFMA_PEAK_TFLOPS, 4)}
        parity = None
        if GOLDEN_SWEEP.exists() and args.epochs == 2000 and args.seq_len == 2048:
            ref = json.loads(GOLDEN_SWEEP.read_text())["records"]
            names = [p[0] for p in plan]
            byname = {r["name"]: r["final_cosine_mean"] for r in ref}
            d = np.array([abs(all_cos[i] - byname[names[i]]) for i in range(n_total)])
            parity = {"max": float(d.max()), "mean": float(d.mean()), "n": int(d.size),
                      "within_1e-3": int((d <= 1e-3).sum())}
        line = {
            "metric": "SIREN fits/sec (280-fit sweep) at 1/2/4/8 GPUs; cos-sim Δ vs ref",
            "value": round(value, 4), "unit": "fits/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(value / RTX4060_FITS_PER_S, 2),
            "ranks_seen": world, "control_backend": "gloo" if world > 1 else None,
            "devices_visible": torch.cuda.device_count(),
            "dtype": "f32" if args.precision == "fp32" else "f32 (bf16x3 split MFMA)",
            "precision": args.precision, "data": "synthetic",
            "config": {"workload": "280-fit sweep: 7 archs x layers{0,8,16,24,31} x heads0-3 x "
                                   "K/V on the reference's synthetic KV (32x8xNx128), "
                                   "seed-0 inits in reference order",
                       "seq_len": args.seq_len, "epochs": args.epochs, "fits": n_total,
                       "parallelism": f"fit-farm over {world} GPU(s), "
                                      f"{farm.auto_partition(world) if world > 1 else 'one'} "
                                      f"partition by FLOPs, gloo control only"},
            "roofline": roof,
            "cos_delta_vs_ref": parity,
        }
        also = args.also_fp32 if args.also_fp32 is not None else args.precision != "fp32"
        if world == 1 and also:
            progress("fp32 sweep")
            line["fp32_mfma"] = fp32_sweep([specs[i] for i in mine], args.epochs, local, plan,
                                           all_cos if parity else None, n_total)
        if world == 1 and not args.no_e2e:
            progress("e2e fit_kv_cache")
            line["e2e_fit_kv_cache"] = e2e_fit_kv_cache(args.seq_len, args.epochs, args.precision)
            line["e2e_fits_per_s"] = line["e2e_fit_kv_cache"]["fits_per_s"]
        if world == 1 and not args.no_cpu_baseline:
            progress("cpu baseline")
            line["cpu_baseline"] = cpu_baseline(args.seq_len, args.cpu_sample_epochs)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def report_children() -> None:
    """Every process this one started that is still alive, on stderr (the
    driver's record showed one process outliving bench.py)."""
    try:
        import psutil
        kids = psutil.Process().children(recursive=True)
    except Exception as e:                              # psutil missing / no /proc
        progress(f"children at exit: unknown ({e})")
        return
    progress(f"children at exit: {len(kids)}" + "".join(
        f"; pid {k.pid} {' '.join(k.cmdline())[:160]}" for k in kids if k.is_running()))


if __name__ == "__main__":
    main()
    report_children()
