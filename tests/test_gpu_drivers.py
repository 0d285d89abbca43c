"""The drop-in drivers and the BASELINE configs end to end on the MI355X,
against results of the reference itself (tests/golden/make_golden.py):

* config 3, the 280-fit sweep at seq 2048 / 2000 epochs, every fit against
  the reference's own seed-0 sweep (sweep_ref_seed0_e2000.json);
* the per-rank shares of a 2- and an 8-GPU farm (smaller groups: the split-K
  gradient path) trained alone, against the same golden;
* config 4's seq-len points 512 / 1024 / 4096: the medium fits the
  reference's scaling experiment runs per length (scan_medium_e2000.json);
* `fit_kv_cache(quick=True)` and `python -m nerf_attention.fit --quick`
  against the reference's own quick run (schema_quick/: records, key order,
  checkpoint layout, stdout structure);
* the one-process-per-GPU farm (two workers) equal to one process, bitwise.

Tolerance: north_star's ±1e-3 on every fit's final cosine.  All GPU work goes
through the C ABI (libnerfhip.so).
"""

import json
import os
import re
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from nerf_attention import SIREN, SIRENConfig, engine, farm

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3
ROOT = Path(__file__).resolve().parent.parent


def _cos(o):
    return float(torch.from_numpy(o.row_cos).mean())


@pytest.fixture(scope="module")
def sweep():
    from nerf_attention.workloads import sweep_280
    plan, specs = sweep_280(2048, seed=0)
    return plan, specs


def _ref_sweep(golden_dir):
    recs = json.loads((golden_dir / "sweep_ref_seed0_e2000.json").read_text())["records"]
    return {r["name"]: r for r in recs}


def test_sweep_280_vs_reference(gpu, golden_dir, sweep):
    """BASELINE config 3 on one GPU: all 280 fits within 1e-3 of the reference."""
    plan, specs = sweep
    ref = _ref_sweep(golden_dir)
    outs = engine.run_fits(specs, 2000, devices=[0])
    d = np.array([abs(_cos(o) - ref[p[0]]["final_cosine_mean"]) for p, o in zip(plan, outs)])
    assert d.size == 280 and d.max() <= COS_TOL, (d.max(), plan[int(d.argmax())][0])
    mse = np.array([o.final_mse / ref[p[0]]["final_mse"] for p, o in zip(plan, outs)])
    assert np.abs(mse - 1).max() <= 0.05
    # train_time_seconds is measured: the device interval of the group that
    # trained the fit (siren.py:96,117's loop wall clock); the longest group is
    # the sweep's training time
    assert all(o.train_time_seconds == o.group_seconds > 0 for o in outs)
    groups = {}
    for o in outs:
        groups.setdefault((o.group_seconds, o.plan["rows_workgroups"]), []).append(o)
    assert len(groups) >= 7                                    # one interval per group / chunk
    for members in groups.values():                            # FLOP shares split each interval
        assert abs(sum(o.flop_share_seconds for o in members) / members[0].group_seconds - 1) <= 1e-6


@pytest.mark.parametrize("world,rank", [(8, 0), (2, 1)])
def test_rank_share_vs_reference(gpu, golden_dir, sweep, world, rank):
    """What one rank of a `world`-GPU farm trains, alone on one GPU: its
    groups are smaller, yet every fit stays within 1e-3.  At 8 ranks the
    W = 512, 128 and 64 groups hold 5 fits each, and the W = 128 and 64 ones
    take the split-K weight-gradient path (16 row slices + k_adam_split)
    WHILE the W = 256 and 512 groups train beside them on the same GPU — the
    job of the round-5 concurrent split-K fault, whose containment
    (engine.split_allowed) round 6 removed."""
    plan, specs = sweep
    ref = _ref_sweep(golden_dir)
    costs = [engine.fit_flops(2048, 128, s.config, 2000) for s in specs]
    mine = farm.rank_share(costs, world, rank, [s.config.hidden_features for s in specs])
    outs = engine.run_fits([specs[i] for i in mine], 2000, devices=[0])
    d = np.array([abs(_cos(o) - ref[plan[i][0]]["final_cosine_mean"]) for i, o in zip(mine, outs)])
    assert d.max() <= COS_TOL, (d.max(), plan[mine[int(d.argmax())]][0])
    if world == 8:
        split = {(o.plan["grad_split"], o.plan["launches_per_epoch"]) for i, o in zip(mine, outs)
                 if specs[i].config.hidden_features <= 128}
        assert split == {(16, 3)}, split
        assert {o.plan["grad_split"] for i, o in zip(mine, outs)
                if specs[i].config.hidden_features >= 256} == {1}


@pytest.mark.parametrize("seq_len", [512, 1024, 4096])
def test_scan_points_vs_reference(gpu, golden_dir, seq_len):
    """BASELINE config 4's seq-len points: medium fits of layers {0, 16, 31},
    head 0, K and V (experiments/scaling.py:160-168) against the reference."""
    from nerf_attention.synthetic import kv_slice
    g = json.loads((golden_dir / "scan_medium_e2000.json").read_text())[str(seq_len)]
    cfg = SIRENConfig(256, 2, 30.0, "medium")
    torch.manual_seed(0)
    init = SIREN(cfg, 128).flat_parameters()
    specs = []
    for r in g["records"]:
        k, v = kv_slice(r["layer"], 0, seq_len=seq_len)
        specs.append(engine.FitSpec(target=k if r["kv_type"] == "key" else v, config=cfg,
                                    init=init))
    outs = engine.run_fits(specs, 2000, devices=[0])
    for r, o in zip(g["records"], outs):
        assert abs(_cos(o) - r["final_cosine_mean"]) <= COS_TOL, (r["name"], _cos(o))
        np.testing.assert_allclose(o.losses[::100][:5], r["losses_every100"][:5], rtol=1e-3)


def test_config2_lone_medium_fit_vs_reference(gpu, golden_dir, sweep):
    """BASELINE config 2 on its exact path: L0_H0_key_medium (seq 2048, 2000
    epochs) alone, from its sweep-order init, against the reference's own
    seed-0 sweep.  A lone fit takes the small-group kernels: K-split rows and
    8 gradient row slices on 64 x 64 tiles + k_adam_split (3 launches per
    epoch).  fit_siren,
    the reference's entry point, drawing the same init from the same RNG
    state, runs that same path (bitwise-equal result)."""
    from nerf_attention import fit_siren
    plan, specs = sweep
    ref = _ref_sweep(golden_dir)
    names = [p[0] for p in plan]
    i = names.index("L0_H0_key_medium")
    assert names[:i] == ["L0_H0_key_tiny", "L0_H0_key_small"]
    out = engine.run_fits([specs[i]], 2000, devices=[0])[0]
    assert out.plan["rows_variant"] == "ksplit", out.plan
    assert out.plan["grad_split"] == 8 and out.plan["launches_per_epoch"] == 3, out.plan
    assert out.plan["params_workgroups"] == 8 * 44, out.plan      # 64 x 64 tiles
    cos = _cos(out)
    assert abs(cos - ref["L0_H0_key_medium"]["final_cosine_mean"]) <= COS_TOL, cos
    assert abs(out.final_mse / ref["L0_H0_key_medium"]["final_mse"] - 1) <= 0.05
    cfg = plan[i][4]
    torch.manual_seed(0)
    for c in plan[0][4], plan[1][4]:                    # the sweep's first two inits
        SIREN(c, 128)
    res = fit_siren(specs[i].target, cfg, epochs=2000, device="cuda", verbose=False)
    assert torch.equal(res.model.cpu().flat_parameters(), out.params.cpu())
    assert res.final_cosine_mean == cos


def test_config4_scan_all_layers_heads_vs_reference(gpu, golden_dir, tmp_path):
    """BASELINE config 4 at its stated size for one length: medium on all 32
    layers x 8 heads x K/V (512 fits) at seq 512, 200 epochs, through the
    drop-in fit_kv_cache(select='all', configs=['medium']) from one
    manual_seed(0).  The scaling experiment's fits (layers {0, 16, 31}, head 0;
    experiments/scaling.py:160-168) match the reference trained from the same
    sweep-order RNG state (scan_all_medium_e200.json, make_golden.py
    scan_all); every fit's record is complete and finite."""
    from nerf_attention.fit import fit_kv_cache
    from nerf_attention.synthetic import write_kv_cache
    g = json.loads((golden_dir / "scan_all_medium_e200.json").read_text())
    kv = tmp_path / "kv"
    write_kv_cache(kv, seq_len=g["seq_len"])
    torch.manual_seed(g["seed"])
    recs = fit_kv_cache(kv, tmp_path / "out", epochs=g["epochs"], device="cuda", select="all",
                        configs=["medium"])
    assert len(recs) == g["n_fits"] == 512
    assert all(np.isfinite(r["final_cosine_mean"]) and np.isfinite(r["final_mse"]) for r in recs)
    for r in g["records"]:
        got = recs[r["index"]]
        assert got["name"] == r["name"]
        assert abs(got["final_cosine_mean"] - r["final_cosine_mean"]) <= COS_TOL, (r["name"], got)
        assert abs(got["final_mse"] / r["final_mse"] - 1) <= 0.02, (r["name"], got)


def _quick_cache(tmp):
    from nerf_attention.synthetic import extract_kv_cache_synthetic
    kv = Path(tmp) / "kv"
    extract_kv_cache_synthetic(seq_len=512, num_layers=4, num_kv_heads=4, head_dim=128,
                               output_dir=kv)
    return kv


_NUM = re.compile(r" *-?\d+\.\d+")   # with its right-aligned padding


def _shape(text: str) -> list:
    """stdout line structure: numbers masked, the device name normalised."""
    return [_NUM.sub(" #", l).replace("Device: cuda", "Device: cpu") for l in text.splitlines()]


def _check_quick_outputs(golden_dir, recs, out_dir):
    ref = json.loads((golden_dir / "schema_quick" / "fit_results.json").read_text())
    layout = json.loads((golden_dir / "schema_quick" / "checkpoint_layout.json").read_text())
    assert [list(r) for r in recs] == [list(r) for r in ref]              # names + key order
    ints = ("layer", "head", "hidden_features", "hidden_layers", "raw_size_bytes",
            "siren_size_bytes", "num_parameters", "seq_len", "d_head")
    for a, b in zip(recs, ref):
        assert all(a[k] == b[k] for k in ints + ("name", "kv_type", "config_name", "omega_0"))
        assert abs(a["final_cosine_mean"] - b["final_cosine_mean"]) <= COS_TOL, a["name"]
        assert a["compression_ratio"] == pytest.approx(b["compression_ratio"])
    saved = json.loads((out_dir / "fit_results.json").read_text())
    assert saved == json.loads(json.dumps(recs))
    cks = sorted(out_dir.glob("*_model.pt"))
    assert len(cks) == 6
    ck = torch.load(out_dir / "L0_H0_key_medium_model.pt", weights_only=True)
    assert list(ck) == layout["top_keys"]
    assert list(ck["model_state"]) == layout["model_state_keys"]
    assert {k: list(v.shape) for k, v in ck["model_state"].items()} == \
        layout["model_state_shapes"]
    assert ck["config"] == layout["config"]
    assert list(ck["metrics"]) == layout["metrics_keys"]


def test_fit_kv_cache_quick_vs_reference(gpu, golden_dir, tmp_path, capsys):
    """fit_kv_cache(quick=True) end to end on the GPU — the drop-in driver
    (fit.py:20-92) against the reference's own quick run."""
    from nerf_attention import fit_kv_cache
    kv = _quick_cache(tmp_path)
    capsys.readouterr()
    torch.manual_seed(0)
    recs = fit_kv_cache(kv, tmp_path / "fits", epochs=20, device="cuda", quick=True)
    out = capsys.readouterr().out
    _check_quick_outputs(golden_dir, recs, tmp_path / "fits")
    ref_out = (golden_dir / "schema_quick" / "stdout.txt").read_text()
    assert _shape(out) == _shape(ref_out)


def test_fit_cli_quick(gpu, golden_dir, tmp_path):
    """`python -m nerf_attention.fit --quick` (fit.py:183-196) in a fresh process."""
    kv = _quick_cache(tmp_path)
    env = dict(os.environ, PYTHONPATH=str(ROOT / "nerf-attention_amd"))
    r = subprocess.run([sys.executable, "-m", "nerf_attention.fit", "--kv_dir", str(kv),
                        "--output_dir", str(tmp_path / "fits"), "--epochs", "20", "--quick",
                        "--seed", "0"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = json.loads((tmp_path / "fits" / "fit_results.json").read_text())
    _check_quick_outputs(golden_dir, recs, tmp_path / "fits")
    ref_out = (golden_dir / "schema_quick" / "stdout.txt").read_text()
    lines = _shape(r.stdout)
    assert lines[:-1] == _shape(ref_out) + [""] and "sweep wall clock" in lines[-1]


def test_farm_two_workers_equal_one_process(gpu, monkeypatch):
    """run_fits over two devices = two farm worker processes (here both on
    GPU 0): every fit bitwise equal to training it in this process.  (The
    split-K path is off on both sides here: a worker's groups hold two tiny
    fits, a lone fit is a one-fit group, and the split-K slice count follows
    the group's grid; test_farm_lone_split_fits_bitwise covers split-K.)"""
    from nerf_attention.synthetic import kv_slice
    monkeypatch.setenv("NERFHIP_SPLIT_MAX_FITS", "0")
    keys, vals = kv_slice(5, 1, seq_len=256)
    cfgs = [SIRENConfig(64, 1, 30.0, "tiny"), SIRENConfig(128, 1, 30.0, "small"),
            SIRENConfig(256, 2, 30.0, "medium"), SIRENConfig(64, 1, 30.0, "tiny")]
    specs = []
    for i, c in enumerate(cfgs):
        torch.manual_seed(i)
        specs.append(engine.FitSpec(target=keys if i % 2 else vals, config=c,
                                    init=SIREN(c, 128).flat_parameters()))
    farmed = engine.run_fits(specs, 40, devices=[0, 0])
    for s, f in zip(specs, farmed):
        alone = engine.run_fits([s], 40, devices=[0])[0]
        assert torch.equal(alone.params.cpu(), f.params.cpu())
        assert alone.losses == f.losses


def test_farm_lone_split_fits_bitwise(gpu, monkeypatch):
    """Split-K in and out of the farm: two fits of different
    widths over two farm workers — each worker trains ONE one-fit group on the
    split-K path — are bitwise the fits trained alone in this process, and
    bitwise the same two fits trained together in one process (two concurrent
    split-K groups on one device: the split choice depends on the group's
    shape only, engine.wants_split)."""
    from nerf_attention.synthetic import kv_slice
    monkeypatch.delenv("NERFHIP_SPLIT_MAX_FITS", raising=False)
    keys, vals = kv_slice(3, 2, seq_len=512)
    cfgs = [SIRENConfig(256, 2, 30.0, "medium"), SIRENConfig(128, 1, 30.0, "small")]
    specs = []
    for i, c in enumerate(cfgs):
        torch.manual_seed(10 + i)
        specs.append(engine.FitSpec(target=(keys, vals)[i], config=c,
                                    init=SIREN(c, 128).flat_parameters()))
    farmed = engine.run_fits(specs, 60, devices=[0, 0])
    together = engine.run_fits(specs, 60, devices=[0])
    for s, f, t in zip(specs, farmed, together):
        alone = engine.run_fits([s], 60, devices=[0])[0]
        assert alone.plan["grad_split"] > 1 and t.plan["grad_split"] == alone.plan["grad_split"]
        for o in (f, t):
            assert torch.equal(alone.params.cpu(), o.params.cpu())
            assert alone.losses == o.losses


def test_forward_positions_autograd_and_short_inputs(gpu):
    """SIREN.forward keeps autograd w.r.t. the positions and answers shapes
    the engine does not take (one position) like the plain module."""
    cfg = SIRENConfig(256, 2, 30.0, "medium")
    torch.manual_seed(1)
    m = SIREN(cfg, 128).cuda().eval()
    m.requires_grad_(False)
    x = torch.linspace(0, 1, 64, device="cuda").unsqueeze(1).requires_grad_(True)
    y = m(x)
    assert y.grad_fn is not None
    y.sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    with torch.no_grad():
        one = torch.tensor([[0.25]], device="cuda")
        torch.testing.assert_close(m(one), m.network(one))


REF_LATENCY_KEYS = ['name', 'config', 'siren_time_ms', 'hbm_time_4060_ms', 'hbm_time_h100_ms',
                    'speedup_vs_4060', 'speedup_vs_h100', 'num_params']     # evaluate.py:206-215


def test_latency_harness(gpu, tmp_path, capsys):
    """evaluate.profile_latency / scaling._profile_siren_latency restated
    (latency.py) on checkpoints written by the drop-in driver: record keys in
    the reference's order (plus the MI355X fields), HBM times by the
    reference's formula, one stdout line per model, latency_results.json."""
    from nerf_attention import fit_kv_cache
    from nerf_attention.latency import profile_latency, profile_siren_latency
    kv = _quick_cache(tmp_path)
    torch.manual_seed(0)
    fit_kv_cache(kv, tmp_path / "fits", epochs=20, device="cuda", quick=True)
    capsys.readouterr()
    recs = profile_latency(tmp_path / "fits", tmp_path / "lat", device="cuda")
    out = [l for l in capsys.readouterr().out.splitlines() if l.strip()]
    assert len(recs) == 6 and len(out) == 6
    saved = json.loads((tmp_path / "lat" / "latency_results.json").read_text())
    assert saved == json.loads(json.dumps(recs))
    raw = 512 * 128 * 2
    for r, line in zip(recs, out):
        assert list(r)[:8] == REF_LATENCY_KEYS
        assert r["config"] == "medium" and r["num_params"] == 164992
        assert r["hbm_time_4060_ms"] == pytest.approx(raw / 272e9 * 1000)
        assert r["hbm_time_h100_ms"] == pytest.approx(raw / 3350e9 * 1000)
        assert r["speedup_vs_4060"] == pytest.approx((raw / 272e9) / (r["siren_time_ms"] / 1e3))
        assert 0 < r["siren_device_time_ms"] < 50 and 0 < r["siren_time_ms"] < 50
        assert re.fullmatch(rf"  {r['name']}: SIREN=\d+\.\d{{3}}ms \| HBM\(4060\)=\d+\.\d{{3}}ms \| "
                            rf"HBM\(H100\)=\d+\.\d{{3}}ms", line)
    assert 0 < profile_siren_latency(tmp_path / "fits", 512, "cuda") < 50


def test_fit_device_bytes_covers_group_buffers(gpu):
    """engine.fit_device_bytes (the memory-wave planner's per-fit size) is at
    least what a real one-fit group allocates, buffer by buffer."""
    from nerf_attention.synthetic import kv_slice
    keys, _ = kv_slice(0, 0, seq_len=512)
    for cfg, prec in ((SIRENConfig(256, 2, 30.0, "medium"), "bf16x3"),
                      (SIRENConfig(64, 1, 30.0, "tiny"), "fp32")):
        torch.manual_seed(0)
        spec = engine.FitSpec(target=keys, config=cfg, init=SIREN(cfg, 128).flat_parameters())
        job = engine.FitJob([spec], 20, log_every=5, devices=[0], precision=prec)
        g = job.groups[0]
        held = sum(t.numel() * t.element_size() for t in vars(g).values()
                   if isinstance(t, torch.Tensor) and t.device.type == "cuda")
        need = engine.fit_device_bytes(spec, 20, 5, prec)
        assert need >= held, (cfg.name, need, held)
        assert need <= 1.3 * held + (1 << 20), (cfg.name, need, held)


def test_streaming_job_equals_fitjob(gpu):
    """fit_kv_cache's streaming path (engine.StreamingJob: each group launched
    the moment its last init exists, results collected as groups finish)
    trains exactly what a FitJob over the same plan trains: bitwise the same
    parameters and losses; on_ready reports every fit once, and each fit's
    train_time_seconds is its group's measured device interval."""
    from nerf_attention import fit as fitmod
    from nerf_attention.synthetic import kv_cache
    from nerf_attention.types import CONFIGS_FULL
    cache = kv_cache([0, 8], 512, 32, 8, 128, heads=range(2))
    plan, _ = fitmod.sweep_plan([0, 8], 2, CONFIGS_FULL, lambda l: cache[l])
    torch.manual_seed(0)
    seen = []
    streamed = fitmod.train_plan_streaming(plan, 40, 0, log_every=20,
                                           on_ready=lambda k, r, p: seen.append(k))
    assert sorted(seen) == list(range(len(plan)))
    torch.manual_seed(0)
    batched = fitmod.train_plan(plan, 40, [0], log_every=20)
    assert len(streamed) == len(batched) == len(plan) == 56
    for (a, pa), (b, pb) in zip(streamed, batched):
        assert torch.equal(a.model.network[-1].weight.cpu(), b.model.network[-1].weight.cpu())
        assert a.losses == b.losses and pa == pb
        assert a.final_cosine_mean == b.final_cosine_mean
    share = [r.train_time_seconds for r, _ in streamed]
    assert all(t > 0 for t in share)


@pytest.mark.gpu
def test_fitjob_threaded_launch_is_bitwise_equal(gpu, monkeypatch):
    """FitJob.launch with one launcher thread per group (NERFHIP_LAUNCH_THREADS)
    trains exactly what the single interleaving thread trains, launch after
    launch (reset + relaunch, as bench.py's steps do)."""
    from nerf_attention import engine
    from nerf_attention.siren import init_flat
    from nerf_attention.synthetic import kv_cache
    from nerf_attention.types import CONFIGS_FULL
    cache = kv_cache([0], 512, 32, 8, 128, heads=range(2))
    torch.manual_seed(0)
    specs = [engine.FitSpec(target=cache[0][kv][h], config=c, init=init_flat(c, 128))
             for h in range(2) for kv in ("keys", "values") for c in CONFIGS_FULL]
    outs = {}
    for threads in (False, True):
        monkeypatch.setattr(engine, "LAUNCH_THREADS", threads)
        job = engine.FitJob(specs, 30, devices=[0], precision="bf16x3")
        assert len(job.groups) > 1
        runs = []
        for _ in range(2):
            job.launch()
            job.wait()
            runs.append([o.params.cpu() for o in job.outputs()])
        assert all(torch.equal(a, b) for a, b in zip(*runs))
        outs[threads] = runs[0]
        del job
    assert all(torch.equal(a, b) for a, b in zip(outs[False], outs[True]))


def test_xcd_order_bitwise(gpu, sweep, monkeypatch):
    """The XCD-balanced, depth-sorted chunk plan (engine.plan_groups, default
    NERFHIP_CHUNKS=depth) trains every sweep fit bitwise as the round-4 plan
    (reference-order chunks, NERFHIP_CHUNKS=spec) does: parameters, every
    epoch's loss and the final row cosines.  The plans really differ (the
    W = 256 chunks change composition and every chunk's fit order), and the
    outputs come back in spec (= reference record) order either way."""
    _plan, specs = sweep
    outs, plans = {}, {}
    for policy in ("spec", "depth", "mixed"):
        monkeypatch.setenv("NERFHIP_CHUNKS", policy)
        job = engine.FitJob(specs, 60, devices=[0], precision="bf16x3")
        plans[policy] = [list(m) for _d, m in job.plan]
        job.launch()
        job.wait()
        outs[policy] = [(o.params.cpu(), o.losses, o.row_cos) for o in job.outputs()]
        del job
    assert plans["spec"] != plans["depth"] != plans["mixed"]
    for policy in ("depth", "mixed"):
        for k, (a, b) in enumerate(zip(outs["spec"], outs[policy])):
            assert torch.equal(a[0], b[0]), (policy, k)
            assert a[1] == b[1], (policy, k)
            assert np.array_equal(a[2], b[2]), (policy, k)
