"""Host-side logic of the product package (no GPU): model init and its RNG
order, the synthetic KV generator, the optimiser schedule, sweep selection and
ordering, record / checkpoint schema, LPT sharding."""

import hashlib
import json

import numpy as np
import pytest
import torch

from nerf_attention import CONFIGS_FULL, SIREN, SIRENConfig, types
from nerf_attention import engine, schedule
from nerf_attention.fit import (RECORD_KEYS, _result_to_record, _save_model, select_fits,
                                sweep_plan)
from nerf_attention.siren import _finish
from nerf_attention.synthetic import kv_layer, kv_slice


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_init_matches_reference(golden_dir):
    g = json.loads((golden_dir / "init.json").read_text())
    arrays = np.load(golden_dir / "init_tiny_small.npz")
    for name, rec in g.items():
        cfg = SIRENConfig(rec["hidden_features"], rec["hidden_layers"], rec["omega_0"], name)
        torch.manual_seed(0)
        m = SIREN(cfg, 128)
        flat = m.flat_parameters().numpy()
        assert list(m.state_dict().keys()) == rec["keys"]
        assert flat.size == rec["num_parameters"] == cfg.num_parameters(128)
        assert m.count_parameters() == rec["num_parameters"]
        assert sha(flat) == rec["sha256"], name
        if name in arrays:
            assert np.array_equal(flat, arrays[name])


def test_sweep_init_order(golden_dir):
    """Pre-generating the 280 inits in loop order == the reference's sequential run."""
    ref = json.loads((golden_dir / "sweep_init_order.json").read_text())
    cfg = {c.name: c for c in CONFIGS_FULL}
    torch.manual_seed(0)
    for name, h in ref:
        m = SIREN(cfg[name.split("_")[-1]], 128)
        assert sha(m.flat_parameters().numpy()) == h, name


def test_synthetic_quickstart_bit_exact(golden_dir):
    g = json.loads((golden_dir / "synthetic.json").read_text())["q512"]
    for l in range(4):
        t = kv_layer(l, 512, 4, 4, 128)
        assert sha(t["keys"].numpy()) == g[f"layer_{l:02d}"]["keys"]
        assert sha(t["values"].numpy()) == g[f"layer_{l:02d}"]["values"]


@pytest.mark.parametrize("layer,head", [(0, 0), (8, 3), (31, 7)])
def test_synthetic_llama_shape_bit_exact(golden_dir, layer, head):
    g = json.loads((golden_dir / "synthetic.json").read_text())
    if "s2048" not in g:
        pytest.skip("s2048 hashes not generated yet")
    k, v = kv_slice(layer, head, seq_len=2048)
    assert sha(k.numpy()) == g["s2048"][f"layer_{layer:02d}"]["keys"][head]
    assert sha(v.numpy()) == g["s2048"][f"layer_{layer:02d}"]["values"][head]


def test_extract_writes_reference_layout(tmp_path):
    from nerf_attention import extract_kv_cache_synthetic
    meta = extract_kv_cache_synthetic(seq_len=64, num_layers=2, num_kv_heads=2, head_dim=64,
                                      output_dir=tmp_path)
    d = json.loads((tmp_path / "metadata.json").read_text())
    assert d == {"model_name": "synthetic", "num_layers": 2, "num_kv_heads": 2, "seq_len": 64,
                 "head_dim": 64, "actual_tokens": 64, "dtype": "float32"}
    assert types.KVMetadata.from_dict(d) == meta
    t = torch.load(tmp_path / "layer_01.pt", weights_only=True)
    assert t["keys"].shape == (2, 64, 64) and t["values"].dtype == torch.float32


def test_adam_schedule():
    tab = schedule.adam_table(2000, 1e-4)
    lrs = schedule.lr_sequence(2000, 1e-4)
    assert lrs[0] == 1e-4 and abs(lrs[-1] - 1e-6) < 1e-8
    # closed form of the cosine schedule, to rounding
    e = np.arange(2000)
    closed = 1e-6 + 0.5 * (1e-4 - 1e-6) * (1 + np.cos(np.pi * e / 2000))
    np.testing.assert_allclose(lrs, closed, rtol=1e-9)
    t = e + 1.0
    np.testing.assert_array_equal(tab[:, 0], np.float32(np.array(lrs) / (1 - 0.9 ** t)))
    np.testing.assert_array_equal(tab[:, 1], np.float32((1 - 0.999 ** t) ** 0.5))


def test_selection_and_order(golden_dir):
    """Quick-mode plan names/order equal the reference run's records."""
    ref = json.loads((golden_dir / "schema_quick" / "fit_results.json").read_text())
    meta = types.KVMetadata("synthetic", 4, 4, 512, 128, 512)
    layers, heads, cfgs = select_fits(meta, quick=True)
    plan, skipped = sweep_plan(layers, heads, cfgs,
                               lambda l: {"keys": torch.zeros(1, 8, 4),
                                          "values": torch.zeros(1, 8, 4)})
    assert [p[0] for p in plan] == [r["name"] for r in ref] and not skipped
    full = types.KVMetadata("x", 32, 8, 2048, 128, 2048)
    layers, heads, cfgs = select_fits(full, quick=False)
    assert layers == [0, 8, 16, 24, 31] and heads == 4 and len(cfgs) == 7


def test_missing_layer_skipped():
    meta = types.KVMetadata("x", 4, 1, 8, 4, 8)
    layers, heads, cfgs = select_fits(meta, quick=True)
    plan, skipped = sweep_plan(layers, heads, cfgs,
                               lambda l: None if l == 2 else {"keys": torch.zeros(1, 8, 4),
                                                              "values": torch.zeros(1, 8, 4)})
    assert skipped == [2] and all(p[1] != 2 for p in plan)


def test_fit_kv_cache_empty_selection(tmp_path, monkeypatch, capsys):
    """Every selected layer file missing: the plan is empty, each layer prints
    'Skipping layer' and fit_results.json is an empty list (fit.py:56-58,88-89)
    — the streaming path is not taken for an empty plan.  The device is faked
    (no GPU here); nothing reaches the engine."""
    import types as pytypes
    from nerf_attention import fit as fitmod
    meta = types.KVMetadata("x", 4, 1, 8, 4, 8)
    (tmp_path / "kv").mkdir()
    (tmp_path / "kv" / "metadata.json").write_text(json.dumps(meta.to_dict()))
    monkeypatch.setattr(engine, "resolve_device", lambda d: pytypes.SimpleNamespace(index=0))
    monkeypatch.setattr(engine, "memory_budget", lambda dev: 1 << 40)
    assert not fitmod._stream_ok([], 10, [0], 100, None)
    out = fitmod.fit_kv_cache(tmp_path / "kv", tmp_path / "out", epochs=10, quick=True)
    assert out == []
    assert json.loads((tmp_path / "out" / "fit_results.json").read_text()) == []
    assert capsys.readouterr().out.count("Skipping layer") == 3


def test_streaming_job_seconds_without_groups():
    job = object.__new__(engine.StreamingJob)
    job.groups, job._threads = [], {}
    assert job.job_seconds() == 0.0


def _fake_output(cfg, N=16, D=8):
    torch.manual_seed(1)
    m = SIREN(cfg, D)
    out = engine.FitOutput(params=m.flat_parameters(), target_mean=torch.zeros(1, D),
                           target_std=torch.ones(1, D), losses=[1.0, 0.5],
                           row_cos=np.linspace(0.5, 1, N, dtype=np.float32),
                           row_mse=np.ones(N, np.float32), final_mse=0.25)
    return m, out


def test_record_and_checkpoint_schema(golden_dir, tmp_path):
    ref = json.loads((golden_dir / "schema_quick" / "fit_results.json").read_text())
    layout = json.loads((golden_dir / "schema_quick" / "checkpoint_layout.json").read_text())
    assert list(ref[0].keys()) == list(RECORD_KEYS)
    cfg = SIRENConfig(256, 2, 30.0, "medium")
    m, out = _fake_output(cfg, N=16, D=128)
    res = _finish(m, cfg, out, 16, 128)
    rec = _result_to_record("L0_H0_key_medium", 0, 0, "key", res)
    assert list(rec.keys()) == list(ref[0].keys())
    assert rec["num_parameters"] == 164992 and rec["raw_size_bytes"] == 16 * 128 * 2
    assert rec["final_cosine_std"] == pytest.approx(float(np.std(out.row_cos, ddof=1)), rel=1e-5)
    _save_model(tmp_path, "L0_H0_key_medium", res, rec)
    ck = torch.load(tmp_path / "L0_H0_key_medium_model.pt", weights_only=True)
    assert list(ck.keys()) == layout["top_keys"]
    assert list(ck["model_state"].keys()) == layout["model_state_keys"]
    assert {k: list(v.shape) for k, v in ck["model_state"].items()} == \
        layout["model_state_shapes"]
    assert ck["config"] == layout["config"]
    assert list(ck["metrics"].keys()) == layout["metrics_keys"]


def test_flat_parameter_roundtrip():
    cfg = SIRENConfig(64, 2, 30.0, "x")
    torch.manual_seed(3)
    a = SIREN(cfg, 64)
    b = SIREN(cfg, 64)
    b.load_flat_parameters(a.flat_parameters())
    x = torch.rand(10, 1)
    assert torch.equal(a(x), b(x))


def test_lpt_partition_balances():
    cfg = {c.name: c for c in CONFIGS_FULL}
    costs = [engine.fit_flops(2048, 128, c, 2000) for c in CONFIGS_FULL] * 40
    for n in (1, 2, 4, 8):
        own = engine.lpt_partition(costs, n)
        loads = [sum(c for c, o in zip(costs, own) if o == r) for r in range(n)]
        assert sorted(set(own)) == list(range(n))
        assert max(loads) / (sum(costs) / n) < 1.02
    assert engine.fit_flops(2048, 128, cfg["medium"], 2000) == pytest.approx(4.03e12, rel=1e-2)


def test_plan_groups_by_width():
    cfgs = [SIRENConfig(256, 2, 30.0, "m"), SIRENConfig(64, 1, 30.0, "t"),
            SIRENConfig(256, 3, 30.0, "d"), SIRENConfig(256, 2, 60.0, "h")]
    specs = [engine.FitSpec(torch.zeros(128, 128), c, torch.zeros(1)) for c in cfgs]
    groups = engine.plan_groups(specs, 0)
    assert sorted(sorted(m) for _, m in groups) == [[0, 2, 3], [1]]
    assert sorted(groups[0][1]) == [0, 2, 3]          # heaviest first
    assert groups[0][1][0] == 2                       # deepest first (NERFHIP_CHUNKS=depth)


def test_non_hip_device_raises():
    """The engine path has no CPU fallback: only an explicit 'cpu' takes the
    host path (test_host_path.py); any other non-HIP device raises."""
    from nerf_attention import fit_siren
    from nerf_attention._native import NerfhipError
    with pytest.raises(NerfhipError, match="no CPU"):
        fit_siren(torch.zeros(64, 64), SIRENConfig(64, 1, 30.0, "t"), epochs=1, device="meta",
                  verbose=False)


def test_custom_ops_registered_with_fakes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    assert hasattr(torch.ops.nerfhip, "siren_fit") and hasattr(torch.ops.nerfhip, "siren_forward")
    P = SIRENConfig(64, 1, 30.0, "t").num_parameters(64)
    with FakeTensorMode():
        t = torch.empty(2, 96, 64)
        init = torch.empty(2, P)
        params, losses, rc, rm = torch.ops.nerfhip.siren_fit(t, init, 64, [1, 1], [30.0, 30.0],
                                                              7, 1e-4)
        assert params.shape == (2, P) and losses.shape == (2, 7) and rc.shape == (2, 96)
        y = torch.ops.nerfhip.siren_forward(init[0], torch.empty(96), 64, 1, 30.0, 64)
        assert y.shape == (96, 64)


def test_plan_groups_chunks_large_groups():
    """Groups above GROUP_MAX split into multiple-of-8 chunks (one stream each);
    the sweep's 160-fit W=256 group becomes 4 x 40; small groups stay whole."""
    from nerf_attention.workloads import sweep_280
    _, specs = sweep_280(64, seed=0)
    groups = engine.plan_groups(specs, 0)
    sizes = sorted(len(m) for _, m in groups)
    assert sizes == [40] * 7
    assert sorted(i for _, m in groups for i in m) == list(range(280))
    assert [len(c) for c in engine._chunks(list(range(100)), 40)] == [32, 32, 36]
    assert [len(c) for c in engine._chunks(list(range(9)), 40)] == [9]
    assert [len(c) for c in engine._chunks(list(range(160)), 0)] == [160]


def _xcd_loads(members, costs):
    return [sum(costs[i] for i in members[x::engine.XCDS]) for x in range(engine.XCDS)]


@pytest.mark.parametrize("policy", ["depth", "mixed", "spec"])
def test_sweep_chunks_xcd_balance(policy, monkeypatch):
    """map_block puts fit k of a group on XCD k mod 8.  Reference order put
    all 10 deep fits of every W = 256 chunk on XCDs 1 and 5 (max/mean XCD
    work 1.27); the default plan cuts depth-uniform chunks
    (one of 40 deep fits, three of 40 L = 2 fits: every XCD equal), 'mixed'
    deals 10 deep fits to every chunk and spreads them over the XCDs."""
    from nerf_attention.workloads import sweep_280
    monkeypatch.setenv("NERFHIP_CHUNKS", policy)
    _, specs = sweep_280(64, seed=0)
    costs = [engine.fit_flops(2048, 128, s.config, 1) for s in specs]
    groups = engine.plan_groups(specs, 0)
    assert sorted(i for _, m in groups for i in m) == list(range(280))
    w256 = [m for _, m in groups if specs[m[0]].config.hidden_features == 256]
    assert [len(m) for m in w256] == [40] * 4
    depths = sorted(tuple(sorted({specs[i].config.hidden_layers for i in m})) for m in w256)
    imb = max(max(_xcd_loads(m, costs)) / (sum(costs[i] for i in m) / 8) for m in w256)
    if policy == "spec":
        assert imb == pytest.approx(1.2727, abs=1e-3)
    elif policy == "depth":
        assert depths == [(2,), (2,), (2,), (3,)]
        assert imb == pytest.approx(1.0)
    else:
        assert all(sum(specs[i].config.hidden_layers == 3 for i in m) == 10 for m in w256)
        assert imb < 1.06


def test_xcd_order_balances_and_permutes():
    costs = [1.0, 1.4, 1.0, 1.0] * 10 + [2.0] * 3
    m = list(range(43))
    out = engine.xcd_order(m, costs)
    assert sorted(out) == m
    loads = _xcd_loads(out, costs)
    assert max(loads) - min(loads) <= 2.0
    assert engine.xcd_order([3, 1, 2], costs) == [3, 1, 2]        # < 8 fits: linear map


def test_param_tiles_matches_kernel_grid():
    """engine.param_tiles restates nerfhip.hip ParamsCfg::tiles (the fused
    parameter-step grid per fit), which decides split-K for small groups."""
    from nerf_attention import engine
    assert engine.param_tiles(256, 128, 2) == 14      # medium: 2·4 hidden + 2 final + 4 first-layer
    assert engine.param_tiles(512, 128, 2) == 44      # large
    assert engine.param_tiles(512, 128, 3) == 60      # wide (512, 3)
    assert engine.param_tiles(128, 128, 1) == 4       # small
    assert engine.param_tiles(64, 128, 1) == 4        # tiny
    assert 5 * engine.param_tiles(512, 128, 2) >= engine.SPLIT_MIN_TILES    # 8-rank large group: fused
    assert engine.param_tiles(256, 128, 2) < engine.SPLIT_MIN_TILES         # config 2: split-K


# --- native init replay (siren.init_flat / nerfhip_rng_uniform_segments) ---

@pytest.mark.parametrize("seed", [0, 1, 12345])
@pytest.mark.parametrize("w,layers,d", [(64, 1, 128), (128, 2, 64), (256, 3, 128), (512, 2, 64)])
def test_init_flat_equals_siren_constructor(seed, w, layers, d):
    """Same bits as SIREN(cfg, d).flat_parameters(), and the generator left
    where the constructor leaves it (a torch draw before and after agrees)."""
    from nerf_attention.siren import init_flat
    cfg = SIRENConfig(w, layers, 30.0, "t")
    torch.manual_seed(seed)
    torch.rand(seed % 97)
    a, a_next = init_flat(cfg, d), torch.rand(7)
    torch.manual_seed(seed)
    torch.rand(seed % 97)
    b, b_next = SIREN(cfg, d).flat_parameters(), torch.rand(7)
    assert torch.equal(a, b)
    assert torch.equal(a_next, b_next)


def test_init_flat_sweep_order(golden_dir):
    """The 280 sweep inits drawn natively == the reference's sequential run."""
    from nerf_attention.siren import init_flat
    ref = json.loads((golden_dir / "sweep_init_order.json").read_text())
    cfg = {c.name: c for c in CONFIGS_FULL}
    torch.manual_seed(0)
    for name, h in ref:
        assert sha(init_flat(cfg[name.split("_")[-1]], 128).numpy()) == h, name


def test_uninitialised_draws_nothing():
    from nerf_attention.siren import uninitialised
    cfg = {c.name: c for c in CONFIGS_FULL}["medium"]
    torch.manual_seed(3)
    before = torch.get_rng_state()
    m = uninitialised(cfg, 128, "cpu")
    assert torch.equal(before, torch.get_rng_state())
    assert list(m.state_dict()) == list(SIREN(cfg, 128).state_dict())
    assert m.count_parameters() == cfg.num_parameters(128)


class _FakeEvent:
    def __init__(self, clock):
        self.clock, self.t = clock, None

    def record(self, _stream=None):
        self.t = self.clock()

    def query(self):
        return self.t is not None

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def _fake_streaming(monkeypatch, rc=0):
    """StreamingJob with the device side replaced by fakes (CPU only): the
    launcher threads, the arrival-triggered launches, finished() and the error
    path run for real; nerfhip_siren_fit returns `rc`."""
    import itertools
    import threading
    import types
    tick = itertools.count()
    lock = threading.Lock()

    def clock():
        with lock:
            return float(next(tick))

    calls = []

    class FakeGroup:
        def __init__(self, members, specs, *a, **k):
            self.members = members
            self.stream = types.SimpleNamespace(cuda_stream=None)
            self.desc = engine._native.NerfhipGroup()
            self.ev_start, self.ev_end = _FakeEvent(clock), _FakeEvent(clock)

        def outputs(self, specs, gs):
            return [gs] * len(self.members)

    class FakeLib:
        def nerfhip_siren_fit(self, desc, n, st):
            calls.append(threading.current_thread().name)
            return rc

        def nerfhip_status_string(self, code):
            return b"launch failed"

    lib = FakeLib()
    monkeypatch.setattr(engine, "resolve_device", lambda d: types.SimpleNamespace(index=0))
    monkeypatch.setattr(engine, "plan_groups", lambda protos, dev: [(0, [0, 2]), (0, [1])])
    monkeypatch.setattr(engine, "_Group", FakeGroup)
    monkeypatch.setattr(engine._native, "load", lambda path=None: lib)
    cfg = SIRENConfig(64, 1, 30.0, "tiny")
    protos = [engine.FitSpec(target=torch.zeros(4, 64), config=cfg, init=None) for _ in range(3)]
    job = engine.StreamingJob(protos, 2, device=0, precision="bf16x3")
    return job, protos, calls


def test_streaming_job_launch_threads(monkeypatch):
    """Each group is launched from its own thread as soon as its last fit
    arrives (group 1 = fit 1 launches before group 0 = fits 0, 2 is complete);
    finished() yields every group once, after its thread and end event."""
    job, protos, calls = _fake_streaming(monkeypatch)
    job.add(0, protos[0])
    assert job.launch_order == []
    job.add(1, protos[1])
    assert job.launch_order == [1]
    with pytest.raises(ValueError):
        list(job.finished())                  # not every fit added yet
    job.add(2, protos[2])
    assert job.launch_order == [1, 0]
    assert sorted(job.finished()) == [0, 1]
    assert sorted(calls) == ["nerfhip-group-0", "nerfhip-group-1"]
    assert [k for k, _ in job.outputs(0)] == [0, 2]
    assert job.job_seconds() > 0
    with pytest.raises(ValueError):
        job.add(2, protos[2])                 # added twice


def test_streaming_job_launch_error_surfaces(monkeypatch):
    """A failing launch inside a launcher thread is raised by finished()."""
    job, protos, _ = _fake_streaming(monkeypatch, rc=-6)
    for i, p in enumerate(protos):
        job.add(i, p)
    with pytest.raises(engine._native.NerfhipError):
        list(job.finished())


def test_synthetic_spawn_pool_bitwise_and_leaves_nothing(monkeypatch):
    """The generator's spawn-process path (taken once the process holds HIP
    state) gives the same bits as one process, and leaves no child process
    (no multiprocessing resource tracker: BENCH_r04 procs_at_end) and no
    /dev/shm file behind."""
    import glob
    import multiprocessing as mp
    from nerf_attention import synthetic
    monkeypatch.setattr(synthetic, "_hip_untouched", lambda: False)
    monkeypatch.setattr(synthetic, "POOL_MIN_ROWS", 0)
    monkeypatch.setattr(synthetic, "_threads", lambda: 2)
    from multiprocessing import resource_tracker
    pairs = [(0, 0), (3, 1), (5, 2)]
    before = set(glob.glob("/dev/shm/nerf_synth_*"))
    # (another test of this session may already have started the process's
    # tracker: this call must not start one, and must not restart it)
    tracker = getattr(resource_tracker._resource_tracker, "_pid", None)
    got = synthetic.kv_slices(pairs, seq_len=256, num_layers=8, num_kv_heads=4)
    for (l, h), (k, v) in zip(pairs, got):
        k0, v0 = kv_slice(l, h, seq_len=256, num_layers=8, num_kv_heads=4)
        assert torch.equal(k, k0) and torch.equal(v, v0)
    assert mp.active_children() == []
    assert set(glob.glob("/dev/shm/nerf_synth_*")) == before
    assert getattr(resource_tracker._resource_tracker, "_pid", None) == tracker


def test_init_replay_self_check(monkeypatch):
    """init_flat's one-time self-check: the replay matches torch's uniform_
    here (so init_flat takes it), leaves the caller's generator untouched,
    and a failing check (a host whose torch kernel rounds differently) sends
    init_flat to the module constructor — same bits either way."""
    from nerf_attention import siren
    monkeypatch.setattr(siren, "_REPLAY_OK", None)
    torch.manual_seed(7)
    before = torch.get_rng_state()
    assert siren.replay_matches_torch()
    assert torch.equal(before, torch.get_rng_state())
    cfg = SIRENConfig(128, 2, 30.0, "t")
    torch.manual_seed(3)
    a = siren.init_flat(cfg, 64)
    monkeypatch.setattr(siren, "_REPLAY_OK", False)
    monkeypatch.setattr(siren, "_replay", lambda segs: (_ for _ in ()).throw(AssertionError))
    torch.manual_seed(3)
    b = siren.init_flat(cfg, 64)
    assert torch.equal(a, b)


def test_split_choice_depends_on_the_group_shape_only(monkeypatch):
    """The split-K workspace goes to every group under 8 fits whose fused
    parameter grid is under 128 workgroups, whatever else trains on the device
    (round 5's engine.split_allowed, which withheld it from concurrent groups,
    is gone: DESIGN.md §13).  The 8-rank share's 5-fit W = 128 / 64 groups take
    it, its 5-fit W = 512 group (220 tiles) and 20-fit W = 256 group do not."""
    monkeypatch.delenv("NERFHIP_SPLIT_MAX_FITS", raising=False)
    assert not hasattr(engine, "split_allowed")
    assert engine.wants_split(5, 128, 128, 1, 16) and engine.wants_split(5, 64, 128, 1, 16)
    assert engine.wants_split(1, 256, 128, 2, 16) and engine.wants_split(1, 512, 128, 3, 16)
    assert not engine.wants_split(5, 512, 128, 2, 16)      # 5 x 44 tiles >= 128
    assert not engine.wants_split(20, 256, 128, 3, 16) and not engine.wants_split(8, 64, 128, 1, 16)
    assert not engine.wants_split(1, 256, 128, 2, 1)       # no row slices to split into
    monkeypatch.setenv("NERFHIP_SPLIT_MAX_FITS", "0")
    assert not engine.wants_split(1, 256, 128, 2, 16)


def test_ks_lds_hb_checker_on_synthetic_traces():
    """tools/r5/ks_lds_hb.py's happens-before rule on hand-made traces: a
    cross-wave write→read or read→overwrite of one LDS address inside one
    barrier interval is a race; the same pair across a barrier, or within one
    wave, is not; and ignoring the barriers exposes the separated pairs."""
    import importlib.util
    import numpy as np
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    spec = importlib.util.spec_from_file_location("ks_lds_hb", root / "tools/r5/ks_lds_hb.py")
    hb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(hb)

    def trace(events):   # events: {wave: [(bc, rw, addr), ...]} -> [4][MAXEV][64]
        tr = np.full((4, hb.MAXEV, 64), 0xFFFFFFFF, dtype=np.uint32)
        for w, evs in events.items():
            for n, (bc, rw, addr) in enumerate(evs):
                tr[w, n, :] = (bc << 18) | (rw << 17) | addr
        return tr

    clean = trace({0: [(0, 1, 64), (1, 0, 128)], 1: [(1, 0, 64), (0, 1, 128)],
                   2: [(0, 1, 256), (0, 0, 256)], 3: [(2, 1, 64)]})
    r = hb.check(clean)
    assert r["races"] == 0 and r["events_per_wave"] == [2, 2, 2, 1]
    assert hb.check(clean, bc_override=True)["races"] > 0
    raw = trace({0: [(3, 1, 512)], 1: [(3, 0, 512)]})          # write -> read, same interval
    war = trace({0: [(5, 0, 768)], 2: [(5, 1, 768)]})          # read -> overwrite
    assert hb.check(raw)["races"] == 1 and hb.check(war)["races"] == 1


def test_fit_report_streams_blocks_in_reference_order(capsys, tmp_path):
    """fit_kv_cache's progress (reference fit.py:54-86):
    each fit's block prints the moment it and every fit before it in the
    reference's order have finished — layer by layer, a missing layer's
    'Skipping' line in its place — whatever order the groups finish in, and the
    records come out in that same order with the measured train time."""
    from types import SimpleNamespace
    from nerf_attention.fit import RECORD_KEYS, _Report
    from nerf_attention.types import SIRENConfig

    tiny, small = SIRENConfig(64, 1, 30.0, "tiny"), SIRENConfig(128, 1, 30.0, "small")
    plan = [(f"L{l}_H0_key_{c.name}", l, 0, "key", c, None) for l in (0, 2) for c in (tiny, small)]

    def res(k):
        return SimpleNamespace(config=plan[k][4], final_mse=0.1, final_cosine_mean=0.9 + k / 100,
                               final_cosine_min=0.8, final_cosine_std=0.01, compression_ratio=4.0,
                               raw_size_bytes=1, siren_size_bytes=1, train_time_seconds=1.5 + k,
                               num_parameters=10, seq_len=16, d_head=8)

    rep = _Report(plan, layers=[0, 1, 2], skipped={1}, total=len(plan), epochs=10,
                  output_dir=tmp_path)
    assert capsys.readouterr().out == ""              # nothing before fit 0
    rep.fit_done(2, res(2), [])                       # a later group finishes first
    assert capsys.readouterr().out == ""              # still waiting for fits 0, 1
    rep.fit_done(0, res(0), [(5, 0.5, 0.25, 0.75)])
    out = capsys.readouterr().out
    assert "[1/4] L0_H0_key_tiny" in out and "Epoch 5/10" in out and "[2/4]" not in out
    rep.fit_done(1, res(1), [])
    out = capsys.readouterr().out                     # fit 1, the skipped layer, then fit 2
    assert out.index("[2/4] L0_H0_key_small") < out.index("Skipping layer 1") < \
        out.index("[3/4] L2_H0_key_tiny")
    rep.fit_done(3, res(3), [])
    records = rep.finish()
    assert [r["name"] for r in records] == [p[0] for p in plan]
    assert [r["train_time_seconds"] for r in records] == [1.5, 2.5, 3.5, 4.5]
    assert list(records[0]) == list(RECORD_KEYS)
    assert "Time: 4.5s" in capsys.readouterr().out
