"""BASELINE config 1 (`quickstart --cpu`) and the host-side pieces around the
engine, on the CPU:

* the explicit host path `fit_siren(..., device='cpu')` against the
  reference's own 2000-epoch fits (tests/golden/fits_q512.json) and its
  step-level parameters (steps_tiny.npz);
* the quickstart pipeline through this package's public names (the ones
  /root/reference/quickstart.py:8-15 imports) end to end on the CPU;
* the CPU analysis path against the reference's per-slice analysis;
* memory-bounded waves and the no-fallback rule for HIP requests.
"""

import json

import numpy as np
import pytest
import torch

from nerf_attention import SIRENConfig, engine, fit_siren
from nerf_attention.synthetic import kv_slice

COS_TOL = 1e-3


def test_host_fit_matches_reference_q512(golden_dir):
    meta = json.loads((golden_dir / "fits_q512.json").read_text())
    keys, vals = kv_slice(0, 0, seq_len=512, num_layers=4, num_kv_heads=4)
    for name, t, cfg in (("key_tiny", keys, SIRENConfig(64, 1, 30.0, "tiny")),
                         ("value_tiny", vals, SIRENConfig(64, 1, 30.0, "tiny"))):
        torch.manual_seed(0)
        r = fit_siren(t, cfg, epochs=2000, device="cpu", log_every=400, verbose=False)
        ref = meta[name]
        assert abs(r.final_cosine_mean - ref["final_cosine_mean"]) <= COS_TOL
        assert r.num_parameters == ref["num_parameters"]
        assert r.compression_ratio == pytest.approx(ref["compression_ratio"])
        assert r.model.network[0].linear.weight.device.type == "cpu"


def test_host_steps_match_reference(golden_dir):
    z = np.load(golden_dir / "steps_tiny.npz")
    cfg = SIRENConfig(64, 1, 30.0, "tiny")
    t = torch.from_numpy(z["target"])
    for k in (1, 3, 10):
        torch.manual_seed(0)
        r = fit_siren(t, cfg, epochs=k, device="cpu", verbose=False)
        p = torch.cat([v.reshape(-1) for v in r.model.state_dict().values()]).numpy()
        np.testing.assert_allclose(p, z[f"params_{k}"], atol=2.5e-4 * k)
        assert np.mean(np.abs(p - z[f"params_{k}"]) <= 1e-6) >= 0.999
        np.testing.assert_allclose(r.losses, z[f"losses_{k}"], rtol=1e-5)


def test_host_verbose_lines(capsys):
    keys, _ = kv_slice(0, 0, seq_len=128, num_layers=4, num_kv_heads=4)
    fit_siren(keys, SIRENConfig(64, 1, 30.0, "tiny"), epochs=20, device="cpu", log_every=10)
    lines = capsys.readouterr().out.strip().splitlines()
    assert [l.split("|")[0].strip() for l in lines] == ["Epoch 10/20", "Epoch 20/20"]
    assert all(len(l.split("|")) == 4 for l in lines)


def test_quickstart_pipeline_cpu(tmp_path, golden_dir, capsys):
    """quickstart.py:18-68's four steps through this package's names, on the
    CPU (epochs cut to 30 to keep the CPU suite short)."""
    from nerf_attention import (analyze_kv_cache, extract_kv_cache_synthetic, fit_kv_cache,
                                generate_summary_figure, load_results, plot_pareto_frontier)
    kv, an, fits, figs = (tmp_path / d for d in ("kv", "analysis", "fits", "figures"))
    extract_kv_cache_synthetic(seq_len=512, num_layers=4, num_kv_heads=4, head_dim=128,
                               output_dir=kv)
    res = analyze_kv_cache(kv_dir=kv, output_dir=an, device="cpu")
    assert (an / "analysis_results.json").exists() and len(res.layer_summaries) == 4
    torch.manual_seed(0)
    recs = fit_kv_cache(kv_dir=kv, output_dir=fits, epochs=30, device="cpu", quick=True)
    ref = json.loads((golden_dir / "schema_quick" / "fit_results.json").read_text())
    assert [r["name"] for r in recs] == [r["name"] for r in ref]
    assert [list(r) for r in recs] == [list(r) for r in ref]
    assert len(list(fits.glob("*_model.pt"))) == 6
    figs.mkdir()
    results = load_results(fits)
    assert results == json.loads(json.dumps(recs))
    plot_pareto_frontier(results, figs)
    generate_summary_figure(results, figs)
    assert list(figs.iterdir()) == []
    out = capsys.readouterr().out
    assert "[12/12] L3_H0_value_medium" in out and "RESULTS SUMMARY" in out


def test_host_analysis_matches_reference(golden_dir):
    """analyze_slices on CPU tensors (numpy + torch.linalg.svd) against the
    reference's own per-slice analysis of the quickstart cache."""
    from nerf_attention.analyze import analyze_slices, select_layers
    from nerf_attention.synthetic import kv_layer
    g = json.loads((golden_dir / "analysis_q512.json").read_text())
    sh = g["shape"]
    L, H = sh["num_layers"], sh["num_kv_heads"]
    sl, names = [], []
    for layer in select_layers(L):
        t = kv_layer(layer, sh["seq_len"], L, H, sh["head_dim"], heads=range(min(H, 4)))
        for h in range(min(H, 4)):
            sl += [t["keys"][h], t["values"][h]]
            names += [f"L{layer}_H{h}_K", f"L{layer}_H{h}_V"]
    out = analyze_slices(torch.stack(sl), names)
    for a in out:
        b = g["slices"][a["name"]]
        np.testing.assert_allclose(a["mean_autocorrelation"], b["mean_autocorrelation"],
                                   atol=1e-6)
        for k in b["spectral_energy"]:
            assert abs(a["spectral_energy"][k] - b["spectral_energy"][k]) <= 1e-6
        assert a["rank"]["effective_rank_99"] == b["rank"]["effective_rank_99"]
        assert a["rank"]["full_rank"] == b["rank"]["full_rank"]


def test_effective_rank_counts_min_n_d():
    """A slice shorter than d_head has min(N, D) singular values (the
    reference's torch.linalg.svd); the host path keeps that count."""
    from nerf_attention.analyze import analyze_slices
    x = torch.randn(1, 40, 64)
    r = analyze_slices(x, ["short"])[0]["rank"]
    assert r["full_rank"] == 40


def test_hip_request_without_gpu_raises():
    from nerf_attention._native import NerfhipError
    if torch.cuda.is_available():
        pytest.skip("host has a HIP device")
    with pytest.raises(NerfhipError, match="HIP device"):
        fit_siren(torch.zeros(64, 64), SIRENConfig(64, 1, 30.0, "t"), epochs=1, device="cuda",
                  verbose=False)
    with pytest.raises(NerfhipError):
        engine.resolve_device("meta")


def test_plan_waves():
    assert engine.plan_waves([3, 3, 3], 100) == [[0, 1, 2]]
    assert engine.plan_waves([60, 50, 30, 200, 10], 100) == [[0], [1, 2], [3], [4]]
    assert engine.plan_waves([], 10) == []


def test_latency_harness_cpu(tmp_path):
    """The latency harness on CPU checkpoints (the reference's device='cpu'
    branch): no HIP synchronisation, same record keys."""
    from nerf_attention.fit import _result_to_record, _save_model
    from nerf_attention.latency import profile_latency
    keys, _ = kv_slice(0, 0, seq_len=64, num_layers=4, num_kv_heads=4)
    torch.manual_seed(0)
    r = fit_siren(keys, SIRENConfig(64, 1, 30.0, "tiny"), epochs=3, device="cpu", verbose=False)
    _save_model(tmp_path, "L0_H0_key_tiny", r, _result_to_record("L0_H0_key_tiny", 0, 0, "key", r))
    recs = profile_latency(tmp_path, tmp_path / "lat", device="cpu")
    assert len(recs) == 1 and recs[0]["num_params"] == 12608 and recs[0]["siren_time_ms"] > 0


def test_fit_cli_falls_back_to_cpu(tmp_path, golden_dir):
    """`python -m nerf_attention.fit --quick` on a host without a GPU prints
    the reference's fallback line and runs the package's host path
    (reference fit.py:192-194), with the reference quick run's records and
    stdout structure (schema_quick/)."""
    import os
    import re
    import subprocess
    import sys
    from pathlib import Path
    from nerf_attention.synthetic import extract_kv_cache_synthetic
    root = Path(__file__).resolve().parent.parent
    kv = tmp_path / "kv"
    extract_kv_cache_synthetic(seq_len=512, num_layers=4, num_kv_heads=4, head_dim=128,
                               output_dir=kv)
    env = dict(os.environ, PYTHONPATH=str(root / "nerf-attention_amd"),
               HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-m", "nerf_attention.fit", "--kv_dir", str(kv),
                        "--output_dir", str(tmp_path / "fits"), "--epochs", "20", "--quick",
                        "--seed", "0"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    # numbers masked together with their right-aligned padding (a slower host
    # makes "  9.8s" "10.3s": the column width is not part of the structure)
    num = re.compile(r" *-?\d+\.\d+")
    shape = lambda t: [num.sub(" #", l) for l in t.splitlines()]  # noqa: E731
    ref_out = (golden_dir / "schema_quick" / "stdout.txt").read_text()
    lines = shape(r.stdout)
    assert lines[0] == "CUDA not available, falling back to CPU"
    assert lines[1:-1] == shape(ref_out) + [""] and "sweep wall clock" in lines[-1]
    recs = json.loads((tmp_path / "fits" / "fit_results.json").read_text())
    ref = json.loads((golden_dir / "schema_quick" / "fit_results.json").read_text())
    assert [list(a) for a in recs] == [list(b) for b in ref]
    for a, b in zip(recs, ref):
        assert a["name"] == b["name"] and a["num_parameters"] == b["num_parameters"]
        assert abs(a["final_cosine_mean"] - b["final_cosine_mean"]) <= COS_TOL, a["name"]
    assert len(list((tmp_path / "fits").glob("*_model.pt"))) == 6


def test_bench_cpu_baseline_times_host_path():
    """bench.py's cpu_baseline leg times the package's host path
    (host_fit.fit_on_host) and never imports anything under oracle/."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    code = (
        "import json, sys\n"
        f"sys.path.insert(0, {str(root)!r})\n"
        "import bench\n"
        "r = bench.cpu_baseline(64, 2, repeats=2, warmup_epochs=1, sample_s=0.2)\n"
        f"bad = [m for m, v in list(sys.modules.items()) if {str(root / 'oracle')!r} in "
        "str(getattr(v, '__file__', '') or '')]\n"
        "print(json.dumps({'bad': bad, 'kind': r['kind'], 'port': r['port'], "
        "'value': r['value'], 'archs': len(r['per_epoch_ms'])}))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["bad"] == [] and out["kind"] == "port" and "host_fit" in out["port"]
    assert out["value"] > 0 and out["archs"] == 7


@pytest.mark.parametrize("given,keep,want", [(None, None, "8"), ("4", None, "8"),
                                             ("16", None, "16"), ("2", None, "2"),
                                             ("4", "1", "4")])
def test_bench_raises_hw_queues(given, keep, want):
    """bench.py gives every group stream its own hardware queue: it raises
    GPU_MAX_HW_QUEUES to 8 when unset or at HIP's default of 4 (what the GPU
    boxes export); any other explicit value wins, and NERFHIP_KEEP_HW_QUEUES=1
    keeps the default too."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    env.pop("NERFHIP_KEEP_HW_QUEUES", None)
    if given is not None:
        env["GPU_MAX_HW_QUEUES"] = given
    if keep is not None:
        env["NERFHIP_KEEP_HW_QUEUES"] = keep
    code = (f"import os, sys; sys.path.insert(0, {str(root)!r}); import bench; "
            "print(os.environ['GPU_MAX_HW_QUEUES'])")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == want


def test_bench_pmc_figures_only_for_the_measured_library(tmp_path):
    """bench.committed_pmc reports a committed PMC summary only for the
    library build it was measured on (the summary's lib_sha16); for any other
    build it returns a stale marker without bytes or MFMA busy."""
    import json
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    import bench
    f = tmp_path / "pmc.json"
    f.write_text(json.dumps({"k[bf16x3]": {"bytes": 5.0, "mfma_busy": 0.3, "lib_sha16": "aa"}}))
    assert bench.committed_pmc(f, "k[bf16x3]", "aa")["bytes"] == 5.0
    stale = bench.committed_pmc(f, "k[bf16x3]", "bb")
    assert stale["stale"] and "bytes" not in stale and stale["pmc_lib_sha16"] == "aa"
    assert bench.committed_pmc(f, "other", "aa") is None
    assert bench.committed_pmc(tmp_path / "missing.json", "k[bf16x3]", "aa") is None
    # the committed round-5 summary names the in-tree library when it is current
    real = json.loads((root / "profiles/r05/pmc_isolated_rows256.json").read_text())
    assert all("lib_sha16" in v for v in real.values())
