"""KV structure analysis: oracle pinned to the reference's
own per-slice results, and the HIP engine (nerfhip_kv_analysis +
nerfhip_svd_rank_metrics) against both.  Goldens:
tests/golden/make_golden_analysis.py.

Tolerances: the oracle repeats the reference's numpy/torch operations, so it
agrees to rounding (1e-9).  The engine computes in fp64 what the reference
computes partly in fp32 (numpy float32 autocorrelation sums, fp32 LAPACK
singular values): autocorrelations within 2e-6, spectral fractions within
1e-9, singular-value fractions within 1e-5, effective rank exact."""

import json

import numpy as np
import pytest
import torch

import analysis_oracle
from nerf_attention.analyze import sampled_dims, select_layers
from nerf_attention.synthetic import kv_layer


def _golden(golden_dir, tag):
    return json.loads((golden_dir / f"analysis_{tag}.json").read_text())


def _slices(g):
    sh = g["shape"]
    L, H = sh["num_layers"], sh["num_kv_heads"]
    out = {}
    for layer in select_layers(L):
        t = kv_layer(layer, sh["seq_len"], L, H, sh["head_dim"], heads=range(min(H, 4)))
        for h in range(min(H, 4)):
            out[f"L{layer}_H{h}_K"] = t["keys"][h]
            out[f"L{layer}_H{h}_V"] = t["values"][h]
    return out


def _close(a, b, ac_tol, en_tol, sv_tol):
    assert a["name"] == b["name"] and a["shape"] == b["shape"]
    np.testing.assert_allclose(a["mean_autocorrelation"], b["mean_autocorrelation"], atol=ac_tol)
    assert abs(a["lag1_autocorrelation"] - b["lag1_autocorrelation"]) <= ac_tol
    for k in b["spectral_energy"]:
        assert abs(a["spectral_energy"][k] - b["spectral_energy"][k]) <= en_tol, k
    for k in ("effective_rank_99", "full_rank"):
        assert a["rank"][k] == b["rank"][k], (a["name"], k, a["rank"][k], b["rank"][k])
    for k in ("rank_ratio", "top_sv_fraction", "top_10_sv_fraction"):
        assert abs(a["rank"][k] - b["rank"][k]) <= sv_tol, k


@pytest.mark.parametrize("tag", ["q512", "s2048"])
def test_oracle_matches_reference(golden_dir, tag):
    g = _golden(golden_dir, tag)
    sl = _slices(g)
    torch.set_num_threads(8)
    names = list(g["slices"])[:: (1 if tag == "q512" else 4)]
    for name in names:
        _close(analysis_oracle.analyze_tensor(sl[name], name), g["slices"][name],
               1e-9, 1e-9, 1e-7)


def test_selection():
    assert select_layers(32) == [0, 8, 16, 24, 31] and select_layers(4) == [0, 1, 2, 3]
    assert sampled_dims(128) == list(range(0, 128, 8)) and sampled_dims(8) == list(range(8))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["q512", "s2048"])
def test_engine_matches_reference(gpu, golden_dir, tag):
    from nerf_attention.analyze import analyze_slices
    g = _golden(golden_dir, tag)
    sl = _slices(g)
    names = list(g["slices"])
    out = analyze_slices(torch.stack([sl[n] for n in names]).to(gpu), names)
    for a in out:
        _close(a, g["slices"][a["name"]], 2e-6, 1e-9, 1e-5)


@pytest.mark.gpu
def test_engine_edge_cases(gpu):
    """Constant columns (var < 1e-10 → zero autocorrelation, unit spectral
    fractions), odd length (no quarter-wave twiddle symmetry), d_head 64."""
    from nerf_attention.analyze import kv_measures
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 301, 64, generator=g).cumsum(1) * 0.01
    x[1, :, 3] = 0.25
    dims = [0, 3, 63]
    m = kv_measures(x.to(gpu), dims)
    for t in range(2):
        for i, d in enumerate(dims):
            col = x[t, :, d].numpy()
            np.testing.assert_allclose(m["autocorr"][t, i], analysis_oracle.autocorrelation(col),
                                       atol=2e-6)
            ref = analysis_oracle.spectral_energy(col)
            np.testing.assert_allclose(m["energy"][t, i], [ref[k] for k in ref], atol=1e-9)


@pytest.mark.gpu
def test_analyze_kv_cache_schema(gpu, golden_dir, tmp_path, capsys):
    from nerf_attention import analyze_kv_cache, extract_kv_cache_synthetic
    g = _golden(golden_dir, "q512")
    sh = g["shape"]
    extract_kv_cache_synthetic(seq_len=sh["seq_len"], num_layers=sh["num_layers"],
                               num_kv_heads=sh["num_kv_heads"], head_dim=sh["head_dim"],
                               output_dir=tmp_path / "kv")
    capsys.readouterr()
    res = analyze_kv_cache(tmp_path / "kv", tmp_path / "an")
    out = capsys.readouterr().out
    got = json.loads((tmp_path / "an" / "analysis_results.json").read_text())
    ref = g["summary"]
    assert list(got) == list(ref) and got["metadata"] == ref["metadata"]
    assert [s["layer"] for s in got["layer_summaries"]] == [s["layer"] for s in ref["layer_summaries"]]
    for a, b in zip(got["layer_summaries"], ref["layer_summaries"]):
        assert list(a) == list(b)
        for k in b:
            assert abs(a[k] - b[k]) <= 1e-5, k
    for k in ref["assessment"]:
        assert abs(got["assessment"][k] - ref["assessment"][k]) <= 1e-5
    assert res.avg_autocorr_keys == pytest.approx(ref["assessment"]["avg_autocorr_keys"], abs=1e-5)
    keep = lambda s: [l for l in s.splitlines() if "Saved plot" not in l and "saved to" not in l]
    assert keep(out) == keep(g["stdout"])
