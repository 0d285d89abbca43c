"""SVD rank-k baseline: oracle pinned to the reference's
own svd_results.json, and the HIP engine (nerfhip_svd_rank_metrics) against
both.  Goldens: tests/golden/make_golden_svd.py (the reference's
run_svd_experiment on its synthetic KV at the quickstart and Llama shapes).

Tolerances: the oracle is the reference's own op sequence, so it must agree to
fp32 rounding (1e-6).  The engine computes in fp64 (Gram + Jacobi +
projection) what the reference computes in fp32 LAPACK, so its cosine
statistics are held to 2e-5 absolute — two orders below the differences the
SVD-vs-SIREN comparison draws (≥1e-3)."""

import json

import numpy as np
import pytest
import torch

import svd_oracle
from nerf_attention.svd import svd_rank
from nerf_attention.synthetic import kv_layer


def _golden(golden_dir, tag):
    return json.loads((golden_dir / f"svd_{tag}.json").read_text())


def _slices(g):
    sh = g["shape"]
    L, H = sh["num_layers"], sh["num_kv_heads"]
    out = {}
    for layer in sorted({0, L // 2, L - 1}):
        t = kv_layer(layer, sh["seq_len"], L, H, sh["head_dim"], heads=range(min(H, 4)))
        for h in range(min(H, 4)):
            out[(layer, h, "key")] = t["keys"][h]
            out[(layer, h, "value")] = t["values"][h]
    return out


@pytest.mark.parametrize("tag", ["q512", "s2048", "s8192"])
def test_oracle_matches_reference(golden_dir, tag):
    g = _golden(golden_dir, tag)
    sl = _slices(g)
    torch.set_num_threads(8)
    for rec in g["records"][:: {"q512": 1, "s2048": 3, "s8192": 7}[tag]]:
        t = sl[(rec["layer"], rec["head"], rec["kv_type"])]
        assert svd_rank(rec["seq_len"], rec["d_head"], rec["target_compression"]) == rec["rank"]
        m = svd_oracle.slice_metrics(t, rec["rank"])
        for k in ("final_cosine_mean", "final_cosine_min", "final_cosine_std"):
            assert m[k] == pytest.approx(rec[k], abs=1e-6), (rec["name"], k)


def test_record_arithmetic(golden_dir):
    for rec in _golden(golden_dir, "s2048")["records"]:
        n, d, r = rec["seq_len"], rec["d_head"], rec["rank"]
        assert rec["svd_size_bytes"] == (n * r + r + r * d) * 4
        assert rec["actual_compression"] == rec["raw_size_bytes"] / rec["svd_size_bytes"]


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["q512", "s2048", "s8192"])
def test_engine_matches_reference(gpu, golden_dir, tag):
    """s8192: BASELINE config 5's SVD leg (experiments/svd.py:48-57 at the
    Llama shape, seq_len 8192), tests/golden/make_golden_svd.py s8192."""
    from nerf_attention.svd import rank_metrics
    g = _golden(golden_dir, tag)
    sl = _slices(g)
    keys = list(sl)
    ranks = sorted({r["rank"] for r in g["records"]})
    out = rank_metrics(torch.stack([sl[k] for k in keys]).to(gpu), ranks)
    for rec in g["records"]:
        t = keys.index((rec["layer"], rec["head"], rec["kv_type"]))
        mean, mn, std = out["stats"][t, ranks.index(rec["rank"])]
        assert abs(mean - rec["final_cosine_mean"]) <= 2e-5, rec["name"]
        assert abs(mn - rec["final_cosine_min"]) <= 2e-5, rec["name"]
        assert abs(std - rec["final_cosine_std"]) <= 2e-5, rec["name"]
    # singular values against LAPACK on the host
    s_ref = torch.linalg.svdvals(sl[keys[0]].double()).numpy()
    np.testing.assert_allclose(out["sigma"][0], s_ref, rtol=1e-6, atol=1e-9 * s_ref[0])


@pytest.mark.gpu
def test_engine_head_dim_64_and_ragged(gpu):
    from nerf_attention.svd import rank_metrics
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 301, 64, generator=g) @ torch.randn(64, 64, generator=g) * 0.1
    ranks = [1, 7, 32, 64]
    out = rank_metrics(x.to(gpu), ranks)
    for t in range(3):
        for k, r in enumerate(ranks):
            m = svd_oracle.slice_metrics(x[t].double(), r)
            np.testing.assert_allclose(out["row_cos"][t, k].cpu().numpy(),
                                       m["cosine_sims"].numpy(), atol=2e-6)
    assert np.allclose(out["stats"][:, -1, 0], 1.0, atol=1e-6)     # full rank: exact


@pytest.mark.gpu
def test_run_svd_experiment_schema(gpu, golden_dir, tmp_path, capsys):
    from nerf_attention import extract_kv_cache_synthetic
    from nerf_attention.svd import run_svd_experiment
    g = _golden(golden_dir, "q512")
    sh = g["shape"]
    extract_kv_cache_synthetic(seq_len=sh["seq_len"], num_layers=sh["num_layers"],
                               num_kv_heads=sh["num_kv_heads"], head_dim=sh["head_dim"],
                               output_dir=tmp_path / "kv")
    capsys.readouterr()
    recs = run_svd_experiment(tmp_path / "kv", tmp_path / "svd")
    out = capsys.readouterr().out
    ref = g["records"]
    assert [r["name"] for r in recs] == [r["name"] for r in ref]
    assert [list(r) for r in recs] == [list(r) for r in ref]
    on_disk = json.loads((tmp_path / "svd" / "svd_results.json").read_text())
    assert on_disk == recs
    for a, b in zip(recs, ref):
        for k in ("rank", "target_compression", "actual_compression", "raw_size_bytes",
                  "svd_size_bytes", "seq_len", "d_head", "layer", "head", "kv_type"):
            assert a[k] == b[k]
        assert abs(a["final_cosine_mean"] - b["final_cosine_mean"]) <= 2e-5
    # same stdout lines (4-decimal cosines may differ in the last digit only at a tie)
    assert [l.split(":")[0] for l in out.splitlines() if l.startswith("  L")] == \
        [l.split(":")[0] for l in g["stdout"].splitlines() if l.startswith("  L")]
    assert "SVD Summary:" in out
