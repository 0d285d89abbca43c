"""Pin the oracle (oracle/siren_oracle.py) to the reference.

Every fixture here was produced by running the reference itself
(tests/golden/make_golden.py, torch 2.10 CPU, 2 intra-op threads).  The oracle
replays the same ATen op sequence, so at the same thread count it must match
the reference BIT FOR BIT — parameters, per-epoch losses and final metrics.
"""

import hashlib
import json

import numpy as np
import pytest
import torch

import siren_oracle as O
from nerf_attention.synthetic import kv_slice


@pytest.fixture(autouse=True)
def two_threads():
    old = torch.get_num_threads()
    torch.set_num_threads(2)      # the fixtures' thread count
    yield
    torch.set_num_threads(old)


def _cfg(z):
    W, L, om = z["config"]
    return int(W), int(L), float(om)


@pytest.mark.parametrize("name", ["micro", "tiny", "medium"])
def test_oracle_steps_bit_exact(golden_dir, name):
    z = np.load(golden_dir / f"steps_{name}.npz")
    W, L, om = _cfg(z)
    t = torch.from_numpy(z["target"])
    torch.manual_seed(0)
    init = O.init_params(W, L, om, t.shape[1])
    assert np.array_equal(init.numpy(), z["init"])          # RNG replay of SIREN.__init__
    # step 1 uses lr_0 = 1e-4 whatever T_max is: a snapshot of a longer run matches
    r = O.fit(t, W, L, om, init, 10, record_params_at=(1,))
    assert np.array_equal(r["snapshots"][1].numpy(), z["params_1"])
    for k in (1, 2, 3, 10):
        # T_max = k changes the schedule after step 1: rerun with epochs = k
        rk = O.fit(t, W, L, om, init, k)
        assert np.array_equal(rk["params"].numpy(), z[f"params_{k}"])
        assert rk["losses"] == list(z[f"losses_{k}"])
        got = [rk["final_mse"], rk["final_cosine_mean"], rk["final_cosine_min"],
               rk["final_cosine_std"]]
        assert got == list(z[f"metrics_{k}"])


@pytest.mark.parametrize("name", ["key_tiny", "randn_tiny", "value_small"])
def test_oracle_full_fit_bit_exact(golden_dir, name):
    """2000-epoch fits on the quickstart data and on an N(0,1) target."""
    meta = json.loads((golden_dir / "fits_q512.json").read_text())[name]
    z = np.load(golden_dir / "fits_q512.npz")
    keys, vals = kv_slice(0, 0, seq_len=512, num_layers=4, num_kv_heads=4)
    t = {"key": keys, "value": vals, "randn": torch.from_numpy(z["randn_target"])}[
        name.split("_")[0]]
    W = {"tiny": 64, "small": 128}[name.split("_")[1]]
    torch.manual_seed(0)
    init = O.init_params(W, 1, 30.0, 128)
    r = O.fit(t, W, 1, 30.0, init, 2000, log_every=400)
    assert r["final_cosine_mean"] == meta["final_cosine_mean"]
    assert r["final_mse"] == meta["final_mse"]
    assert np.array_equal(np.array(r["losses"]), z[f"{name}_losses"])
    assert np.array_equal(r["cosine_sims"], z[f"{name}_cos"])
    lines = [f"  Epoch {e}/2000 | NormMSE: {a:.6f} | RealMSE: {b:.6f} | CosSim: {c:.4f}"
             for e, a, b, c in r["probes"]]
    assert lines == meta["log_lines"]


def test_oracle_wide_8192(golden_dir):
    """BASELINE config 5 shape: (512, 3) at seq_len 8192, 30 epochs."""
    g = json.loads((golden_dir / "wide_8192_e30.json").read_text())
    keys, _ = kv_slice(0, 0, seq_len=8192, num_layers=1, num_kv_heads=1)
    assert hashlib.sha256(keys.numpy().tobytes()).hexdigest() == g["target_sha256"]
    torch.manual_seed(0)
    init = O.init_params(512, 3, 30.0, 128)
    r = O.fit(keys, 512, 3, 30.0, init, 30)
    assert r["losses"] == g["losses"]
    assert r["final_cosine_mean"] == g["final_cosine_mean"]
    assert hashlib.sha256(r["params"].numpy().tobytes()).hexdigest() == g["params_sha256"]
