"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Test infrastructure only.  This script imports the read-only reference
(`/root/reference`, ruskaruma/nerf-attention) and is meant to run ONLY in the
build container (the reference does not exist on the GPU box).  The GPU box
and the test-suite only ever read the data files this script writes.

Usage (from the repo root):
    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/make_golden.py small      # seconds-to-minutes
    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/make_golden.py sweep      # ~1 h of CPU

What each fixture pins:
  init.json / init_tiny_small.npz  SIREN init under manual_seed(0)       siren.py:19-58
  sweep_init_order.json            280 inits in fit.py loop order         fit.py:303-319
  steps_*.npz                      params/losses after k Adam steps       siren.py:70-105
  fits_q512.npz / fits_q512.json   2000-epoch fits on quickstart data     siren.py:70-149
  schema_quick/                    fit_kv_cache(quick) records + ckpt     fit.py:20-137
  synthetic.json                   sha256 of extract_kv_cache_synthetic   extract.py:182-259
  sweep_ref_seed0_e2000.json       the 280-fit sweep, seed 0, E=2000      fit.py:20-92
"""

from __future__ import annotations

import contextlib
import hashlib
import io
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
SCRATCH = Path(os.environ.get("GOLDEN_SCRATCH", "/tmp/nerf_golden"))


def _ref():
    import nerf_attention  # noqa: F401  (the reference, via PYTHONPATH)
    from nerf_attention import siren, types, extract, fit
    assert "/root/reference" in os.path.abspath(siren.__file__), siren.__file__
    return siren, types, extract, fit


def flat_state(model) -> np.ndarray:
    return np.concatenate([v.detach().cpu().reshape(-1).numpy().astype(np.float32)
                           for v in model.state_dict().values()])


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


WIDE = (512, 3, 30.0, "wide")


def make_init():
    siren, types, _, _ = _ref()
    out, arrays = {}, {}
    cfgs = list(types.CONFIGS_FULL) + [types.SIRENConfig(*WIDE)]
    for cfg in cfgs:
        torch.manual_seed(0)
        m = siren.SIREN(cfg, 128)
        f = flat_state(m)
        out[cfg.name] = {
            "hidden_features": cfg.hidden_features, "hidden_layers": cfg.hidden_layers,
            "omega_0": cfg.omega_0, "num_parameters": int(f.size),
            "keys": list(m.state_dict().keys()),
            "sha256": sha(f), "first8": f[:8].tolist(), "last8": f[-8:].tolist(),
        }
        if cfg.name in ("tiny", "small"):
            arrays[cfg.name] = f
    (HERE / "init.json").write_text(json.dumps(out, indent=1))
    np.savez_compressed(HERE / "init_tiny_small.npz", **arrays)


def make_sweep_init_order():
    siren, types, _, _ = _ref()
    torch.manual_seed(0)
    hashes = []
    for layer in [0, 8, 16, 24, 31]:
        for head in range(4):
            for kv in ("key", "value"):
                for cfg in types.CONFIGS_FULL:
                    m = siren.SIREN(cfg, 128)
                    hashes.append([f"L{layer}_H{head}_{kv}_{cfg.name}", sha(flat_state(m))])
    (HERE / "sweep_init_order.json").write_text(json.dumps(hashes, indent=0))


def micro_target(n=64, d=8):
    # smooth deterministic target (its bytes are stored in the fixture)
    t = np.linspace(0, 1, n, dtype=np.float64)[:, None]
    j = np.arange(d)[None, :]
    y = np.sin(2 * np.pi * (1 + j) * t) + 0.3 * np.cos(5 * np.pi * t * (j + 0.5))
    return torch.tensor(y, dtype=torch.float32)


def q512_tensors():
    """quickstart synthetic data (extract.py:182-259 at 512x4x4x128)."""
    _, _, extract, _ = _ref()
    d = SCRATCH / "kv_q512"
    if not (d / "layer_00.pt").exists():
        with contextlib.redirect_stdout(io.StringIO()):
            extract.extract_kv_cache_synthetic(seq_len=512, num_layers=4, num_kv_heads=4,
                                               head_dim=128, output_dir=d)
    return d


def make_steps():
    siren, types, _, _ = _ref()
    cases = {
        "micro": (micro_target(), types.SIRENConfig(32, 1, 30.0, "micro")),
    }
    q = torch.load(q512_tensors() / "layer_00.pt", weights_only=True)
    cases["tiny"] = (q["keys"][0].clone(), types.SIRENConfig(64, 1, 30.0, "tiny"))
    cases["medium"] = (q["values"][1].clone(), types.SIRENConfig(256, 2, 30.0, "medium"))
    for name, (x, cfg) in cases.items():
        arr = {"target": x.numpy()}
        for k in (1, 2, 3, 10):
            torch.manual_seed(0)
            r = siren.fit_siren(x, cfg, epochs=k, device="cpu", verbose=False)
            arr[f"params_{k}"] = flat_state(r.model)
            arr[f"losses_{k}"] = np.asarray(r.losses, dtype=np.float64)
            arr[f"metrics_{k}"] = np.array([r.final_mse, r.final_cosine_mean,
                                            r.final_cosine_min, r.final_cosine_std])
        torch.manual_seed(0)
        arr["init"] = flat_state(siren.SIREN(cfg, x.shape[1]))
        arr["config"] = np.array([cfg.hidden_features, cfg.hidden_layers, cfg.omega_0])
        np.savez_compressed(HERE / f"steps_{name}.npz", **arr)


def make_fits_q512():
    siren, types, _, _ = _ref()
    q = torch.load(q512_tensors() / "layer_00.pt", weights_only=True)
    g = torch.Generator().manual_seed(123)
    targets = {"key": q["keys"][0], "value": q["values"][0],
               "randn": torch.randn(512, 128, generator=g)}
    cfgs = {c.name: c for c in types.CONFIGS_FULL}
    plan = [("key", "tiny"), ("key", "small"), ("key", "medium"),
            ("value", "tiny"), ("value", "small"), ("value", "medium"),
            ("randn", "tiny"), ("randn", "medium")]
    arr, meta = {"randn_target": targets["randn"].numpy()}, {}
    for tname, cname in plan:
        name = f"{tname}_{cname}"
        torch.manual_seed(0)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            r = siren.fit_siren(targets[tname], cfgs[cname], epochs=2000, device="cpu",
                                log_every=400, verbose=True)
        arr[f"{name}_losses"] = np.asarray(r.losses, dtype=np.float64)
        arr[f"{name}_cos"] = r.cosine_sims
        arr[f"{name}_ppmse"] = r.per_pos_mse
        arr[f"{name}_params"] = flat_state(r.model)
        meta[name] = {"final_mse": r.final_mse, "final_cosine_mean": r.final_cosine_mean,
                      "final_cosine_min": r.final_cosine_min,
                      "final_cosine_std": r.final_cosine_std,
                      "compression_ratio": r.compression_ratio,
                      "num_parameters": r.num_parameters,
                      "log_lines": buf.getvalue().splitlines(),
                      "train_time_seconds_cpu": r.train_time_seconds,
                      "threads": torch.get_num_threads()}
        print(name, r.final_cosine_mean, flush=True)
    np.savez_compressed(HERE / "fits_q512.npz", **arr)
    (HERE / "fits_q512.json").write_text(json.dumps(meta, indent=1))


def make_wide():
    """(512,3) at N=8192, 30 epochs (short: CPU is 46 ms/epoch)."""
    siren, types, extract, _ = _ref()
    d = SCRATCH / "kv_8192_l1"
    if not (d / "layer_00.pt").exists():
        with contextlib.redirect_stdout(io.StringIO()):
            extract.extract_kv_cache_synthetic(seq_len=8192, num_layers=1, num_kv_heads=1,
                                               head_dim=128, output_dir=d)
    x = torch.load(d / "layer_00.pt", weights_only=True)["keys"][0]
    torch.manual_seed(0)
    r = siren.fit_siren(x, types.SIRENConfig(*WIDE), epochs=30, device="cpu", verbose=False)
    out = {"target_sha256": sha(x.numpy()), "epochs": 30, "losses": r.losses,
           "final_mse": r.final_mse, "final_cosine_mean": r.final_cosine_mean,
           "final_cosine_min": r.final_cosine_min, "final_cosine_std": r.final_cosine_std,
           "params_sha256": sha(flat_state(r.model))}
    (HERE / "wide_8192_e30.json").write_text(json.dumps(out, indent=1))


def make_wide_full():
    """BASELINE config 5 at its stated length: (512,3) at N=8192, 2000 epochs,
    the reference's own fit_siren (siren.py:70-149) under manual_seed(0) on the
    reference's synthetic layer-0 key head 0 (extract.py:182-259)."""
    siren, types, extract, _ = _ref()
    d = SCRATCH / "kv_8192_l1"
    if not (d / "layer_00.pt").exists():
        with contextlib.redirect_stdout(io.StringIO()):
            extract.extract_kv_cache_synthetic(seq_len=8192, num_layers=1, num_kv_heads=1,
                                               head_dim=128, output_dir=d)
    x = torch.load(d / "layer_00.pt", weights_only=True)["keys"][0]
    torch.manual_seed(0)
    t0 = time.time()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        r = siren.fit_siren(x, types.SIRENConfig(*WIDE), epochs=2000, device="cpu",
                            log_every=500, verbose=True)
    out = {"target_sha256": sha(x.numpy()), "epochs": 2000, "losses": r.losses,
           "final_mse": r.final_mse, "final_cosine_mean": r.final_cosine_mean,
           "final_cosine_min": r.final_cosine_min, "final_cosine_std": r.final_cosine_std,
           "cosine_sims_every64": r.cosine_sims[::64].tolist(),
           "log_lines": buf.getvalue().splitlines(),
           "params_sha256": sha(flat_state(r.model)),
           "train_time_seconds_cpu": time.time() - t0, "threads": torch.get_num_threads(),
           "torch": torch.__version__}
    (HERE / "wide_8192_e2000.json").write_text(json.dumps(out, indent=1))


SCAN_LENGTHS = (512, 1024, 4096)


def make_scan():
    """BASELINE config 4 seq-len points: medium fits of layers {0, L/2, L-1},
    head 0, K and V at each length, exactly the selection of the reference's
    scaling experiment (experiments/scaling.py:160-168), on the reference's
    synthetic 32x8xNx128 cache.  torch.manual_seed(0) before every fit."""
    siren, types, extract, _ = _ref()
    medium = types.SIRENConfig(256, 2, 30.0, "medium")
    out = {}
    for n in SCAN_LENGTHS:
        d = SCRATCH / f"kv_{n}"
        if not (d / "layer_31.pt").exists():
            with contextlib.redirect_stdout(io.StringIO()):
                extract.extract_kv_cache_synthetic(seq_len=n, num_layers=32, num_kv_heads=8,
                                                   head_dim=128, output_dir=d)
        recs = []
        for layer in (0, 16, 31):
            data = torch.load(d / f"layer_{layer:02d}.pt", weights_only=True)
            for kv, t in (("key", data["keys"][0]), ("value", data["values"][0])):
                torch.manual_seed(0)
                t0 = time.time()
                r = siren.fit_siren(t, medium, epochs=2000, device="cpu", log_every=2000,
                                    verbose=False)
                recs.append({"name": f"L{layer}_H0_{kv}_medium", "layer": layer, "kv_type": kv,
                             "target_sha256": sha(t.numpy()),
                             "final_cosine_mean": r.final_cosine_mean,
                             "final_cosine_min": r.final_cosine_min,
                             "final_mse": r.final_mse, "losses_every100": r.losses[::100],
                             "train_time_seconds_cpu": time.time() - t0})
                print(n, recs[-1]["name"], r.final_cosine_mean, flush=True)
        out[str(n)] = {"records": recs, "threads": torch.get_num_threads(),
                       "torch": torch.__version__, "epochs": 2000, "seed": 0}
    (HERE / "scan_medium_e2000.json").write_text(json.dumps(out, indent=1))


SCAN_ALL_N, SCAN_ALL_EPOCHS = 512, 200


def make_scan_all():
    """BASELINE config 4 at its stated size: medium on every layer x head x K/V
    of the 32x8xNx128 cache (512 fits), seeded once with manual_seed(0) and
    initialised in the reference's loop order (fit.py:54-69: layer -> head ->
    key/value), 200 epochs.  The fits of the scaling experiment's selection
    (layers {0, 16, 31}, head 0, K/V; experiments/scaling.py:160-168) are
    trained by the reference's own fit_siren from exactly the RNG state they
    would see in that loop; every other fit only consumes its init (a
    reference SIREN construction: fit_siren draws nothing else from the RNG)."""
    siren, types, extract, _ = _ref()
    medium = types.SIRENConfig(256, 2, 30.0, "medium")
    d = SCRATCH / f"kv_{SCAN_ALL_N}"
    if not (d / "layer_31.pt").exists():
        with contextlib.redirect_stdout(io.StringIO()):
            extract.extract_kv_cache_synthetic(seq_len=SCAN_ALL_N, num_layers=32, num_kv_heads=8,
                                               head_dim=128, output_dir=d)
    torch.manual_seed(0)
    recs, idx = [], 0
    for layer in range(32):
        data = torch.load(d / f"layer_{layer:02d}.pt", weights_only=True)
        for head in range(8):
            for kv, t in (("key", data["keys"][head]), ("value", data["values"][head])):
                if head == 0 and layer in (0, 16, 31):
                    r = siren.fit_siren(t, medium, epochs=SCAN_ALL_EPOCHS, device="cpu",
                                        log_every=max(SCAN_ALL_EPOCHS // 5, 100), verbose=False)
                    recs.append({"name": f"L{layer}_H0_{kv}_medium", "index": idx,
                                 "target_sha256": sha(t.numpy()),
                                 "final_cosine_mean": r.final_cosine_mean,
                                 "final_cosine_min": r.final_cosine_min,
                                 "final_mse": r.final_mse, "losses_every20": r.losses[::20]})
                    print(recs[-1]["name"], r.final_cosine_mean, flush=True)
                else:
                    siren.SIREN(medium, out_features=128)
                idx += 1
    (HERE / "scan_all_medium_e200.json").write_text(json.dumps({
        "seq_len": SCAN_ALL_N, "epochs": SCAN_ALL_EPOCHS, "n_fits": idx, "seed": 0,
        "threads": torch.get_num_threads(), "torch": torch.__version__, "records": recs},
        indent=1))


def make_schema():
    _, _, _, fit = _ref()
    out = SCRATCH / "fits_quick_e20"
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()) as buf:
        fit.fit_kv_cache(q512_tensors(), out, epochs=20, device="cpu", quick=True)
    d = HERE / "schema_quick"
    d.mkdir(exist_ok=True)
    recs = json.loads((out / "fit_results.json").read_text())
    (d / "fit_results.json").write_text(json.dumps(recs, indent=2))
    ck = torch.load(out / "L0_H0_key_medium_model.pt", weights_only=True)
    (d / "checkpoint_layout.json").write_text(json.dumps({
        "top_keys": list(ck.keys()),
        "model_state_keys": list(ck["model_state"].keys()),
        "model_state_shapes": {k: list(v.shape) for k, v in ck["model_state"].items()},
        "config": ck["config"],
        "target_mean_shape": list(ck["target_mean"].shape),
        "metrics_keys": list(ck["metrics"].keys()),
    }, indent=1))
    (d / "stdout.txt").write_text(buf.getvalue())


def make_synthetic_hashes(kv2048: Path | None = None):
    out = {"q512": {}}
    q = q512_tensors()
    for l in range(4):
        t = torch.load(q / f"layer_{l:02d}.pt", weights_only=True)
        out["q512"][f"layer_{l:02d}"] = {"keys": sha(t["keys"].numpy()),
                                         "values": sha(t["values"].numpy())}
    out["q512"]["metadata"] = json.loads((q / "metadata.json").read_text())
    if kv2048 is not None:
        out["s2048"] = {}
        for l in [0, 8, 16, 24, 31]:
            t = torch.load(kv2048 / f"layer_{l:02d}.pt", weights_only=True)
            out["s2048"][f"layer_{l:02d}"] = {
                "keys": [sha(t["keys"][h].numpy()) for h in range(8)],
                "values": [sha(t["values"][h].numpy()) for h in range(8)]}
        out["s2048"]["metadata"] = json.loads((kv2048 / "metadata.json").read_text())
    p = HERE / "synthetic.json"
    old = json.loads(p.read_text()) if p.exists() else {}
    old.update(out)
    p.write_text(json.dumps(old, indent=1))


def make_sweep():
    _, _, extract, fit = _ref()
    kv = SCRATCH / "kv_2048"
    if not (kv / "layer_31.pt").exists():
        extract.extract_kv_cache_synthetic(seq_len=2048, num_layers=32, num_kv_heads=8,
                                           head_dim=128, output_dir=kv)
    make_synthetic_hashes(kv)
    torch.manual_seed(0)
    t0 = time.time()
    recs = fit.fit_kv_cache(kv, SCRATCH / "fits_sweep", epochs=2000, device="cpu", quick=False)
    wall = time.time() - t0
    (HERE / "sweep_ref_seed0_e2000.json").write_text(json.dumps({
        "wall_seconds_cpu": wall, "threads": torch.get_num_threads(),
        "torch": torch.__version__, "records": recs}, indent=1))


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "small"
    if "threads" in os.environ:
        torch.set_num_threads(int(os.environ["threads"]))
    if what == "sweep":
        make_sweep()
    elif what == "small":
        for f in (make_init, make_sweep_init_order, make_steps, make_schema,
                  make_synthetic_hashes, make_wide, make_fits_q512):
            t = time.time()
            f()
            print(f.__name__, f"{time.time() - t:.1f}s", flush=True)
    else:
        globals()[f"make_{what}"]()
