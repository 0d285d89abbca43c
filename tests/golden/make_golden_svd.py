"""Golden fixtures for the SVD rank-k baseline, by running the REFERENCE.

Test infrastructure only (build container; the reference does not exist on
the GPU box).  Runs the reference `run_svd_experiment`
(nerf_attention/experiments/svd.py:19-85) on the reference's own synthetic KV
cache (extract.py:182-259) at two shapes and stores its svd_results.json:

  svd_q512.json    quickstart shape: 4 layers x 4 KV heads x 512 x 128
  svd_s2048.json   Llama-3.1-8B shape: 32 layers x 8 KV heads x 2048 x 128

Usage (from the repo root):
    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \\
        python tests/golden/make_golden_svd.py
"""

from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import tempfile
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent


def main():
    from nerf_attention import extract
    from nerf_attention.experiments import svd
    assert "/root/reference" in os.path.abspath(svd.__file__), svd.__file__
    torch.set_num_threads(8)
    shapes = {"q512": (512, 4, 4, 128), "s2048": (2048, 32, 8, 128),
              # BASELINE config 5's SVD leg: the Llama shape at seq_len 8192
              "s8192": (8192, 32, 8, 128)}
    tags = sys.argv[1:] or ["q512", "s2048"]
    for tag, shape in ((t, shapes[t]) for t in tags):
        with tempfile.TemporaryDirectory() as tmp:
            kv, out = Path(tmp) / "kv", Path(tmp) / "svd"
            n, layers, heads, d = shape
            with contextlib.redirect_stdout(io.StringIO()):
                extract.extract_kv_cache_synthetic(seq_len=n, num_layers=layers,
                                                   num_kv_heads=heads, head_dim=d, output_dir=kv)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                svd.run_svd_experiment(kv, out)
            records = json.loads((out / "svd_results.json").read_text())
        (HERE / f"svd_{tag}.json").write_text(json.dumps(
            {"shape": {"seq_len": n, "num_layers": layers, "num_kv_heads": heads, "head_dim": d},
             "stdout": buf.getvalue(), "records": records}, indent=1))
        print(tag, len(records), "records")


if __name__ == "__main__":
    main()
