"""Golden fixtures for the KV structure analysis, by running the REFERENCE.

Test infrastructure only (build container; the reference does not exist on
the GPU box).  Runs the reference `analyze_kv_cache`
(nerf_attention/analyze.py:95-213) on its own synthetic KV cache
(extract.py:182-259), and its per-slice `_analyze_tensor` (analyze.py:61-80),
at two shapes; stores analysis_results.json, the stdout, and every slice's
result dict:

  analysis_q512.json    quickstart shape: 4 layers x 4 KV heads x 512 x 128
  analysis_s2048.json   Llama-3.1-8B shape: 32 layers x 8 KV heads x 2048 x 128

Usage (from the repo root):
    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \\
        python tests/golden/make_golden_analysis.py
"""

from __future__ import annotations

import contextlib
import io
import json
import os
import tempfile
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent


def main():
    from nerf_attention import analyze, extract
    assert "/root/reference" in os.path.abspath(analyze.__file__), analyze.__file__
    torch.set_num_threads(8)
    for tag, shape in (("q512", (512, 4, 4, 128)), ("s2048", (2048, 32, 8, 128))):
        with tempfile.TemporaryDirectory() as tmp:
            kv, out = Path(tmp) / "kv", Path(tmp) / "analysis"
            n, layers, heads, d = shape
            with contextlib.redirect_stdout(io.StringIO()):
                extract.extract_kv_cache_synthetic(seq_len=n, num_layers=layers,
                                                   num_kv_heads=heads, head_dim=d, output_dir=kv)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                analyze.analyze_kv_cache(kv, out)
            summary = json.loads((out / "analysis_results.json").read_text())
            slices = {}
            for layer in analyze._select_layers(layers):
                data = torch.load(kv / f"layer_{layer:02d}.pt", weights_only=True)
                for h in range(min(heads, 4)):
                    for tag_kv, t in (("K", data["keys"][h]), ("V", data["values"][h])):
                        name = f"L{layer}_H{h}_{tag_kv}"
                        slices[name] = analyze._analyze_tensor(t, name)
        (HERE / f"analysis_{tag}.json").write_text(json.dumps(
            {"shape": {"seq_len": n, "num_layers": layers, "num_kv_heads": heads,
                       "head_dim": d},
             "stdout": buf.getvalue(), "summary": summary, "slices": slices}, indent=1))
        print(tag, len(slices), "slices")


if __name__ == "__main__":
    main()
