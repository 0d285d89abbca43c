"""The reference's evaluation entry points that its callers import
(quickstart.py:8-15): `load_results` reads the sweep's output schema
(evaluate.py:29-31), `profile_latency` is the engine-backed forward-latency
harness (latency.py, evaluate.py:173-242).

The figures (`plot_pareto_frontier`, `generate_summary_figure`, …,
evaluate.py:48-343) are out of scope: they keep their
signatures so the reference's scripts run unchanged, print that they were
skipped and write no file.
"""

from __future__ import annotations

import json
from pathlib import Path

from .latency import load_model_from_checkpoint, profile_latency  # noqa: F401


def load_results(siren_dir: Path) -> list[dict]:
    """The records of `{siren_dir}/fit_results.json` (fit.py:95-118 schema)."""
    with open(Path(siren_dir) / 'fit_results.json') as f:
        return json.load(f)


def _skipped(figure: str) -> None:
    print(f"  Skipped: {figure} (figures are out of scope for nerf-attention-amd)")


def plot_pareto_frontier(results: list[dict], output_dir: Path, svd_results=None) -> None:
    _skipped('pareto_frontier.png')


def plot_keys_vs_values(results: list[dict], output_dir: Path) -> None:
    _skipped('keys_vs_values.png')


def plot_per_position_error(siren_dir: Path, kv_dir: Path, output_dir: Path,
                            device: str = 'cpu') -> None:
    _skipped('per_position_error.png')


def generate_summary_figure(results: list[dict], output_dir: Path) -> None:
    _skipped('summary_figure.png')
