"""nerf-attention-amd: MI355X-native engine for the SIREN KV-fit path of
ruskaruma/nerf-attention.

Public names mirror the reference package (nerf_attention/__init__.py:1-21)
for the in-scope path: the types, the SIREN model, `fit_siren`,
`fit_kv_cache` and the synthetic KV generator that feeds them, plus the
SURVEY §8f "next" rows on the engine: `analyze_kv_cache` (KV structure
analysis, analyze.py) and `run_svd_experiment` (SVD baseline,
experiments/svd.py), and the evaluation names quickstart.py imports
(`load_results`; the figure functions are no-ops — plotting is out of scope,
SURVEY.md §2.1).
"""

from .types import (
    CONFIG_WIDE,
    CONFIGS_FULL,
    CONFIGS_QUICK,
    AnalysisResult,
    FitResult,
    KVMetadata,
    LayerSummary,
    SIRENConfig,
)
from .siren import SIREN, SineLayer, fit_siren
from .synthetic import extract_kv_cache_synthetic
from .fit import fit_kv_cache
from .analyze import analyze_kv_cache
from .svd import run_svd_experiment
from .evaluate import generate_summary_figure, load_results, plot_pareto_frontier
from . import ops  # registers torch.ops.nerfhip.*

__all__ = [
    "CONFIG_WIDE", "CONFIGS_FULL", "CONFIGS_QUICK", "FitResult", "KVMetadata", "SIRENConfig",
    "SIREN", "SineLayer", "fit_siren", "fit_kv_cache", "extract_kv_cache_synthetic",
    "AnalysisResult", "LayerSummary", "analyze_kv_cache", "run_svd_experiment",
    "load_results", "plot_pareto_frontier", "generate_summary_figure",
]
