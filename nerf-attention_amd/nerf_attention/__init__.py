"""nerf-attention-amd: MI355X-native engine for the SIREN KV-fit path of
ruskaruma/nerf-attention.

Public names mirror the reference package (nerf_attention/__init__.py:1-21)
for the in-scope path: the types, the SIREN model, `fit_siren`,
`fit_kv_cache` and the synthetic KV generator that feeds them.  The
reference's analysis / evaluation / plotting modules are out of scope
 and are not provided.
"""

from .types import (
    CONFIG_WIDE,
    CONFIGS_FULL,
    CONFIGS_QUICK,
    FitResult,
    KVMetadata,
    SIRENConfig,
)
from .siren import SIREN, SineLayer, fit_siren
from .synthetic import extract_kv_cache_synthetic
from .fit import fit_kv_cache
from . import ops  # registers torch.ops.nerfhip.*

__all__ = [
    "CONFIG_WIDE", "CONFIGS_FULL", "CONFIGS_QUICK", "FitResult", "KVMetadata", "SIRENConfig",
    "SIREN", "SineLayer", "fit_siren", "fit_kv_cache", "extract_kv_cache_synthetic",
]
