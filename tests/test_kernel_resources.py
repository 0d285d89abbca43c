"""Scratch (private segment) of the shipped kernels, read from the built
library's gfx950 code objects (host only, tools/kernel_resources.py).

A runtime layout select in the parameter kernel's Adam epilogue once put its
staging arrays in scratch (576 B per lane) and made the W = 512 parameter
kernel 7x slower with results unchanged (DESIGN.md §10, K-split weight
layout): parity tests cannot see that, so the resource metadata is pinned
here.  The regular bf16x3 row kernel at W = 256 keeps its documented spills
(two waves per SIMD beat one wave with no spills by 25 %)."""

import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

import kernel_resources  # noqa: E402

pytestmark = pytest.mark.skipif(
    not kernel_resources.LIB.exists() or shutil.which("objcopy") is None
    or shutil.which("c++filt") is None or not (kernel_resources.LLVM / "llvm-readelf").exists(),
    reason="built library or binutils/LLVM tools missing")

# kernels allowed to use scratch, with their current size (bytes per lane)
KNOWN_SCRATCH = {
    "void k_step_rows<256, 128, true, true>(nerfhip_detail::KArgs)": 120,
    "void k_step_rows<256, 64, true, true>(nerfhip_detail::KArgs)": 120,
    "void k_step_params<128, 128, true, false, false>(nerfhip_detail::KArgs)": 12,
}


@pytest.fixture(scope="module")
def ks():
    return kernel_resources.kernels()


def test_every_step_kernel_present(ks):
    names = " ".join(ks)
    for k in ("k_step_rows<", "k_step_rows_ks<", "k_step_params<", "k_adam_split<",
              "k_transpose_params", "k_normalize", "k_row_metrics"):
        assert k in names, k
    # the fused parameter step in the K-split layout (KSX) exists for every K-split width
    for w in (128, 256, 512):
        assert f"void k_step_params<{w}, 128, true, false, true>(nerfhip_detail::KArgs)" in ks


def test_no_unexpected_scratch(ks):
    bad = {n: v["private_segment_fixed_size"] for n, v in ks.items()
           if v.get("private_segment_fixed_size", 0) > KNOWN_SCRATCH.get(n, 0)}
    assert not bad, bad


def test_lds_within_cu(ks):
    for n, v in ks.items():
        assert v.get("group_segment_fixed_size", 0) <= 160 * 1024, n
