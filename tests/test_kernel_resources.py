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
    "void k_step_params<128, 128, true, false, 0, false>(nerfhip_detail::KArgs)": 12,
    # the opt-in 32-row kernel: a few spill slots at 512 registers
    "void k_step_rows32<256, 128, true>(nerfhip_detail::KArgs)": 20,
}


@pytest.fixture(scope="module")
def ks():
    return kernel_resources.kernels()


def test_every_step_kernel_present(ks):
    names = " ".join(ks)
    for k in ("k_step_rows<", "k_step_rows_ks<", "k_step_params<", "k_adam_split<",
              "k_transpose_params", "k_normalize", "k_row_metrics"):
        assert k in names, k
    # the fused parameter step in the K-split weight layout (KSX = kLayKs = 1)
    # exists for every K-split width
    for w in (128, 256, 512):
        assert f"void k_step_params<{w}, 128, true, false, 1, false>(nerfhip_detail::KArgs)" in ks
    # regular tiles (unsplit, and split-K with the k_adam_split pass), and the
    # 64 x 64 split-K tiles of lone W >= 256 fits
    for w in (64, 128, 256, 512):
        assert f"void k_step_params<{w}, 128, true, false, 0, false>(nerfhip_detail::KArgs)" in ks
    assert "void k_step_params<256, 128, true, true, 0, false>(nerfhip_detail::KArgs)" in ks


def test_product_library_has_no_opt_in_kernels(ks):
    """the shipped library instantiates only kernels the
    engine launches by default.  The 32-row row kernel and the fused split-K
    reduction (measured slower) exist only in NERFHIP_VARIANTS
    builds (tools/build_variant.py): no k_step_rows32, no SK = true parameter
    kernel, no parameter kernel in the 32-row weight layout (KSX = 2)."""
    names = list(ks)
    assert not [n for n in names if "k_step_rows32" in n]
    assert not [n for n in names if n.startswith("void k_step_params<") and n.endswith(", true>(nerfhip_detail::KArgs)")]
    assert not [n for n in names if n.startswith("void k_step_params<") and ", 2, false>" in n]


# the split-K parameter kernels (SK = true, groups under 8 fits): the fused
# reduction's 16-slab batches spill a little after the tile work (cold path,
# once per tile and epoch; the tile loops themselves stay in registers)
SPLIT_SCRATCH_MAX = 160


def test_no_unexpected_scratch(ks):
    def allowed(n):
        if n.startswith("void k_step_params<") and n.endswith(", true>(nerfhip_detail::KArgs)"):
            return max(KNOWN_SCRATCH.get(n, 0), SPLIT_SCRATCH_MAX)
        return KNOWN_SCRATCH.get(n, 0)
    bad = {n: v["private_segment_fixed_size"] for n, v in ks.items()
           if v.get("private_segment_fixed_size", 0) > allowed(n)}
    assert not bad, bad


def test_lds_within_cu(ks):
    for n, v in ks.items():
        assert v.get("group_segment_fixed_size", 0) <= 160 * 1024, n


def test_ksplit_loads_have_no_late_operand_hazard():
    """The K-split row kernels (k_step_rows_ks) issue no EXEC write and no
    write of an SGPR a vector-memory instruction reads within 8 wait states
    of that instruction (tools/r4/exec_war_scan.py over the built library's
    disassembly; conservative: basic-block boundaries are not seen).  That
    pattern was the root cause of the K-split co-residency fault (DESIGN.md
    §11): under two workgroups per CU a load waiting for the memory pipeline
    read EXEC / its soffset after the write, and fetched nothing or the next
    item.  The kernel source avoids it by construction (one buffer resource,
    VGPR offsets, wave-uniform bias staging, no per-lane branches)."""
    import subprocess
    import tempfile
    sys.path.insert(0, str(ROOT / "tools" / "r4"))
    import exec_war_scan
    if not (kernel_resources.LLVM / "llvm-objdump").exists():
        pytest.skip("llvm-objdump missing")
    seen = 0
    with tempfile.TemporaryDirectory() as t:
        for co in kernel_resources.code_objects(kernel_resources.LIB, Path(t)):
            dis = subprocess.run([str(kernel_resources.LLVM / "llvm-objdump"), "-d",
                                  "--mcpu=gfx950", str(co)], capture_output=True, text=True,
                                 check=True).stdout
            if "k_step_rows_ks" not in dis:
                continue
            seen += dis.count("k_step_rows_ks") > 0
            bad = {k: v for k, v in exec_war_scan.scan(dis.splitlines(), 8).items()
                   if "k_step_rows_ks" in k and (v[0] or v[1])}
            assert not bad, bad
    assert seen, "no K-split kernel found in the library"
