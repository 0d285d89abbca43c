"""Scratch (private segment) of the shipped kernels, read from the built
library's gfx950 code objects (host only, tools/kernel_resources.py).

A runtime layout select in the parameter kernel's Adam epilogue once put its
staging arrays in scratch (576 B per lane) and made the W = 512 parameter
kernel 7x slower with results unchanged (DESIGN.md §10, K-split weight
layout): parity tests cannot see that, so the resource metadata is pinned
here.  The regular bf16x3 row kernel at W = 256 keeps its documented spills
(two waves per SIMD beat one wave with no spills by 25 %)."""

import re
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


def _functions(dis: str):
    """{mangled name: [instruction text]} of an llvm-objdump -d listing."""
    out, name = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(_Z\w+)>:$", line)
        if m:
            name = m.group(1)
            out[name] = []
            continue
        s = re.sub(r"\s*//.*", "", line).strip()
        if name and s:
            out[name].append(s)
    return out


def test_adam_split_stores_are_never_exec_masked():
    """The concurrent split-K fault of rounds 5-6 was
    k_adam_split's: lanes past the fit's last parameter returned early and the
    final-layer / hidden-layer / bias cases branched per lane, so its stores ran
    under narrowed EXEC, restored one to three instructions after the store;
    with the grid beside other groups' kernels the device faulted on an address
    whose low word was a valid split-weight address of the group and whose high
    word was not.  The kernel is now straight-line: for every instantiation in
    the shipped library, no instruction writes EXEC, every store is a buffer
    store (lanes masked by an out-of-range offset), and every wave drains its
    stores (s_waitcnt vmcnt(0)) before s_endpgm."""
    import subprocess
    import tempfile
    if not (kernel_resources.LLVM / "llvm-objdump").exists():
        pytest.skip("llvm-objdump missing")
    seen = 0
    with tempfile.TemporaryDirectory() as t:
        for co in kernel_resources.code_objects(kernel_resources.LIB, Path(t)):
            dis = subprocess.run([str(kernel_resources.LLVM / "llvm-objdump"), "-d",
                                  "--mcpu=gfx950", str(co)], capture_output=True, text=True,
                                 check=True).stdout
            for name, body in _functions(dis).items():
                if "k_adam_split" not in name:
                    continue
                seen += 1
                exec_w = [s for s in body if s.startswith("s_") and "exec" in s
                          and not s.startswith(("s_cbranch_execz", "s_cbranch_execnz"))]
                assert not exec_w, (name, exec_w[:3])
                stores = [s for s in body if "store" in s.split()[0]]
                assert stores and all(s.startswith("buffer_store") for s in stores), (name, stores[:3])
                for k, s in enumerate(body):
                    if s.startswith("s_endpgm"):
                        prev = [p for p in body[:k] if not p.startswith(("s_mov", "s_nop"))]
                        assert prev and prev[-1].startswith("s_waitcnt") and "vmcnt(0)" in prev[-1], \
                            (name, body[max(0, k - 4):k + 1])
    assert seen >= 64, seen          # 4 widths x 2 head dims x 4 slice counts, per part
