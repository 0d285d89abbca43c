"""The C-ABI library: builds for gfx950, loads, exports every symbol the
header declares, and validates its arguments — no GPU compute here."""

import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from nerf_attention import _build, _native

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "nerfhip.h"


@pytest.fixture(scope="module")
def lib():
    _build.build(verbose=False)
    return _native.load()


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(nerfhip_\w+)\s*\(", text,
                                 flags=re.M)))


def test_header_symbols_exported(lib):
    names = declared_functions()
    assert names == sorted(_native.SIGNATURES), names
    out = subprocess.run(["nm", "-D", "--defined-only", str(_build.LIB)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (nerfhip_\w+)", out))
    assert set(names) <= exported
    for n in names:
        assert getattr(lib, n)


def test_code_object_is_gfx950(lib, tmp_path):
    # --offloading extracts the bundles next to its input: work on a copy
    import shutil
    so = tmp_path / "lib.so"
    shutil.copy(_build.LIB, so)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(so)],
                         capture_output=True, text=True, cwd=tmp_path)
    assert "gfx950" in (out.stdout + out.stderr)


def test_abi_and_status(lib):
    assert lib.nerfhip_abi_version() == _native.ABI_VERSION
    assert lib.nerfhip_status_string(0) == b"ok"
    assert b"hidden_features" in lib.nerfhip_status_string(-1)


@pytest.mark.parametrize("W,D,N,L,E", [(256, 128, 2048, 3, 2000), (64, 64, 130, 1, 5)])
def test_group_sizes(lib, W, D, N, L, E):
    s = _native.group_sizes(W, D, N, L, E)
    n_pad = (N + 63) // 64 * 64       # whole 64-row workgroups
    assert s.n_pad == n_pad
    assert s.params == 2 * W + L * (W * W + W) + W * D + D
    assert s.params_t == L * W * W + W * D
    assert s.scratch == 3 * (L + 1) * W * n_pad + D * n_pad
    assert s.target == n_pad * D and s.rows == n_pad
    assert s.loss_partial == E * n_pad // 16
    nb, sp = n_pad // 16, 1           # split-K slices: even, >= 4 blocks each, <= 16
    while sp < 16 and nb % (4 * sp) == 0 and nb // (2 * sp) >= 4:
        sp *= 2
    assert s.grad_split == sp == {2048: 16, 192: 2}[n_pad]
    # + one int32 arrival counter per parameter tile of the finest tiling (64 x 64
    # for W >= 128, else W x W; fused split step), rounded to 64 elements
    t = 64 if W >= 128 else W
    tiles = L * (W // t) ** 2 + (D // min(D, t)) * (W // t) + W // 64
    assert s.grad_partial == sp * s.params + (tiles + 63) // 64 * 64
    assert s.wsplit == 6 * (L * W * W + W * D)        # bf16x3 split planes, fwd + transposed


@pytest.mark.parametrize("args,code", [((96, 128, 64, 1, 1), -1), ((64, 96, 64, 1, 1), -2),
                                       ((64, 128, 64, 0, 1), -3), ((64, 128, 64, 5, 1), -3),
                                       ((64, 128, 1, 1, 1), -4), ((64, 128, 64, 1, -1), -4)])
def test_group_sizes_rejects(lib, args, code):
    s = _native.NerfhipSizes()
    assert lib.nerfhip_group_sizes(*args, ctypes.byref(s)) == code


def test_fit_rejects_before_touching_device(lib):
    g = _native.NerfhipGroup(W=256, D=128, N=2048, n_fits=1, L_max=2, epochs=10)
    streams = (ctypes.c_void_p * 1)(None)
    assert lib.nerfhip_siren_fit(ctypes.byref(g), 1, streams) == -5       # NULL buffers
    g.W = 100
    assert lib.nerfhip_siren_fit(ctypes.byref(g), 1, streams) == -1
    assert lib.nerfhip_siren_fit(None, 1, streams) == -5
    assert lib.nerfhip_siren_fit_timed(ctypes.byref(g), 1, streams, None) == -5
    assert lib.nerfhip_siren_forward(None, None) == -5
    g.W, g.precision = 256, 7
    assert lib.nerfhip_siren_fit(ctypes.byref(g), 1, streams) == -7      # unknown precision


def _plan(lib, **kw):
    g = _native.NerfhipGroup(**kw)
    p = _native.NerfhipPlan()
    rc = lib.nerfhip_group_plan(ctypes.byref(g), ctypes.byref(p))
    return rc, p


def test_group_plan(lib, monkeypatch):
    """nerfhip_group_plan (host only): BASELINE config 2, one medium fit at
    seq 2048 in bf16x3 with the split-K workspace, takes the K-split row kernel
    (one 16-row block per workgroup) and 8 gradient row slices on 64 x 64
    tiles, reduced by the k_adam_split pass (three launches per epoch); a
    wide fit at 8192 (128 regular workgroups) K-split rows too and 128 x 128
    tiles x 8 slices; 40-fit W = 256 and W = 512 sweep chunks the regular
    kernels.  The opt-in switches of the variant kernels (NERFHIP_SPLIT_FUSED,
    NERFHIP_ROWS32) change nothing in the product library, which does not
    contain those kernels (nerfhip_build_flags bit NERFHIP_BUILD_VARIANTS)."""
    assert lib.nerfhip_build_flags() & 8 == 0
    rc, p = _plan(lib, W=256, D=128, N=2048, n_fits=1, L_max=2, epochs=2000, precision=1,
                  grad_partial=1)
    assert rc == 0
    assert (p.rows_variant, p.grad_split, p.rows_workgroups) == (1, 8, 2048 // 16)
    assert p.params_workgroups == 8 * (2 * 16 + 2 * 4 + 256 // 64)     # 44 64x64 tiles x 8 slices
    assert p.launches_per_epoch == 3
    monkeypatch.setenv("NERFHIP_SPLIT_FUSED", "1")
    assert _plan(lib, W=256, D=128, N=2048, n_fits=1, L_max=2, epochs=2000, precision=1,
                 grad_partial=1)[1].launches_per_epoch == 3
    monkeypatch.delenv("NERFHIP_SPLIT_FUSED")
    rc, p = _plan(lib, W=512, D=128, N=8192, n_fits=1, L_max=3, epochs=2000, precision=1,
                  grad_partial=1)
    assert rc == 0 and (p.rows_variant, p.grad_split) == (1, 8)       # 128 regular -> K-split
    assert p.params_workgroups == 8 * (3 * 16 + 1 * 4 + 512 // 64)     # 60 128x128 tiles
    monkeypatch.setenv("NERFHIP_ROWS32", "1")
    rc, p = _plan(lib, W=256, D=128, N=2048, n_fits=40, L_max=3, epochs=2000, precision=1)
    assert rc == 0 and (p.rows_variant, p.grad_split, p.launches_per_epoch) == (0, 1, 2)
    assert p.rows_workgroups == 8 * 32 * 5                            # XCD map: 40 fits x 32
    rc, p = _plan(lib, W=512, D=128, N=2048, n_fits=40, L_max=2, epochs=2000, precision=1)
    assert rc == 0 and (p.rows_variant, p.grad_split, p.launches_per_epoch) == (0, 1, 2)
    assert p.rows_workgroups == 8 * 32 * 5                            # XCD map: 40 fits x 32
    rc, p = _plan(lib, W=256, D=128, N=1984, n_fits=40, L_max=2, epochs=2000, precision=1)
    assert rc == 0 and p.rows_variant == 0                            # n_pad 1984 = 15.5 x 128
    rc, p = _plan(lib, W=256, D=64, N=2048, n_fits=40, L_max=2, epochs=2000, precision=1)
    assert rc == 0 and p.rows_variant == 0                            # D = 64: regular
    rc, p = _plan(lib, W=256, D=128, N=2048, n_fits=1, L_max=2, epochs=2000, precision=0)
    assert rc == 0 and p.rows_variant == 0                            # fp32: regular rows
    # five wide fits at 512 without the workspace (the engine gives none to
    # 5 x 44 tiles): K-split rows, fused parameter step (k_step_params KSX)
    rc, p = _plan(lib, W=512, D=128, N=512, n_fits=5, L_max=2, epochs=2000, precision=1)
    assert rc == 0 and (p.rows_variant, p.grad_split, p.launches_per_epoch) == (1, 1, 2)
    assert p.rows_workgroups == 5 * 512 // 16
    assert _plan(lib, W=100, D=128, N=64, n_fits=1, L_max=1, epochs=1)[0] == -1
    assert lib.nerfhip_group_plan(None, None) == -5


def test_shipped_library_is_a_product_build(lib):
    """The in-tree libnerfhip.so reports no diagnostic compile-time switch
    (nerfhip_build_flags: NERFHIP_EXP_* timing builds may compute wrong
    results on purpose, NERFHIP_STAMPS / NERFHIP_DIAG_* alter the kernels),
    and every such macro the engine source tests is one the function checks."""
    assert lib.nerfhip_build_flags() == 0
    src = (ROOT / "nerf-attention_amd" / "csrc" / "nerfhip.hip").read_text()
    body = src[src.index("int nerfhip_build_flags(void)"):]
    body = body[:body.index("\n}\n")]
    names = set(re.findall(r"\b(NERFHIP_(?:EXP|DIAG)_[A-Z0-9_]+)\b", src))
    missing = sorted(n for n in names if n not in body)
    assert not missing, missing


def _mt_seed(seed):
    """std::mt19937's seeding recurrence (torch's init_with_uint32)."""
    s = np.zeros(624, dtype=np.uint32)
    s[0] = seed
    for j in range(1, 624):
        p = int(s[j - 1])
        s[j] = (1812433253 * (p ^ (p >> 30)) + j) & 0xFFFFFFFF
    return s


def test_rng_known_answers(lib):
    """nerfhip_rng_uniform_segments on U[0, 1): draw k is (y_k & 2^24-1)/2^24
    for the tempered mt19937 output y_k.  Known answers of the standard
    generator, seed 5489: y_1 = 3499211612, y_10000 = 4123659995 (the C++
    standard's check value); discarded segments advance the same words."""
    st, left, nxt = _mt_seed(5489), ctypes.c_int32(1), ctypes.c_uint32(0)
    out = np.zeros(3, dtype=np.float32)
    counts = np.array([1, 9998, 1, 1], dtype=np.int64)
    lo, hi = np.zeros(4), np.ones(4)
    off = np.array([0, -1, 1, 2], dtype=np.int64)
    assert lib.nerfhip_rng_uniform_segments(
        st.ctypes.data, ctypes.byref(left), ctypes.byref(nxt), 4, counts.ctypes.data,
        lo.ctypes.data, hi.ctypes.data, off.ctypes.data, out.ctypes.data) == 0
    assert out[0] == np.float32((3499211612 & 0xFFFFFF) / 2.0 ** 24)
    assert out[1] == np.float32((4123659995 & 0xFFFFFF) / 2.0 ** 24)
    assert (left.value, nxt.value) == (624 - (10001 - 624 * 16) + 1, 10001 - 624 * 16)


def test_rng_rejects_without_moving_state(lib):
    st, left, nxt = _mt_seed(1), ctypes.c_int32(1), ctypes.c_uint32(0)
    keep = st.copy()
    counts = np.array([5, -1], dtype=np.int64)
    lo, hi, off = np.zeros(2), np.ones(2), np.array([-1, -1], dtype=np.int64)
    args = (counts.ctypes.data, lo.ctypes.data, hi.ctypes.data, off.ctypes.data)
    assert lib.nerfhip_rng_uniform_segments(st.ctypes.data, ctypes.byref(left),
                                            ctypes.byref(nxt), 2, *args, None) == -4
    assert np.array_equal(st, keep) and (left.value, nxt.value) == (1, 0)
    off[0] = 0                                               # kept segment, no output buffer
    counts[1] = 1
    assert lib.nerfhip_rng_uniform_segments(st.ctypes.data, ctypes.byref(left),
                                            ctypes.byref(nxt), 2, *args, None) == -5
    assert lib.nerfhip_rng_uniform_segments(None, ctypes.byref(left), ctypes.byref(nxt),
                                            0, None, None, None, None, None) == -5
    left.value = 0                                           # not a valid generator state
    assert lib.nerfhip_rng_uniform_segments(st.ctypes.data, ctypes.byref(left),
                                            ctypes.byref(nxt), 0, None, None, None, None,
                                            None) == -4
