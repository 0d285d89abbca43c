"""CPU replay of the engine's kernel addresses under AddressSanitizer
(tools/r6/split_replay.cpp).

The replay walks every block, wave and lane of the kernels an epoch launches
(row step, parameter step with and without split-K slices, k_adam_split, the
prologue and the final evaluation) with the kernels' own index functions
(csrc/nerfhip_layout.h) over exactly-sized heap buffers.  Here: the groups of
the 8-rank share 0 that take the split-K path (5 W = 128 and 5 W = 64 fits,
16 row slices — the job of the round-5 concurrent split-K fault), BASELINE
config 2's lone medium fit (K-split rows, 64 x 64 split-K tiles), and ragged /
d_head 64 / probe / fp32 edges.  The whole share and every other rank's share
are replayed by `python tools/r6/split_replay.py` (profiles/r06/split_replay_full.log)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools" / "r6"))


@pytest.fixture(scope="module")
def replay(tmp_path_factory):
    import split_replay
    try:
        return split_replay, split_replay.build(tmp_path_factory.mktemp("replay") / "split_replay")
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"g++ with ASan unavailable: {e}")


def _run(exe, lines, **env):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1", **env)
    return subprocess.run([str(exe)], input="\n".join(lines) + "\n", text=True, capture_output=True,
                          env=e, timeout=600)


def test_replay_harness_catches_an_overflow(replay):
    _mod, exe = replay
    r = _run(exe, [], NERFHIP_REPLAY_SELFTEST="1")
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr


def test_split_path_addresses_in_bounds(replay):
    mod, exe = replay
    from nerf_attention import engine, farm
    from nerf_attention.types import SIRENConfig
    sweep = mod.sweep_specs(2048)
    costs = [engine.fit_flops(2048, 128, s.config, 1) for s in sweep]
    share0 = farm.rank_share(costs, 8, 0, [s.config.hidden_features for s in sweep])
    lines = [l for l in mod.group_lines([sweep[i] for i in share0]) if int(l.split()[0]) <= 128]
    assert len(lines) == 2 and all(l.split()[6] == "1" for l in lines)   # both on split-K
    med = SIRENConfig(256, 2, 30.0, "medium")
    lines += mod.group_lines(mod._specs(2048, [med], [0], 1)[:1])
    for W, n, d in ((64, 130, 64), (128, 1000, 128)):
        sp = [engine.FitSpec(target=torch.empty(n, d, device="meta"),
                             config=SIRENConfig(W, 1, 30.0, "t"), init=None)]
        lines += mod.group_lines(sp * 2, log_every=1) + mod.group_lines(sp * 3, x3=0)
    r = _run(exe, lines)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip().splitlines()[-1].startswith(f"OK {len(lines)} groups")
    assert "slices 16" in r.stdout and "64x64 tiles" in r.stdout and "rows=ksplit" in r.stdout
