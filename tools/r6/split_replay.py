"""Drive tools/r6/split_replay.cpp (the CPU/ASan replay of every address the
engine's kernels form) over the group shapes the engine actually plans:

* every rank's share of the 280-fit sweep at 1, 2, 4 and 8 ranks (the 8-rank
  share 0 is the job of the round-5 concurrent split-K fault), with the
  split-K path ON for every group under 8 fits, as engine._Group requests it
  once engine.split_allowed is gone;
* BASELINE config 2 (one medium fit at 2048), config 5 (one wide fit at
  8192), config 4's 40-fit medium chunks at 512..4096, the quick run's shapes;
* edge shapes: ragged seq_len, d_head 64, one and two fits, fp32, probes.

usage: python tools/r6/split_replay.py [--quick] [--bin PATH]
Builds the replay with g++ -fsanitize=address,undefined unless --bin is given.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

import torch  # noqa: E402

from nerf_attention import engine, farm  # noqa: E402
from nerf_attention.fit import select_fits  # noqa: E402
from nerf_attention.types import CONFIG_WIDE, CONFIGS_FULL, KVMetadata, SIRENConfig  # noqa: E402

SRC = ROOT / "tools" / "r6" / "split_replay.cpp"


def build(out: Path) -> Path:
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-I", str(ROOT / "include"),
           "-I", str(ROOT / "nerf-attention_amd" / "csrc"), str(SRC), "-o", str(out)]
    subprocess.run(cmd, check=True)
    return out


def _specs(seq_len, configs, layers, heads):
    """FitSpecs with shape-only targets (plan_groups reads shapes and configs)."""
    out = []
    for _l in layers:
        for _h in range(heads):
            for _kv in ("key", "value"):
                for cfg in configs:
                    out.append(engine.FitSpec(target=torch.empty(seq_len, 128, device="meta"),
                                              config=cfg, init=None))
    return out


def sweep_specs(seq_len=2048):
    meta = KVMetadata(model_name="synthetic", seq_len=seq_len, actual_tokens=seq_len,
                      num_layers=32, num_kv_heads=8, head_dim=128)
    layers, heads, cfgs = select_fits(meta, False)
    return _specs(seq_len, cfgs, layers, heads)


def group_lines(specs, x3=1, split=1, log_every=0):
    """One replay input line per group engine.plan_groups forms for `specs`."""
    lines = []
    for _dev, members in engine.plan_groups(specs, 0):
        cfgs = [specs[i].config for i in members]
        N, D = (int(x) for x in specs[members[0]].target.shape)
        L = [c.hidden_layers for c in cfgs]
        # engine._Group: split-K workspace for groups under SPLIT_MAX_FITS fits
        # whose fused grid is under SPLIT_MIN_TILES workgroups
        small = len(members) * engine.param_tiles(cfgs[0].hidden_features, D, max(L)) \
            < engine.SPLIT_MIN_TILES
        sp = int(split and len(members) < engine.SPLIT_MAX_FITS and small)
        lines.append(" ".join(map(str, [cfgs[0].hidden_features, D, N, len(members), max(L), x3,
                                        sp, log_every] + L)))
    return lines


def shapes(quick=False):
    sweep = sweep_specs(2048)
    costs = [engine.fit_flops(2048, 128, s.config, 1) for s in sweep]
    widths = [s.config.hidden_features for s in sweep]
    lines = ["# the 8-rank share 0 (the round-5 fault's job), split-K on"]
    share0 = farm.rank_share(costs, 8, 0, widths)
    lines += group_lines([sweep[i] for i in share0])
    if not quick:
        for world in (1, 2, 4, 8):
            for rank in range(world):
                mine = farm.rank_share(costs, world, rank, widths)
                lines.append(f"# world {world} rank {rank}")
                lines += group_lines([sweep[i] for i in mine])
        lines.append("# the 8-rank share 0 in fp32")
        lines += group_lines([sweep[i] for i in share0], x3=0)
    med = SIRENConfig(256, 2, 30.0, "medium")
    lines.append("# BASELINE config 2: one medium fit at 2048 (K-split rows, split-K)")
    lines += group_lines(_specs(2048, [med], [0], 1)[:1])
    lines.append("# BASELINE config 5: one wide fit at 8192")
    lines += group_lines(_specs(8192, [CONFIG_WIDE], [0], 1)[:1])
    if not quick:
        for n in (512, 1024, 4096):
            lines.append(f"# BASELINE config 4: 40-fit medium chunk at {n}")
            lines += group_lines(_specs(n, [med], range(20), 1))[:1]
    lines.append("# edges: ragged seq_len, d_head 64, two fits, probes, fp32")
    for cfg in CONFIGS_FULL[:4] if quick else CONFIGS_FULL:
        for n, d in ((1000, 128), (130, 64), (2047, 128)):
            sp = [engine.FitSpec(target=torch.empty(n, d, device="meta"), config=cfg, init=None)]
            lines += group_lines(sp, log_every=1)
            lines += group_lines(sp * 2, x3=0, log_every=1)
            lines += group_lines(sp * 3)
    return lines


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--bin")
    a = ap.parse_args(argv)
    with tempfile.TemporaryDirectory() as t:
        exe = Path(a.bin) if a.bin else build(Path(t) / "split_replay")
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
        r = subprocess.run([str(exe)], input="\n".join(shapes(a.quick)) + "\n", text=True,
                           capture_output=True, env=env)
        sys.stdout.write(r.stdout)
        sys.stderr.write(r.stderr[-5000:])
        return r.returncode


if __name__ == "__main__":
    sys.exit(main())
