#!/usr/bin/env bash
# GPU parity suite + predicted multi-GPU scaling (every rank's share alone).
set -u
out=gpurun_out/${1:-scale}; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gputests.log 2>&1 || { tail -30 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
timeout -k 10 400 python -u tools/rank_probe.py --worlds 1,2,4,8 --all-ranks --partition auto > $out/rank_probe.log 2>&1 || { tail $out/rank_probe.log; exit 1; }
grep -v "^W\|amdgpu.ids" $out/rank_probe.log
