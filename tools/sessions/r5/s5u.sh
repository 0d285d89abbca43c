#!/usr/bin/env bash
# round 5: predicted strong scaling (every rank's share alone, 400 epochs) with split-K off for concurrent groups
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/rank_probe.py --epochs 400 --worlds 1,2,4,8 --all-ranks --partition auto > gpurun_out/rank_probe_r05.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/rank_probe_r05.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rank_probe_r05.log | tail -8 | cut -c1-400
