#!/usr/bin/env bash
# round 5: predicted strong scaling (every rank's share alone, 2000 epochs) with split-K off for concurrent groups
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/rank_probe.py --epochs 2000 --worlds 8,4 --all-ranks --partition auto > gpurun_out/rank_probe_r05_e2000.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/rank_probe_r05_e2000.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rank_probe_r05_e2000.log | tail -8 | cut -c1-400
