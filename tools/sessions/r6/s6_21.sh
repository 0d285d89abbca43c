#!/usr/bin/env bash
# round 6: predicted strong scaling on the final library (every rank's share
# timed alone; 8-rank shares now train their small groups split-K
# concurrently): 400 epochs at 1/2/4/8 ranks, then 2000 epochs at 8 and 4
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/rank_probe.py --epochs 400 --worlds 1,2,4,8 --all-ranks --partition auto > gpurun_out/rank_probe_r06.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/rank_probe_r06.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rank_probe_r06.log | tail -6 | cut -c1-300
timeout -k 10 900 python3 -u tools/rank_probe.py --epochs 2000 --worlds 8,4 --all-ranks --partition auto > gpurun_out/rank_probe_r06_e2000.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/rank_probe_r06_e2000.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rank_probe_r06_e2000.log | tail -4 | cut -c1-300
