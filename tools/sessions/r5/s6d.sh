#!/usr/bin/env bash
# round 5: BASELINE config 4 at its stated size (512 medium fits per length, 2000 epochs) and configs 2 / 5, current tree
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/configs_bench.py single wide scan > gpurun_out/configs_r05.log 2>&1 || { echo "configs rc=$?"; tail -20 gpurun_out/configs_r05.log; exit 1; }
grep '^{' gpurun_out/configs_r05.log | cut -c1-300
