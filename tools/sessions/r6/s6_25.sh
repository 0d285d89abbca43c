#!/usr/bin/env bash
# round 6: BASELINE configs 2, 4 (512 medium fits at 512..4096) and 5 on the
# final library, one GPU
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/configs_bench.py single wide scan > gpurun_out/configs_r06.log 2>&1 || { echo "configs rc=$?"; tail -20 gpurun_out/configs_r06.log; exit 1; }
grep '^{' gpurun_out/configs_r06.log | cut -c1-220
