#!/usr/bin/env bash
# round 5: first run of the 32-row kernel (k_step_rows32) against the 16-row one
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/r5/rows32_check.py > gpurun_out/rows32_check.log 2>&1 || { echo "check rc=$?"; tail -30 gpurun_out/rows32_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rows32_check.log
