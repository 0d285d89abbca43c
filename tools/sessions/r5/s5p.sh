#!/usr/bin/env bash
# round 5: isolated-leg roofline profile (kernel trace + PMC passes) of the current library
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 bash tools/r4/iso_prof.sh r05 256 rows > gpurun_out/iso_prof_r05.log 2>&1 || { echo "iso rc=$?"; tail -20 gpurun_out/iso_prof_r05.log; exit 1; }
tail -30 gpurun_out/iso_prof_r05.log
