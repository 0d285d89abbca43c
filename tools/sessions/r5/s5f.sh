#!/usr/bin/env bash
# round 5: MFMA k-step microbenchmark, then rows32 after pinning the fragment wait
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 60 tools/r5/mfma_probe/probe 200 > gpurun_out/mfma_probe.log 2>&1 || { echo "probe rc=$?"; cat gpurun_out/mfma_probe.log; exit 1; }
cat gpurun_out/mfma_probe.log
