#!/usr/bin/env bash
# round 5: fused split-K Adam probe (bf16x3 mismatch)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/r5/split_fused_probe.py > gpurun_out/split_fused_probe.log 2>&1 || { echo "probe rc=$?"; tail -30 gpurun_out/split_fused_probe.log; exit 1; }
grep '^{' gpurun_out/split_fused_probe.log
