#!/usr/bin/env bash
# round 5: rows32 interleave depth (VALU per MFMA in the k-step schedule): 6 (shipped) vs 3 vs 12
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
V=build/variants
NERFHIP_ROWS32=1 timeout -k 10 400 bash tools/ab.sh "--config medium --fits 40 --epochs 41 --precision bf16x3" nerf-attention_amd/nerf_attention/_lib/libnerfhip.so $V/v_r32vpg3.so $V/v_r32vpg12.so > gpurun_out/ab_r32_vpg.log 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/ab_r32_vpg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r32_vpg.log | cut -c1-220
