#!/usr/bin/env bash
# round 5: rows32 after the epilogue-operand and lazy-split changes; ring-depth
# and no-SLP variants (A/B on 40 medium / deep fits)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/r5/rows32_check.py > gpurun_out/rows32_check2.log 2>&1 || { echo "check rc=$?"; tail -30 gpurun_out/rows32_check2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rows32_check2.log
V=build/variants
timeout -k 10 300 bash tools/ab.sh "--config medium --fits 40 --epochs 41 --precision bf16x3" nerf-attention_amd/nerf_attention/_lib/libnerfhip.so $V/v_r32ring4.so $V/v_r32noslp.so > gpurun_out/ab_r32_variants.log 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/ab_r32_variants.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_r32_variants.log | cut -c1-300
