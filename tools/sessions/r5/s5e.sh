#!/usr/bin/env bash
# round 5: rows32 with cross-phase prefetch + staged biases: check, timing, stamps
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/r5/rows32_check.py > gpurun_out/rows32_check3.log 2>&1 || { echo "check rc=$?"; tail -30 gpurun_out/rows32_check3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rows32_check3.log
for c in medium deep; do
  NERFHIP_LIB=build/variants/v_r32stamps.so timeout -k 10 120 python3 -u tools/r5/stamps32.py --config $c > gpurun_out/stamps32b_$c.log 2>&1 || { echo "stamps rc=$?"; tail -30 gpurun_out/stamps32b_$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps32b_$c.log | tr -d '\n' | cut -c1-1500; echo
done
