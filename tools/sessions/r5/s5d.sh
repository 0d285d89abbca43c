#!/usr/bin/env bash
# round 5: rows32 phase stamps (medium, deep)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
for c in medium deep; do
  NERFHIP_LIB=build/variants/v_r32stamps.so timeout -k 10 120 python3 -u tools/r5/stamps32.py --config $c > gpurun_out/stamps32_$c.log 2>&1 || { echo "stamps rc=$?"; tail -30 gpurun_out/stamps32_$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps32_$c.log
done
