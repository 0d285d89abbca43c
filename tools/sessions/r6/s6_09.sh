#!/usr/bin/env bash
# round 6: workgroup timeline of the parameter kernel on the isolated deep
# W = 256 chunk (NERFHIP_STAMPS build, tools/r6/pstamps_deep.py): per-workgroup
# durations, heavy tiles running at once per XCD, the drain tail
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
NERFHIP_LIB=build/variants/v_pstamps.so timeout -k 10 240 python3 -u tools/r6/pstamps_deep.py 6 gpurun_out/pstamps_deep.json > gpurun_out/pstamps_deep.log 2>&1
rc=$?
echo "pstamps rc=$rc"
grep -v amdgpu.ids gpurun_out/pstamps_deep.log | tail -80
exit $rc
