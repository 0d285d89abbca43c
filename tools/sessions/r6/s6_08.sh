#!/usr/bin/env bash
# round 6: isolated deep W = 256 chunk-epoch profile on the fixed product
# library — rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE / MFMA-busy passes;
# iso_summary now reports the row AND the parameter kernel
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
bash tools/r4/iso_prof.sh r6 256 rows > gpurun_out/iso_prof_r6.log 2>&1
rc=$?
echo "iso_prof rc=$rc"
tail -60 gpurun_out/iso_prof_r6.log
exit $rc
