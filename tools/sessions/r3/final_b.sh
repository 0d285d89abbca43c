#!/usr/bin/env bash
# round 3: the exact default bench command under rocprofv3 --kernel-trace --stats + the round PMC profile
set -u
R="$GRAFT_REPO_ROOT"; tag="${1:-r03}"
bash $R/tools/prof_default.sh $tag || exit 1
find $R/gpurun_out -name '*kernel_trace.csv' -delete
find $R/gpurun_out -name '*counter_collection.csv' -size +20M -delete
du -sh $R/gpurun_out
