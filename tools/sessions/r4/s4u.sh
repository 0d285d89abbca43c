#!/usr/bin/env bash
# e2e timeline (cProfile + streaming driver marks)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python3 tools/r4/e2e_timeline.py > gpurun_out/e2e_timeline.log 2>&1 || { tail -30 gpurun_out/e2e_timeline.log; exit 1; }
head -60 gpurun_out/e2e_timeline.log
