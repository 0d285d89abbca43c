#!/usr/bin/env bash
# round 5 verification (1/2): full GPU suite and smoke on the current tree
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gputests_r5.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 gpurun_out/gputests_r5.log; exit 1; }
tail -2 gpurun_out/gputests_r5.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke_r5.log; exit 1; }
tail -3 gpurun_out/smoke_r5.log
