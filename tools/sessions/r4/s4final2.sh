#!/usr/bin/env bash
# final tree: GPU suite + smoke
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gputests_r4_final2.log 2>&1 || { tail -40 gpurun_out/gputests_r4_final2.log; exit 1; }
tail -2 gpurun_out/gputests_r4_final2.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
