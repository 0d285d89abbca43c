#!/usr/bin/env bash
# round 6, last call: GPU suite and smoke on the final tree (library d9da449d)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_36; mkdir -p $o
sha256sum nerf-attention_amd/nerf_attention/_lib/libnerfhip.so | cut -c1-16
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gputests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" $o/gputests.log | head -20; tail -30 $o/gputests.log; exit 1; }
tail -1 $o/gputests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
