#!/usr/bin/env bash
# round 6: k_adam_split without EXEC-masked stores (straight-line, buffer stores
# masked by offset, drained before the wave ends) — everything else as in the
# faulting runs s6_02 / s6_04 / s6_05.  The 8-rank share standalone with the
# fault handler; only if it is clean, the GPU suite.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/r6/fault_probe.py share8 2000 gpurun_out/fault_probe_fix1.json > gpurun_out/fault_probe_fix1.log 2>&1
rc=$?
echo "probe rc=$rc"
grep -v amdgpu.ids gpurun_out/fault_probe_fix1.log | head -12
[ $rc -eq 0 ] || exit 0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_gputests_6.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" gpurun_out/r6_gputests_6.log | head -20; tail -30 gpurun_out/r6_gputests_6.log; exit 1; }
tail -3 gpurun_out/r6_gputests_6.log
