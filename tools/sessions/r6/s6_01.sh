#!/usr/bin/env bash
# round 6: baseline on the round-5 tree — GPU suite, then the default bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_gputests_base.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r6_gputests_base.log; exit 1; }
tail -2 gpurun_out/r6_gputests_base.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r6_bench_base.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r6_bench_base.log; exit 1; }
grep '^{' gpurun_out/r6_bench_base.log | cut -c1-400
