#!/usr/bin/env bash
# round 5: a second default bench run on the final tree (run-to-run spread)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default_r05b.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default_r05b.log; exit 1; }
tail -1 gpurun_out/bench_default_r05b.log | cut -c1-300
