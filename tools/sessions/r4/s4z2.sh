#!/usr/bin/env bash
# default bench (the driver's N=1 invocation)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py > gpurun_out/bench_default_r04b.log 2> gpurun_out/bench_default_r04b.err || { tail -20 gpurun_out/bench_default_r04b.err; exit 1; }
tail -1 gpurun_out/bench_default_r04b.log
