#!/usr/bin/env bash
# round 5: the default bench line, and the same command under rocprofv3 --kernel-trace --stats
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default_r05.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default_r05.log; exit 1; }
tail -1 gpurun_out/bench_default_r05.log | cut -c1-600
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench_r05" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-e2e --no-also-fp32 > gpurun_out/bench_under_rocprof_r05.log 2>&1 || { echo "rocprof rc=$?"; tail -20 gpurun_out/bench_under_rocprof_r05.log; exit 1; }
find "$R/gpurun_out/prof_bench_r05" -name '*kernel_stats.csv' -exec cp {} "$R/gpurun_out/rocprof_kernel_stats_bench_r05.csv" \;
tail -1 gpurun_out/bench_under_rocprof_r05.log | cut -c1-300
