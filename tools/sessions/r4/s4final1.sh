#!/usr/bin/env bash
# round-4 verification: full GPU suite, smoke, bench (headline legs) under rocprofv3 --kernel-trace --stats
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gputests_r4_final.log 2>&1 || { tail -40 gpurun_out/gputests_r4_final.log; exit 1; }
tail -2 gpurun_out/gputests_r4_final.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4.log 2>&1 || { tail -20 gpurun_out/smoke_r4.log; exit 1; }
tail -3 gpurun_out/smoke_r4.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench_r4" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-e2e --no-also-fp32 > gpurun_out/bench_under_rocprof_r4.log 2>&1 || { tail -20 gpurun_out/bench_under_rocprof_r4.log; exit 1; }
find gpurun_out/prof_bench_r4 -name '*kernel_stats.csv' -exec cp {} gpurun_out/rocprof_kernel_stats_bench_r4.csv \;
tail -1 gpurun_out/bench_under_rocprof_r4.log | cut -c1-300
