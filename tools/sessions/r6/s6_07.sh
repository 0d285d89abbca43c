#!/usr/bin/env bash
# round 6: GPU suite on the fixed library (straight-line k_adam_split, no
# in-flight throttle), the default bench, and the processes left after it
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_gputests_7.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" gpurun_out/r6_gputests_7.log | head -20; tail -30 gpurun_out/r6_gputests_7.log; exit 1; }
tail -2 gpurun_out/r6_gputests_7.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke_7.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r6_smoke_7.log; exit 1; }
tail -1 gpurun_out/r6_smoke_7.log
timeout -k 10 900 python3 -u bench.py > gpurun_out/r6_bench_7.log 2> gpurun_out/r6_bench_7.err || { echo "bench rc=$?"; tail -20 gpurun_out/r6_bench_7.err; exit 1; }
grep '^{' gpurun_out/r6_bench_7.log | cut -c1-200
grep "children at exit" gpurun_out/r6_bench_7.err
sleep 3
ps -eo pid,ppid,user,etimes,stat,cmd > gpurun_out/r6_ps_after_bench_7.txt
awk -v u="$(id -un)" '$3==u' gpurun_out/r6_ps_after_bench_7.txt | grep -v "ps -eo\|awk\|sleep" | head -20
