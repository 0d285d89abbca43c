#!/usr/bin/env bash
# round 6: GPU suite on the library with the bounded in-flight depth
# (K = 16 epochs, nerfhip.hip inflight_epochs), split-K for concurrent groups,
# then a short default bench and the processes left after it
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_gputests_4.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" gpurun_out/r6_gputests_4.log | head -20; tail -30 gpurun_out/r6_gputests_4.log; exit 1; }
tail -3 gpurun_out/r6_gputests_4.log
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 > gpurun_out/r6_bench_4.log 2> gpurun_out/r6_bench_4.err || { echo "bench rc=$?"; tail -20 gpurun_out/r6_bench_4.err; exit 1; }
grep '^{' gpurun_out/r6_bench_4.log | cut -c1-300
grep "children at exit" gpurun_out/r6_bench_4.err
sleep 3
ps -eo pid,ppid,user,etimes,stat,cmd > gpurun_out/r6_ps_after_bench.txt
awk -v u="$(id -un)" '$3==u' gpurun_out/r6_ps_after_bench.txt | grep -v "ps -eo\|awk\|sleep" | head -20
