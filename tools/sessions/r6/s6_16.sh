#!/usr/bin/env bash
# round 6: GPU suite, smoke and the default bench on the library with the
# streamed parameter-kernel epilogue and pinned block loads
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_16; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gputests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" $o/gputests.log | head -20; tail -30 $o/gputests.log; exit 1; }
tail -1 $o/gputests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 900 python3 -u bench.py > $o/bench.log 2> $o/bench.err || { echo "bench rc=$?"; tail -20 $o/bench.err; exit 1; }
grep '^{' $o/bench.log | cut -c1-300
grep "children at exit" $o/bench.err
