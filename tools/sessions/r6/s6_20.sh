#!/usr/bin/env bash
# round 6: final library — isolated chunk-epoch profile (rows + params PMC,
# same hash the bench reports against), GPU suite, smoke, default bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_20; mkdir -p $o
bash tools/r4/iso_prof.sh r6c 256 rows > $o/iso_prof.log 2>&1 || { echo "iso_prof rc=$?"; tail -20 $o/iso_prof.log; exit 1; }
cp gpurun_out/iso_r6c/summary.json profiles/r06/pmc_isolated_256.json
cp gpurun_out/iso_r6c/kernel_stats.csv profiles/r06/rocprof_kernel_stats_isolated_256.csv
python3 -c "
import json; d=json.load(open('profiles/r06/pmc_isolated_256.json'))
for k,v in d.items(): print(k, {x: v[x] for x in ('bytes','mfma_busy','rocprof_avg_ms','hipevent_avg_ms','lib_sha16')})"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gputests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error" $o/gputests.log | head -20; tail -30 $o/gputests.log; exit 1; }
tail -1 $o/gputests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 900 python3 -u bench.py > $o/bench.log 2> $o/bench.err || { echo "bench rc=$?"; tail -20 $o/bench.err; exit 1; }
grep '^{' $o/bench.log | cut -c1-200
grep "children at exit" $o/bench.err
