#!/usr/bin/env bash
# round 6: final library (even VALU/MFMA interleave in the parameter kernel)
# — bitwise A/B against the round-6 start library in both precisions, the
# isolated chunk-epoch profile (rows + params PMC on this hash), GPU suite,
# smoke, default bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_29; mkdir -p $o
for prec in bf16x3 fp32; do
  NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz $prec > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
  timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz $prec > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -5 $o/ab_new.log; exit 1; }
  python3 tools/bitwise_ab.py --cmp $o/base.npz $o/new.npz > $o/ab_cmp_$prec.log; rc=$?; rm -f $o/base.npz $o/new.npz
  echo "$prec: $(cat $o/ab_cmp_$prec.log)"; [ $rc -eq 0 ] || exit 1
done
bash tools/r4/iso_prof.sh r6d 256 rows > $o/iso_prof.log 2>&1 || { echo "iso_prof rc=$?"; tail -20 $o/iso_prof.log; exit 1; }
cp gpurun_out/iso_r6d/summary.json profiles/r06/pmc_isolated_256.json
cp gpurun_out/iso_r6d/kernel_stats.csv profiles/r06/rocprof_kernel_stats_isolated_256.csv
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
