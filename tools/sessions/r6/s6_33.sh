#!/usr/bin/env bash
# round 6: parameter-kernel block loop, barrier-side wait per wave (stamps
# build, slot 7), then one more default bench of the product library
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_33; mkdir -p $o
NERFHIP_LIB=build/variants/v_pstamps.so timeout -k 10 200 python3 -u tools/r6/pstamps_deep.py 6 $o/pstamps_loop.json > $o/pstamps.log 2>&1 || { echo "pstamps rc=$?"; tail -5 $o/pstamps.log; exit 1; }
rm -f $o/pstamps_loop.npz
grep -A 12 block_loop $o/pstamps_loop.json
timeout -k 10 900 python3 -u bench.py > $o/bench.log 2> $o/bench.err || { echo "bench rc=$?"; tail -5 $o/bench.err; exit 1; }
cut -c1-200 $o/bench.log; tail -2 $o/bench.err
