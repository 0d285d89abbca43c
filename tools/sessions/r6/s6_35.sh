#!/usr/bin/env bash
# round 6: parameter-kernel block loop (stamps build) after 2000 epochs of
# back-to-back launches, the clock held warm (s6_33 ran 6 epochs)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_35; mkdir -p $o
NERFHIP_LIB=build/variants/v_stamps.so timeout -k 10 200 python3 -u tools/r6/pstamps_deep.py 2000 $o/pstamps_loop_e2000.json > $o/pstamps.log 2>&1 || { echo "pstamps rc=$?"; tail -5 $o/pstamps.log; exit 1; }
rm -f $o/pstamps_loop_e2000.npz
grep -A 12 block_loop $o/pstamps_loop_e2000.json; grep -A 5 phases_mean $o/pstamps_loop_e2000.json
