#!/usr/bin/env bash
# round 6: parameter kernel with the quad-transposed Adam epilogue (16-B P/M/V
# buffer accesses, 8-B forward split-copy runs): bitwise A/B against the
# round-6 start library (bf16x3), the isolated deep W = 256 leg, the timeline
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_15; mkdir -p $o
NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -5 $o/ab_new.log; exit 1; }
python3 tools/bitwise_ab.py --cmp $o/base.npz $o/new.npz | tee $o/ab_cmp.log; rm -f $o/base.npz $o/new.npz
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
  grep '^{' $o/iso.log | cut -c1-120
done
NERFHIP_LIB=build/variants/v_pstamps.so timeout -k 10 240 python3 -u tools/r6/pstamps_deep.py 6 $o/pstamps.json > $o/pstamps.log 2>&1 || { echo "pstamps rc=$?"; tail -5 $o/pstamps.log; exit 1; }
python3 -c "import json; d=json.load(open('$o/pstamps.json')); print({k: d[k] for k in ('launch_us','last_heavy_start_us','heavy_dur_us','phases_mean_us')})"
