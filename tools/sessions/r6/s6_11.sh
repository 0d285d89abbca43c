#!/usr/bin/env bash
# round 6: parameter kernel with the block loads pinned at the top of each block
# (bitwise A/B against the round-6 start library, the isolated deep W = 256
# leg on both, the workgroup timeline)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_11; mkdir -p $o
NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -5 $o/ab_new.log; exit 1; }
python3 tools/bitwise_ab.py --cmp $o/base.npz $o/new.npz | tee $o/ab_cmp.log; rm -f $o/base.npz $o/new.npz
for rep in 1 2; do
  NERFHIP_LIB=build/variants/v_base.so timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso_base_$rep.log 2>&1 || { echo "iso base rc=$?"; tail -5 $o/iso_base_$rep.log; exit 1; }
  timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso_new_$rep.log 2>&1 || { echo "iso new rc=$?"; tail -5 $o/iso_new_$rep.log; exit 1; }
  grep '^{' $o/iso_base_$rep.log | cut -c1-200; grep '^{' $o/iso_new_$rep.log | cut -c1-200
done
NERFHIP_LIB=build/variants/v_pstamps.so timeout -k 10 240 python3 -u tools/r6/pstamps_deep.py 6 $o/pstamps_deep.json > $o/pstamps.log 2>&1 || { echo "pstamps rc=$?"; tail -5 $o/pstamps.log; exit 1; }
head -22 $o/pstamps_deep.json
