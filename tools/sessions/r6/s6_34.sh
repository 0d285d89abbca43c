#!/usr/bin/env bash
# round 6: row kernel (deep x 40, bf16x3) phase cycles, clock held and MFMA
# pipe share from a stamps build without read-modify-write counters
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_34; mkdir -p $o
for ep in ${EPOCHS:-3 2000}; do
  NERFHIP_LIB=build/variants/v_stamps.so timeout -k 10 200 python3 -u tools/stamps.py --config deep --fits 40 --precision bf16x3 --epochs $ep > $o/stamps_e$ep.json 2> $o/stamps_e$ep.err || { echo "stamps rc=$?"; tail -5 $o/stamps_e$ep.err; exit 1; }
  echo "epochs $ep"; cat $o/stamps_e$ep.json
done
