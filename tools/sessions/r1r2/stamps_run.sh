#!/usr/bin/env bash
# per-phase stamps of the row kernel for lone fits and full groups (bf16x3)
set -u
mkdir -p gpurun_out/stamps
for c in "medium 1" "medium 40" "large 1" "large 8" "large 40"; do
  set -- $c
  NERFHIP_LIB=build/variants/v_stamps.so timeout -k 5 120 python tools/stamps.py --config $1 --fits $2 --precision bf16x3 > gpurun_out/stamps/$1_$2.json 2>gpurun_out/stamps/$1_$2.err || { echo "fail $c"; tail -3 gpurun_out/stamps/$1_$2.err; exit 1; }
  echo "== $c"; cat gpurun_out/stamps/$1_$2.json | tr -d '\n' | tr -s ' '; echo
done
