#!/usr/bin/env bash
# split-K vs fused gradient reduction for the small groups of 8-rank shares.
set -u
out=gpurun_out/split_probe; mkdir -p $out
for sm in 8 5 2; do
  echo "NERFHIP_SPLIT_MAX_FITS=$sm" >> $out/log
  NERFHIP_SPLIT_MAX_FITS=$sm timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config large --fits 5 --epochs 100 >> $out/log 2>&1 || exit 1
  NERFHIP_SPLIT_MAX_FITS=$sm timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config small --fits 5 --epochs 100 >> $out/log 2>&1 || exit 1
  NERFHIP_SPLIT_MAX_FITS=$sm timeout -k 10 200 python -u tools/rank_probe.py --worlds 8 --all-ranks >> $out/log 2>&1 || exit 1
done
grep -v "^W\|amdgpu.ids" $out/log
