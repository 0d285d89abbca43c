#!/usr/bin/env bash
# K-split vs regular row kernel around the selection threshold.
set -u
out=gpurun_out/ksth; mkdir -p $out
for args in "--fits 1 --seq-len 1024" "--fits 1 --seq-len 4096" "--fits 2 --seq-len 2048" "--fits 3 --seq-len 2048"; do
  for ks in 0 1; do
    echo "## $args KS=$ks" >> $out/log
    NERFHIP_ROWS_KS=$ks timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --config medium $args --epochs 100 >> $out/log 2>&1 || exit 1
  done
done
grep -v "^W\|amdgpu.ids" $out/log | cut -c1-140
