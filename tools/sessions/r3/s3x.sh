#!/usr/bin/env bash
# config 5: split-K slice cap 8 (default) vs 4, with the K-split rows (interleaved, 2 rounds)
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3x; mkdir -p $out
for round in 1 2; do
  for cap in 16 4; do
    NERFHIP_GRAD_SPLIT_MAX=$cap timeout -k 10 120 python -u tools/configs_bench.py single wide 2>/dev/null | grep ms_per | sed "s/^/cap=$cap /" | cut -c1-180 | tee -a $out/configs.log || exit 1
  done
done
