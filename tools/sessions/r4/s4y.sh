#!/usr/bin/env bash
# per-width kernel throughput, 40-fit groups in isolation (bf16x3, seq 2048, 200 epochs)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/width_kernels.log; : > $out
for c in tiny small medium large; do
  timeout -k 10 120 python3 tools/kbench.py --config $c --fits 40 --epochs 200 --precision bf16x3 --repeat 2 2>&1 | grep rows_ms >> $out || exit 1
done
cat $out
