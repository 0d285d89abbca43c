#!/usr/bin/env bash
# which part of the third plane's data movement costs: weight DMA, A-fragment reads, B split, parameter-kernel staging
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/x2parts_ab.log; : > $out
V="build/variants/v_base.so build/variants/v_x2dma.so build/variants/v_x2frag.so build/variants/v_x2split.so build/variants/v_x2par.so"
for c in medium large; do
  bash tools/ab.sh "--config $c --fits 40 --epochs 200 --precision bf16x3" $V >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "^W2026" $out
