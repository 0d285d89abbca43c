#!/usr/bin/env bash
# timing proxy of a two-plane / three-product split (NERFHIP_EXP_X2PROXY, wrong numerics) vs base
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/x2move_ab.log; : > $out
for c in medium large; do
  bash tools/ab.sh "--config $c --fits 40 --epochs 200 --precision bf16x3" build/variants/v_base.so build/variants/v_x2proxy.so build/variants/v_x2move.so >> $out 2>&1 || { tail -20 $out; exit 1; }
done
grep -v "^W2026" $out
