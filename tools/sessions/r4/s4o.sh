#!/usr/bin/env bash
# Full GPU suite of the current tree + param-kernel scaling probe (medium fits
# 8..120 in one group: per-fit parameter-step time vs group size)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_r4a.log 2>&1; rc=$?
tail -15 gpurun_out/gputests_r4a.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit 1; }
out=gpurun_out/params_scaling.log; : > $out
for n in 8 16 24 40 64 80 120; do
  NERFHIP_GROUP_MAX=0 timeout -k 10 120 python3 tools/kbench.py --config medium --fits $n --epochs 41 --precision bf16x3 --repeat 1 2>&1 | grep rep >> $out || { echo "kbench rc=$?"; exit 1; }
done
cat $out
