#!/usr/bin/env bash
# round-5 first GPU call: bitwise check of the XCD-balanced chunk plans, then
# 400-epoch sweep A/B of the chunk policies (two interleaved rounds)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_drivers.py -k "xcd_order_bitwise" > gpurun_out/s5a_tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/s5a_tests.log; exit 1; }
tail -3 gpurun_out/s5a_tests.log
: > gpurun_out/chunks_ab.log
for rnd in 1 2; do
  for cfg in "spec 40" "depth 40" "mixed 40" "mixed 32" "depth 32"; do
    set -- $cfg
    NERFHIP_CHUNKS=$1 NERFHIP_GROUP_MAX=$2 timeout -k 10 120 python3 tools/r4/sweep_sched.py \
      --epochs 400 --steps 2 --tag "r$rnd" >> gpurun_out/chunks_ab.log 2>&1 \
      || { echo "sched rc=$?"; tail -20 gpurun_out/chunks_ab.log; exit 1; }
  done
done
cat gpurun_out/chunks_ab.log | cut -c1-400
