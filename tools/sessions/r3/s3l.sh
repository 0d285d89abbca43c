#!/usr/bin/env bash
# split-K for the 40-fit W=64/128 groups (fused grid 120/160 workgroups): isolated and sweep
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3l; mkdir -p $out
for rep in 1 2; do
  for v in 1 0; do
    for cfg in small tiny; do
      NERFHIP_SPLIT_BIG=$v timeout -k 10 120 python -u tools/kbench.py --config $cfg --fits 40 --epochs 41 --repeat 2 --precision bf16x3 2>/dev/null | tail -1 | sed "s/^/big=$v /" | tee -a $out/kbench.log
    done
  done
done
for v in 1 0 1 0; do
  NERFHIP_SPLIT_BIG=$v timeout -k 10 300 python -u bench.py --epochs 200 --no-cpu-baseline --no-also-fp32 --no-e2e > $out/bench200_$v.log 2>&1 || { tail $out/bench200_$v.log; exit 1; }
  grep '^{"metric' $out/bench200_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('big=$v', d['value'], d['ms_per_step'])" | tee -a $out/bench200.log
done
