#!/usr/bin/env bash
# chunk cap x hardware queues with the queue setting actually applied (2000-epoch sweep)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/caps_queues_ab.log; : > $out
for r in 1 2; do
  for cfg in "8 40" "16 40" "16 20" "16 27" "8 80"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 NERFHIP_GROUP_MAX=$2 timeout -k 10 150 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 2 --tag "q$1-cap$2-r$r" 2>&1 | grep tag >> $out || exit 1
  done
done
grep -o '"tag": "[^"]*"\|"s_per_sweep": [0-9.]*' $out | paste - -
