#!/usr/bin/env bash
# heaviest group on a high-priority stream vs default (2000-epoch sweep, 8 queues)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/prio_heavy_ab.log; : > $out
for r in 1 2; do
  for p in 0 1; do
    NERFHIP_PRIO_HEAVY=$p timeout -k 10 150 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 2 --tag "prio$p-r$r" 2>&1 | grep tag >> $out || exit 1
  done
done
cat $out
