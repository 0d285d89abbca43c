#!/usr/bin/env bash
# FitJob launch A/B: one interleaving thread vs one launcher thread per group (2000-epoch sweep)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/launch_threads_ab.log; : > $out
for r in 1 2; do
  for th in 0 1; do
    NERFHIP_LAUNCH_THREADS=$th timeout -k 10 150 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 2 --tag "threads$th-r$r" 2>&1 | grep tag >> $out || exit 1
  done
done
cat $out
