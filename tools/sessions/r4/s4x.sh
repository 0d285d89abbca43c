#!/usr/bin/env bash
# hardware queues 4 (the box default) vs 8, serial and threaded launch (2000-epoch sweep)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/queues_ab.log; : > $out
for r in 1 2; do
  for q in 4 8; do
    for th in 0 1; do
      GPU_MAX_HW_QUEUES=$q NERFHIP_LAUNCH_THREADS=$th timeout -k 10 150 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 2 --tag "q$q-threads$th-r$r" 2>&1 | grep tag >> $out || exit 1
    done
  done
done
cat $out
