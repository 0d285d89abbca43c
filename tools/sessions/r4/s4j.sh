#!/usr/bin/env bash
# (1) VGPR-WAR padding test of the fixed-source MODE-1 K-split kernel;
# (2) sweep schedule experiments (chunk size, hardware queues), 400 epochs
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 bash tools/r4/s4i.sh > /dev/null 2>&1 || { echo "s4i failed"; exit 1; }
cat gpurun_out/ks_fix_r4b.log | cut -c1-170
out=gpurun_out/sweep_sched.log; : > $out
for gm in 40 20 80; do for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q NERFHIP_GROUP_MAX=$gm timeout -k 10 120 python3 tools/r4/sweep_sched.py --epochs 400 --tag "gm$gm-q$q" 2>&1 | grep tag >> $out || { echo "sched rc=$?"; exit 1; }
done; done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 1 --tag "default-2000" 2>&1 | grep tag >> $out || exit 1
cat $out
