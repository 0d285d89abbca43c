#!/usr/bin/env bash
# e2e fit_kv_cache: streaming on/off, W=512 chunks of 8 while streaming
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/e2e_probe.log; : > $out
NERFHIP_STREAM=0 timeout -k 10 200 python3 tools/r4/e2e_probe.py 2 2>&1 | grep fits >> $out || exit 1
timeout -k 10 200 python3 tools/r4/e2e_probe.py 2 2>&1 | grep fits >> $out || exit 1
NERFHIP_GROUP_MAX_512=8 timeout -k 10 200 python3 tools/r4/e2e_probe.py 2 2>&1 | grep fits >> $out || exit 1
NERFHIP_GROUP_MAX_512=8 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 tools/r4/sweep_sched.py --epochs 2000 --steps 1 --tag "cap512-8" 2>&1 | grep tag >> $out || exit 1
cat $out
