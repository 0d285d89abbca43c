#!/usr/bin/env bash
# native init replay: driver GPU tests, then the e2e leg (streaming on / off)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/e2e_rng.log; : > $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_drivers.py > gpurun_out/gpu_drivers_rng.log 2>&1 || { tail -30 gpurun_out/gpu_drivers_rng.log; exit 1; }
tail -2 gpurun_out/gpu_drivers_rng.log >> $out
timeout -k 10 200 python3 tools/r4/e2e_probe.py 3 2>&1 | grep fits >> $out || exit 1
NERFHIP_STREAM=0 timeout -k 10 200 python3 tools/r4/e2e_probe.py 2 2>&1 | grep fits >> $out || exit 1
cat $out
