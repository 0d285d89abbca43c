#!/usr/bin/env bash
# threaded streaming launch: driver GPU tests, e2e timeline, e2e reps
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_drivers.py > gpurun_out/gpu_drivers_thr.log 2>&1 || { tail -30 gpurun_out/gpu_drivers_thr.log; exit 1; }
tail -2 gpurun_out/gpu_drivers_thr.log
timeout -k 10 200 python3 tools/r4/e2e_timeline.py > gpurun_out/e2e_timeline_thr.log 2>&1 || { tail -30 gpurun_out/e2e_timeline_thr.log; exit 1; }
head -24 gpurun_out/e2e_timeline_thr.log
timeout -k 10 200 python3 tools/r4/e2e_probe.py 3 2>&1 | grep fits > gpurun_out/e2e_thr.log || exit 1
cat gpurun_out/e2e_thr.log
