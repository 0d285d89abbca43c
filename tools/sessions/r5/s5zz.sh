#!/usr/bin/env bash
# round 5: bench smoke on the final bench.py (headline leg + roofline only)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-e2e --no-also-fp32 > gpurun_out/bench_final_check.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_final_check.log; exit 1; }
tail -1 gpurun_out/bench_final_check.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['frac'], r['traffic'], r['traffic_over_algorithmic'], r['hbm_gbs'])"
