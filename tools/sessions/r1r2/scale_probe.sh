#!/usr/bin/env bash
# predicted strong scaling per partition (every rank's share alone on this GPU)
set -u
mkdir -p gpurun_out/scale
for p in lpt blocked; do
  timeout -k 10 300 python tools/rank_probe.py --epochs 200 --worlds 1,2,4,8 --all-ranks --partition $p > gpurun_out/scale/probe_$p.log 2>&1 || { echo "probe $p failed"; tail -5 gpurun_out/scale/probe_$p.log; exit 1; }
  grep world gpurun_out/scale/probe_$p.log
done
