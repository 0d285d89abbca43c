#!/usr/bin/env bash
# round-4 first GPU call: sin/cos probe, isolated profile of the dominant
# kernel, hardware-sincos A/B, a short bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 60 tools/r4/sin_probe2/sin_probe2 400 > gpurun_out/sin_probe2.log 2>&1 || { echo "probe rc=$?"; cat gpurun_out/sin_probe2.log; exit 1; }
cat gpurun_out/sin_probe2.log
V=build/variants
timeout -k 10 400 bash tools/r4/ab_iso.sh "--width 256 --epochs 41" $V/v_base.so $V/v_sc1.so $V/v_sc2.so > gpurun_out/ab_sincos_256.log 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/ab_sincos_256.log; exit 1; }
grep -v "^\[" gpurun_out/ab_sincos_256.log | cut -c1-220
timeout -k 10 400 bash tools/r4/ab_iso.sh "--width 512 --epochs 41" $V/v_base.so $V/v_sc1.so > gpurun_out/ab_sincos_512.log 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/ab_sincos_512.log; exit 1; }
grep -v "^\[" gpurun_out/ab_sincos_512.log | cut -c1-220
timeout -k 10 600 bash tools/r4/iso_prof.sh r4base 256 rows > gpurun_out/iso_r4base.log 2>&1 || { echo "iso rc=$?"; tail -20 gpurun_out/iso_r4base.log; exit 1; }
tail -30 gpurun_out/iso_r4base.log
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-also-fp32 > gpurun_out/bench_s4a.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_s4a.log; exit 1; }
tail -c 2500 gpurun_out/bench_s4a.log
