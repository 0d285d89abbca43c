#!/usr/bin/env bash
# round 6: W = 64 row kernel at four waves per SIMD (launch bound 4: 128
# VGPRs, no spills) — bitwise A/B, isolated tiny x 40 group, and the sweep
# (no CPU / fp32 / e2e legs), interleaved with the product library
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_22; mkdir -p $o
P=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so; V=build/variants/v_wps4.so
timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/a.npz > $o/ab_a.log 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_a.log; exit 1; }
NERFHIP_LIB=$V timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/b.npz > $o/ab_b.log 2>&1 || { echo "ab rc=$?"; tail -5 $o/ab_b.log; exit 1; }
python3 tools/bitwise_ab.py --cmp $o/a.npz $o/b.npz; rm -f $o/a.npz $o/b.npz
for lib in $P $V $P $V; do
  NERFHIP_LIB=$lib timeout -k 10 120 python3 -u tools/kbench.py --config tiny --fits 40 --epochs 101 --precision bf16x3 --repeat 1 > $o/kb.log 2>&1 || { echo "kbench rc=$?"; tail -5 $o/kb.log; exit 1; }
  echo "$lib $(grep '^{' $o/kb.log | cut -c1-160)"
done
for lib in $P $V $P $V; do
  NERFHIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-also-fp32 --no-e2e --no-kernel-timing > $o/b.log 2> $o/b.err || { echo "bench rc=$?"; tail -5 $o/b.err; exit 1; }
  echo "$lib $(grep '^{' $o/b.log | cut -c1-140)"
done
