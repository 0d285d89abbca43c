#!/usr/bin/env bash
# round 6: row-kernel scratch stores transposed through a per-wave LDS tile
# instead of quad_transpose — bitwise A/B (bf16x3 and fp32) against the
# round-6 start library, then the isolated deep W = 256 row leg and the sweep
# (no CPU / fp32 / e2e legs), interleaved with the previous commit's library
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_24; mkdir -p $o
P=build/variants/v_prev.so; N=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
for prec in bf16x3 fp32; do
  NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz $prec > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
  timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz $prec > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -5 $o/ab_new.log; exit 1; }
  echo "$prec: $(python3 tools/bitwise_ab.py --cmp $o/base.npz $o/new.npz)"; rm -f $o/base.npz $o/new.npz
done
for lib in $P $N $P $N; do
  NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel rows > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
  echo "$lib $(grep '^{' $o/iso.log | cut -c1-110)"
done
for lib in $P $N $P $N; do
  NERFHIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-also-fp32 --no-e2e --no-kernel-timing > $o/b.log 2> $o/b.err || { echo "bench rc=$?"; tail -5 $o/b.err; exit 1; }
  echo "$lib $(grep '^{' $o/b.log | cut -c100-200)"
done
