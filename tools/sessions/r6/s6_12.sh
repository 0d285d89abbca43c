#!/usr/bin/env bash
# round 6: (1) fp32 parameter kernel with the streamed epilogue and pinned
# block loads: bitwise A/B against the round-6 start library and the isolated
# leg; (2) NERFHIP_EXP_HOTBLOCK timing build (every block re-reads blocks 0/1,
# L2-hot; wrong numerics): how much of the bf16x3 loop is operand-load latency
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_12; mkdir -p $o
NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz fp32 > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz fp32 > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -5 $o/ab_new.log; exit 1; }
python3 tools/bitwise_ab.py --cmp $o/base.npz $o/new.npz | tee $o/ab_cmp.log; rm -f $o/base.npz $o/new.npz
for lib in build/variants/v_base.so nerf-attention_amd/nerf_attention/_lib/libnerfhip.so; do
  NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params --precision fp32 > $o/iso_fp32.log 2>&1 || { echo "iso fp32 rc=$?"; tail -5 $o/iso_fp32.log; exit 1; }
  echo "fp32 $lib"; grep '^{' $o/iso_fp32.log | cut -c1-120
done
for lib in nerf-attention_amd/nerf_attention/_lib/libnerfhip.so build/variants/v_hot.so nerf-attention_amd/nerf_attention/_lib/libnerfhip.so build/variants/v_hot.so; do
  NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
  echo "bf16x3 $lib"; grep '^{' $o/iso.log | cut -c1-120
done
