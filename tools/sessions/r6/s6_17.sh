#!/usr/bin/env bash
# round 6: parameter kernel with three rotating LDS buffers (next block's
# fragments read before the barrier) and the swizzled 32-B feature layout:
# bitwise A/B against the round-6 start library, isolated deep W = 256 leg
# interleaved with the previous commit's library on the same box
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_17; mkdir -p $o
NERFHIP_LIB=build/variants/v_base.so timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/base.npz > $o/ab_base.log 2>&1 || { echo "base ab rc=$?"; tail -5 $o/ab_base.log; exit 1; }
timeout -k 10 300 python3 -u tools/bitwise_ab.py $o/new.npz > $o/ab_new.log 2>&1 || { echo "new ab rc=$?"; tail -5 $o/ab_new.log; exit 1; }
python3 tools/bitwise_ab.py --cmp $o/base.npz $o/new.npz | tee $o/ab_cmp.log; rm -f $o/base.npz $o/new.npz
for lib in build/variants/v_prev.so nerf-attention_amd/nerf_attention/_lib/libnerfhip.so build/variants/v_prev.so nerf-attention_amd/nerf_attention/_lib/libnerfhip.so; do
  NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
  echo "$lib"; grep '^{' $o/iso.log | cut -c1-100
done
