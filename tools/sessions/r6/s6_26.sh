#!/usr/bin/env bash
# round 6: parameter kernel with the operand split kept after the block's
# MFMAs (NERFHIP_EXP_SPLIT_AFTER_MFMA: a longer distance between the block
# loads and their use, no VALU/MFMA interleave) vs the product, isolated leg
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_26; mkdir -p $o
N=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so; V=build/variants/v_sam.so
for lib in $N $V $N $V; do
  NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
  echo "$lib $(grep '^{' $o/iso.log | cut -c1-100)"
done
