#!/usr/bin/env bash
# round 6: parameter kernel with raised wave priority over the MFMA section
# (NERFHIP_EXP_PARAMS_PRIO = 1, 2) vs the product, isolated leg
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_32; mkdir -p $o
N=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
for rep in 1 2; do
  for lib in $N build/variants/v_prio1.so build/variants/v_prio2.so; do
    NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel params > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
    echo "$lib $(grep '^{' $o/iso.log | cut -c1-60)"
  done
done
