#!/usr/bin/env bash
# round 6: W = 256 part built with the max-ilp / max-memory-clause machine
# schedulers vs the product, isolated leg, row and parameter kernels
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_31; mkdir -p $o
N=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
for rep in 1 2; do
  for lib in $N build/variants/v_s_ilp.so build/variants/v_s_mcl.so; do
    for k in rows params; do
      NERFHIP_LIB=$lib timeout -k 10 200 python3 -u tools/r4/isokernel.py --kernel $k > $o/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $o/iso.log; exit 1; }
      echo "$lib $k $(grep '^{' $o/iso.log | cut -c1-60)"
    done
  done
done
