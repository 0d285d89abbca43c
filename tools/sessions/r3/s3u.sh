#!/usr/bin/env bash
# K-split prefetch depth (A-fragment items in flight per wave) with the xoff_ks layout: configs 2 and 5
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3u; mkdir -p $out
for round in 1 2; do
  for v in base pd4 pd10 pd14; do
    if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$R/build/variants/v_$v.so; fi
    timeout -k 10 120 python -u tools/configs_bench.py single wide 2>/dev/null | grep ms_per | sed "s/^/$v /" | cut -c1-200 | tee -a $out/configs.log || exit 1
  done
done
