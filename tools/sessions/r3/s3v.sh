#!/usr/bin/env bash
# cost of the K-split one-workgroup-per-CU padding on config 5 (512 K-split workgroups), then the final-tree suite/smoke/bench
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3v; mkdir -p $out
for round in 1 2; do
  for share in 0 1; do
    NERFHIP_KS_SHARE_CU=$share timeout -k 10 120 python -u tools/configs_bench.py wide 2>/dev/null | grep ms_per | sed "s/^/share_cu=$share /" | cut -c1-200 | tee -a $out/configs.log || exit 1
  done
done
bash $R/tools/r3/final_a.sh r3fb
