#!/usr/bin/env bash
# round 6: BASELINE configs 2 and 5 (lone split-K fits: K-split rows, split-K
# parameter step, the rewritten k_adam_split) on the round-6 start library and
# the current one, interleaved on one box
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_18; mkdir -p $o
for lib in build/variants/v_base.so nerf-attention_amd/nerf_attention/_lib/libnerfhip.so build/variants/v_base.so nerf-attention_amd/nerf_attention/_lib/libnerfhip.so; do
  NERFHIP_LIB=$lib timeout -k 10 300 python3 -u tools/configs_bench.py single wide > $o/cfg.log 2>&1 || { echo "cfg rc=$?"; tail -5 $o/cfg.log; exit 1; }
  echo "== $lib"; grep '^{' $o/cfg.log | cut -c1-260
done
