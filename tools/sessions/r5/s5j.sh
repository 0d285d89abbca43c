#!/usr/bin/env bash
# round 5: K-split LDS happens-before trace check (runtime-mode and compile-time-mode builds),
# vectorised fused split-K reducer — bitwise tests, config 2/5 A/B (two rounds)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
for v in kstrace kstrace_modes; do
  NERFHIP_LIB=build/variants/v_$v.so timeout -k 10 200 python3 -u tools/r5/ks_lds_hb.py > gpurun_out/ks_lds_hb_$v.log 2>&1 || { echo "hb $v rc=$?"; tail -20 gpurun_out/ks_lds_hb_$v.log; exit 1; }
  echo "== $v"; grep '^{' gpurun_out/ks_lds_hb_$v.log | cut -c1-900
done
bash tools/sessions/r5/s5i.sh
