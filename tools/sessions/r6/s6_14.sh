#!/usr/bin/env bash
# round 6: parameter-kernel workgroup timelines, current product code vs the
# same without the forward split-copy stores (NERFHIP_EXP_NO_FWDCOPY, timing
# only): does the epilogue's store count set its length?
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
o=gpurun_out/r6_14; mkdir -p $o
for v in pstamps nofwd_st; do
  NERFHIP_LIB=build/variants/v_$v.so timeout -k 10 240 python3 -u tools/r6/pstamps_deep.py 6 $o/$v.json > $o/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $o/$v.log; exit 1; }
  echo "== $v"; python3 -c "import json; d=json.load(open('$o/$v.json')); print({k: d[k] for k in ('launch_us','last_heavy_start_us','heavy_dur_us','phases_mean_us')})"
done
