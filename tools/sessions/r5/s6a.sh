#!/usr/bin/env bash
# round 5: W = 512 chunk cap A/B on the 400-epoch sweep (the critical-path width on more streams)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/cap512_ab.log; : > $out
for r in 1 2; do
  for c in 40 20 27; do
    NERFHIP_GROUP_MAX_512=$c timeout -k 10 200 python3 -u tools/r4/sweep_sched.py --epochs 400 --steps 2 --tag "r$r cap512=$c" >> $out 2>&1 || { echo "rc=$?"; tail -5 $out; exit 1; }
  done
done
grep '^{' $out | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d.get('s_per_sweep'), d.get('fits_per_s_2000ep_equiv'), [g[:2]+[g[3]] for g in d.get('groups',[])][:3])"
