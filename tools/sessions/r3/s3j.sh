#!/usr/bin/env bash
# split-K parameter step on 64x64 tiles for lone W>=256 fits (config 2, config 5) vs 128x128
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3j; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "split or config2 or steps or ks or shapes or wide or rank_share" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; }
tail -2 $out/tests.log
cd /tmp && export TMPDIR=/tmp
for v in "T128" "S16" "S8" "S4"; do
  case $v in
    T128) envs="NERFHIP_SPLIT_T128=1";;
    S16) envs="NERFHIP_GRAD_SPLIT_MAX=16";;
    S8) envs="NERFHIP_GRAD_SPLIT_MAX=8";;
    S4) envs="NERFHIP_GRAD_SPLIT_MAX=4";;
  esac
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p$v -o run --output-format csv -- python3 $R/tools/configs_bench.py single wide > $out/p$v.log 2>&1 || { echo "$v failed"; tail -3 $out/p$v.log; exit 1; }
  rm -f $out/p$v/*trace.csv
  python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p$v/run_kernel_stats.csv')))
print('$v', ' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:26], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:6]))
" | tee -a $out/summary.log
  grep ms_per_epoch $out/p$v.log | tee -a $out/summary.log
done
