#!/usr/bin/env bash
# K-split rows: are the strided weight-item loads (16 rows x 64 B per instruction) the per-item cost?
# diagnostic build with lane-linear 1 KB loads (wrong results, timing only) vs the real kernel
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3n; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in kslin base; do
  if [ $v = kslin ]; then export NERFHIP_LIB=$R/build/variants/v_kslin.so; else unset NERFHIP_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p$v -o run --output-format csv -- python3 $R/tools/configs_bench.py single --epochs 500 > $out/p$v.log 2>&1 || { tail -3 $out/p$v.log; exit 1; }
  rm -f $out/p$v/*trace.csv
  python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p$v/run_kernel_stats.csv')))
print('$v', ' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:26], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:3]))
" | tee -a $out/summary.log
done
