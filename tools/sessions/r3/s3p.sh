#!/usr/bin/env bash
# config 5 (wide @8192): per-kernel stats, new lib vs the previous one
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3p${SUFFIX:-}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export NERFHIP_LIB=$R/build/variants/v_oldks.so; else unset NERFHIP_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p$v -o run --output-format csv -- python3 $R/tools/configs_bench.py wide --epochs 200 > $out/p$v.log 2>&1 || { tail -3 $out/p$v.log; exit 1; }
  rm -f $out/p$v/*trace.csv
  python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p$v/run_kernel_stats.csv')))
print('$v', ' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:30], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:5]))
" | tee -a $out/summary.log
done
