#!/usr/bin/env bash
# diagnostic: k_adam_split with and without its split-copy (wsplit) stores, configs 2 and 5 (kernel stats)
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3w; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in base noxs; do
  if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$R/build/variants/v_noxs.so; fi
  for c in single wide; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p_${v}_$c -o run --output-format csv -- python3 $R/tools/configs_bench.py $c > $out/p_${v}_$c.log 2>&1 || { tail -3 $out/p_${v}_$c.log; exit 1; }
    rm -f $out/p_${v}_$c/*trace.csv
    python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p_${v}_$c/run_kernel_stats.csv')))
print('$v $c', ' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:28], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:3]))
" | tee -a $out/summary.log
  done
done
