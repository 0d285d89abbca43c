#!/usr/bin/env bash
# K-split threshold 128: GPU suite, configs 2 and 5, config 5 kernel stats
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3s; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gputests.log 2>&1 || { tail -40 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
for i in 1 2; do timeout -k 10 120 python -u tools/configs_bench.py single wide 2>/dev/null | grep ms_per; done | tee $out/configs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p -o run --output-format csv -- python3 $R/tools/configs_bench.py wide > $out/p.log 2>&1 || { tail -3 $out/p.log; exit 1; }
rm -f $out/p/*trace.csv
python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p/run_kernel_stats.csv')))
print(' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:30], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:4]))
" | tee -a $out/configs.log
