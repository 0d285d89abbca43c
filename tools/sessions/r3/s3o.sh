#!/usr/bin/env bash
# K-split weight layout (xoff_ks): bitwise A/B vs the previous layout, GPU suite, configs 2 and 5, kernel stats
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3o${SUFFIX:-}; mkdir -p $out
NERFHIP_LIB=build/variants/v_oldks.so timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_old.npz > $out/ab_old.log 2>&1 || { tail $out/ab_old.log; exit 1; }
timeout -k 10 200 python -u tools/bitwise_ab.py /tmp/ab_new.npz > $out/ab_new.log 2>&1 || { tail $out/ab_new.log; exit 1; }
python -u tools/bitwise_ab.py --cmp /tmp/ab_new.npz /tmp/ab_old.npz | tee $out/ab_cmp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gputests.log 2>&1 || { tail -40 $out/gputests.log; exit 1; }
tail -2 $out/gputests.log
for i in 1 2; do timeout -k 10 120 python -u tools/configs_bench.py single wide 2>/dev/null | grep ms_per; done | tee $out/configs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p -o run --output-format csv -- python3 $R/tools/configs_bench.py single > $out/p.log 2>&1 || { tail -3 $out/p.log; exit 1; }
rm -f $out/p/*trace.csv
python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p/run_kernel_stats.csv')))
print(' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:26], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:3]))
" | tee -a $out/configs.log
