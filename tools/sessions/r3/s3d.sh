#!/usr/bin/env bash
# 8-wave K-split row kernel: parity tests that run it, config 2 timing + kernel trace, K-split crossover probe
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3d; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "ks or config2 or q512 or shapes or steps or split or smoke or fit_siren" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for i in 1 2; do timeout -k 10 120 python -u tools/configs_bench.py single 2>/dev/null | tail -1; done | tee $out/single.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof_single -o run --output-format csv -- python3 $R/tools/configs_bench.py single > $out/prof_single.log 2>&1 || { tail $out/prof_single.log; exit 1; }
rm -f $out/prof_single/*trace*
python3 -c "
import csv
for r in list(csv.DictReader(open('$out/prof_single/run_kernel_stats.csv')))[:4]: print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
