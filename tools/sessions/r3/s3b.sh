#!/usr/bin/env bash
# round 3 session 3: split-K prefetch-all parameter path + unrolled k_adam_split
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3b; mkdir -p $out
timeout -k 10 200 python -u tools/bitwise_ab.py $out/ab_pf.npz > $out/ab_pf.log 2>&1 || { tail $out/ab_pf.log; exit 1; }
NERFHIP_NO_SPLIT_PF=1 timeout -k 10 200 python -u tools/bitwise_ab.py $out/ab_nopf.npz > $out/ab_nopf.log 2>&1 || { tail $out/ab_nopf.log; exit 1; }
python -u tools/bitwise_ab.py --cmp $out/ab_pf.npz $out/ab_nopf.npz | tee $out/ab_cmp.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "split or rank_share or config2 or steps or ks" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for i in 1 2; do timeout -k 10 120 python -u tools/configs_bench.py single 2>/dev/null | tail -1; done | tee $out/single.log
NERFHIP_NO_SPLIT_PF=1 timeout -k 10 120 python -u tools/configs_bench.py single 2>/dev/null | tail -1 | sed 's/^/nopf /' | tee -a $out/single.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof_single -o run --output-format csv -- python3 $R/tools/configs_bench.py single > $out/prof_single.log 2>&1 || { tail $out/prof_single.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$out/prof_single/run_kernel_stats.csv')))[:5]: print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
