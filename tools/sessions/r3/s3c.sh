#!/usr/bin/env bash
# config 2 parameter step: kernel times vs split-K slice count, and SQ counters of the 16-slice kernel
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3c; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for sp in 1 2 4 8 16; do
  NERFHIP_GRAD_SPLIT_MAX=$sp timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p$sp -o run --output-format csv -- python3 $R/tools/configs_bench.py single > $out/p$sp.log 2>&1 || { tail $out/p$sp.log; exit 1; }
  python3 -c "
import csv
rs=list(csv.DictReader(open('$out/p$sp/run_kernel_stats.csv')))
print('split $sp', ' | '.join('%s %s %.1fus' % (r['Name'].split('::')[1][:22], r['Calls'], float(r['AverageNs'])/1e3) for r in rs[:3]))
" | tee -a $out/summary.log
  grep ms_per_epoch $out/p$sp.log | tail -1 | tee -a $out/summary.log
  rm -rf $out/p$sp/*trace* 
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD -d $out/pmc1 -o run --output-format csv -- python3 $R/tools/configs_bench.py single --epochs 200 > $out/pmc1.log 2>&1 || { tail -3 $out/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU -d $out/pmc2 -o run --output-format csv -- python3 $R/tools/configs_bench.py single --epochs 200 > $out/pmc2.log 2>&1 || { tail -3 $out/pmc2.log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("::")[-1][:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    if "step" in k or "adam" in k:
        print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
