#!/usr/bin/env bash
# instruction-cache counters of the row / parameter / K-split kernels
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3f; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/avail.txt 2>&1 || true
grep -ioE "SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_INSTS_[A-Z_]*|SQC_INST[A-Z_]*" $out/avail.txt | sort -u | tr '\n' ' ' > $out/icache_ctrs.txt; echo >> $out/icache_ctrs.txt
cat $out/icache_ctrs.txt
i=0
for ctr in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/ks$i -o run --output-format csv -- python3 $R/tools/configs_bench.py single --epochs 50 > $out/ks$i.log 2>&1 || { echo "ks pass $i failed"; tail -3 $out/ks$i.log; }
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/kb$i -o run --output-format csv -- python3 $R/tools/kbench.py --config medium --fits 40 --epochs 8 --repeat 1 --precision bf16x3 > $out/kb$i.log 2>&1 || { echo "kb pass $i failed"; tail -3 $out/kb$i.log; }
done
python3 - $out <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/k*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:52]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    if "step" in k or "adam" in k:
        print(k)
        print('   ', {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
