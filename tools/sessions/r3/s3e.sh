#!/usr/bin/env bash
# K-split row kernel (config 2): cache / memory counters
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3e; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/pmc$i -o run --output-format csv -- python3 $R/tools/configs_bench.py single --epochs 100 > $out/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/pmc$i.log; }
done
python3 - $out <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:48]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    if "step" in k or "adam" in k:
        print(k)
        print('   ', {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
