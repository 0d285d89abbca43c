#!/usr/bin/env bash
# PMC passes (one rocprofv3 run each) over isolated kbench groups, for the
# dominant step kernels: MFMA busy, VALU/LDS activity, waits, L2.
# usage: tools/pmc_groups.sh <out_tag>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag="$1"
export TMPDIR=/tmp
out="$R/gpurun_out/pmc_$tag"
mkdir -p "$out"
(cd /tmp && timeout -s KILL 60 rocprofv3 -L) > "$out/counters_list.txt" 2>&1 || true
i=0
for cfg in "medium 40" "large 40"; do
  set -- $cfg
  for cs in \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
    "SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
    "TCC_HIT_sum TCC_MISS_sum" ; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $cs -d "$out/p$i" -o run --output-format csv -- python3 "$R/tools/kbench.py" --config "$1" --fits "$2" --epochs 10 --repeat 1 --precision bf16x3) > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
  done
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections, re, json
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)<([^>]*)>", r["Kernel_Name"])
        if not m or not m.group(1).startswith("k_step"): continue
        acc[(m.group(1) + "<" + m.group(2) + ">", r["Counter_Name"])].append(float(r["Counter_Value"]))
res = collections.defaultdict(dict)
for (k, c), v in sorted(acc.items()):
    res[k][c] = sum(v) / len(v)
    print(f"{k:40s} {c:28s} {sum(v)/len(v):16.1f}  n={len(v)}")
json.dump(res, open(sys.argv[1] + "/pmc_groups.json", "w"), indent=1)
PY
